"""Phase breakdown of the BA's reduced-system LDLT (ba_ldlt_reg_kernel) from a YAVO_LM_PROFILE build.

    make -C ya_vo_amd/csrc prof && python tools/ldlt_profile.py [--n 120] [--calls 50]

Runs yv_ba_debug_ldlt on a configs[2]-window-shaped system (block tridiagonal, 6 x 6 pose blocks) and prints the
mean shader-clock cycles per call that each wave's lane 0 spent in each phase."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ya_vo_amd as yv  # noqa: E402

PHASES = ["preamble (stage S, ranks, registers)", "wait for column k", "step loads + diagonal chain",
          "owner: pair q + 1 finalised and published", "bulk update (+ wave 0 forward solve)", "final barrier", "solves (wave 0)", "-"]


def window_system(nb, seed):
    rng = np.random.default_rng(seed)
    n = 6 * nb
    J = np.zeros((3 * n, n))
    for p in range(nb):
        J[18 * p:18 * p + 18, 6 * p:6 * p + 6] = rng.normal(size=(18, 6))
        if p + 1 < nb:
            J[18 * p:18 * p + 18, 6 * p + 6:6 * p + 12] = 0.3 * rng.normal(size=(18, 6))
    H = J.T @ J + 1e-3 * np.eye(n)
    return np.tril(H) + np.tril(H, -1).T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=120)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--lib", default=os.path.join(ROOT, "ya_vo_amd", "lib", "libyavo_prof.so"),
                    help="a YAVO_LM_PROFILE build (experiment builds of the kernel too)")
    args = ap.parse_args()
    lib = yv.load_library(args.lib)
    lib.yv_debug_ldlt_prof.argtypes = [ctypes.c_void_p]
    ctx = yv.Context(0)
    S = window_system(args.n // 6, 1)
    b = np.random.default_rng(2).normal(size=args.n)
    ctx.ba_ldlt(S, b)
    prof = np.zeros((8, 8), np.uint64)
    lib.yv_debug_ldlt_prof(prof.ctypes.data)
    for _ in range(args.calls):
        ctx.ba_ldlt(S, b)
    assert lib.yv_debug_ldlt_prof(prof.ctypes.data) == 0
    per = prof.astype(np.float64) / args.calls
    out = {"n": args.n, "calls": args.calls, "cycles_per_call_per_wave": {
        PHASES[q]: [round(float(per[w, q])) for w in range(8)] for q in range(7)},
        "total_per_wave": [round(float(per[w].sum())) for w in range(8)]}
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
