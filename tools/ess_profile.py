"""Phase breakdown of the five-point solver (ess_models_kernel, EMEstimatorCallback::runKernel) from a YAVO_LM_PROFILE
build, on one list as the LoopHandler's findEssentialMat sees it (1935 correspondences, 20% gross mismatches).

    make -C ya_vo_amd/csrc prof && python tools/ess_profile.py [--loop-lists 2]

Prints the mean / max shader-clock cycles per RANSAC iteration of each phase over the round's iterations, the
Durand-Kerner sweep counts, and the host call's wall time."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402,F401

import ya_vo_amd as yv  # noqa: E402

PHASES = ["svd 9x5", "coeff matrix", "lu inverse + product", "det B(z)", "durand-kerner", "solveZ + models"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loop-lists", type=int, default=0,
                    help="profile this many LoopHandler re-initialisation lists (reinit_probe.py) instead")
    a = ap.parse_args()
    lib = yv.load_library(os.path.join(ROOT, "ya_vo_amd", "lib", "libyavo_prof.so"))
    lib.yv_debug_ess_prof.argtypes = [ctypes.c_void_p]
    from epipolar_scene import two_view_scene
    ctx = yv.Context(0)
    lists = {}
    if a.loop_lists:
        from reinit_probe import loop_handler_lists
        ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"),
                                          np.int8))
        for j, m in enumerate(loop_handler_lists(ctx, a.loop_lists)):
            prev = np.c_[m["pt1"]["x"], m["pt1"]["y"]].astype(np.float32)
            curr = np.c_[m["pt2"]["x"], m["pt2"]["y"]].astype(np.float32)
            lists[f"loop_list_{j}"] = (curr, prev)
    else:
        for seed in (500, 501, 502):
            p1, p2, _, _ = two_view_scene(1935, outlier_frac=0.2, seed=seed, angle=0.02)
            lists[f"two_view_{seed}"] = (p2, p1)
    out = {}
    for name, (b, a_) in lists.items():
        ctx.find_essential(b, a_)  # warm-up (workspace)
        t0 = time.perf_counter()
        ctx.find_essential(b, a_)
        wall = time.perf_counter() - t0
        prof = np.zeros((256, 8), np.uint64)
        assert lib.yv_debug_ess_prof(prof.ctypes.data) == 0
        used = prof[:, 7] > 0
        p = prof[used].astype(np.float64)
        out[name] = {"call_ms": round(1e3 * wall, 3), "iterations_profiled": int(used.sum()),
                     "phase_cycles_mean": {PHASES[i]: round(float(p[:, i].mean()), 0) for i in range(6)},
                     "phase_cycles_max": {PHASES[i]: round(float(p[:, i].max()), 0) for i in range(6)},
                     "dk_sweeps": {"mean": float(p[:, 7].mean()), "min": float(p[:, 7].min()),
                                   "max": float(p[:, 7].max()), "at_300": int(np.sum(p[:, 7] >= 300))}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
