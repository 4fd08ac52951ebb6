"""Bisect a GPU / oracle divergence in the sliding-window BA: per LM iteration, compare every workspace buffer the
first damping trial leaves (yv_ba_debug_read) with the oracle's copy of the same buffer (or_ba_dump)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ya_vo_amd as yv  # noqa: E402
from ya_vo_amd import scene  # noqa: E402
import oracle_bind  # noqa: E402

NAMES = ["err", "Jp", "Jl", "Hpl", "W", "Hpp", "bp", "Hll", "bl", "Dinv", "S", "bs", "xp", "xl", "poses", "X"]
NOT_STORED = {"Hpl", "W", "Dinv"}  # formed where they are read since round 5 (yv_ba_debug_read refuses them)


def main():
    P, L, obs, noise, nf, seed = 5, 200, 3, 1.0, 1, 0
    w = scene.ba_window(n_poses=P, n_landmarks=L, obs=obs, noise_px=noise, seed=seed)
    E = len(w["ep"])
    ns = 6 * (P - nf)
    sizes = [2 * E, 12 * E, 6 * E, 18 * E, 18 * E, 36 * P, 6 * P, 9 * L, 3 * L, 9 * L, ns * ns, ns, ns, 3 * L, 7 * P,
             3 * L]
    orc = oracle_bind.Oracle()
    lib = orc.lib
    ctx = yv.Context(0)
    ctx.lib.yv_ba_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]
    dump_iter = ctypes.c_int.in_dll(lib, "or_ba_dump_iter")
    dump_ptrs = (ctypes.c_void_p * 16).in_dll(lib, "or_ba_dump")
    for it in range(3):
        ba = yv.BundleAdjuster(ctx, P, L, E)
        ba.set_problem(P, nf, L, w["ep"], w["el"], w["meas"], scene.K_KITTI)
        T, X, log, nit = ba.solve(w["poses0"], w["X0"], it + 1)
        gbuf = []
        for k, n in enumerate(sizes):
            a = np.zeros(n)
            if NAMES[k] in NOT_STORED:
                a = None
            else:
                assert ctx.lib.yv_ba_debug_read(ba.handle, k, a.ctypes.data, n) == 0
            gbuf.append(a)
        obuf = [np.zeros(n) for n in sizes]
        for k in range(16):
            dump_ptrs[k] = obuf[k].ctypes.data
        dump_iter.value = it
        oT, oX, oit, olog = orc.ba_lm(w["poses0"], nf, w["X0"], w["ep"], w["el"], w["meas"], scene.K_KITTI, it + 1)
        dump_iter.value = -1
        print(f"iteration {it}: log gpu {log.tolist()} oracle {olog.tolist()}")
        for k, name in enumerate(NAMES):
            g, o = gbuf[k], obuf[k]
            if g is None:
                continue
            if name in ("Hpp", "bp"):  # fixed poses are not assembled on the GPU
                m = 36 if name == "Hpp" else 6
                g, o = g[nf * m:], o[nf * m:]
            bad = np.flatnonzero(g != o)
            rel = np.max(np.abs(g - o) / np.maximum(np.abs(o), 1e-300)) if len(bad) else 0.0
            first = bad[:4].tolist()
            print(f"  {name:6s} n={len(g):6d} mismatches={len(bad):6d} max_rel={rel:.3e} first={first}")
        ba.close()
    ctx.close()


if __name__ == "__main__":
    main()
