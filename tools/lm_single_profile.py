"""Latency of one pose-only LM call (yv_pose_lm, LoopHandler::optimizePoseOnly as the drop-in LoopHandler makes it)
and its phase breakdown from a YAVO_LM_PROFILE build.

    make -C ya_vo_amd/csrc prof && python tools/lm_single_profile.py [--edges 400 1000 1900]

For each problem size: the host call's wall time with the product library (median of --reps calls, the same
problem), then the per-phase shader-clock cycles of the one workgroup from lib/libyavo_prof.so (a second process
would be cleaner; both libraries are loaded here one after the other through separate contexts)."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

import ya_vo_amd as yv  # noqa: E402
from ya_vo_amd import scene  # noqa: E402

PHASES = ["edge compute (lane 0's share)", "tree reduce proper", "lane-0 exp/mul", "accept + barriers",
          "classify/compact", "iteration setup", "lane-0 T backup + LDLT", "lane-0 system copy (iteration)",
          "wait for other waves' edges"]


def problems(sizes):
    out = []
    for i, n in enumerate(sizes):
        X, uv, T, _ = scene.random_scene(n, seed=300 + i, noise_px=0.5, outlier_frac=0.1)
        out.append((X, uv, scene.perturb(T, np.random.default_rng(i))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--edges", type=int, nargs="+", default=[400, 1000, 1900])
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--prof", action="store_true", help="phase cycles from lib/libyavo_prof.so instead of wall times")
    a = ap.parse_args()
    probs = problems(a.edges)
    if a.prof:  # before anything loads the product library
        lib = yv.load_library(os.path.join(ROOT, "ya_vo_amd", "lib", "libyavo_prof.so"))
        lib.yv_debug_lm_prof.argtypes = [ctypes.c_void_p]
    res = {"sum_mode": yv.lm_sum_mode(1)}
    if not a.prof:
        ctx = yv.Context(0)
        for n, (X, uv, prior) in zip(a.edges, probs):
            ctx.pose_lm(X, uv, scene.K_KITTI, prior)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                ctx.pose_lm(X, uv, scene.K_KITTI, prior)
                ts.append(time.perf_counter() - t0)
            res[str(n)] = {"call_ms_median": round(1e3 * float(np.median(ts)), 4),
                           "call_ms_min": round(1e3 * float(np.min(ts)), 4)}
        ctx.close()
    else:
        ctx = yv.Context(0)
        for n, (X, uv, prior) in zip(a.edges, probs):
            ctx.pose_lm(X, uv, scene.K_KITTI, prior)
            prof = np.zeros((1024, 10), np.uint64)
            assert lib.yv_debug_lm_prof(prof.ctypes.data) == 0
            p = prof[0].astype(np.float64)
            tot = p[:9].sum()
            res[str(n)] = {"cycles_total": int(tot), "passes": int(p[9]),
                           "phases": {PHASES[i]: [int(p[i]), round(100 * p[i] / max(tot, 1), 1)] for i in range(9)}}
        ctx.close()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
