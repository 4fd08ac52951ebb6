"""Latency of the LoopHandler's reinitialisation primitives on the lists it actually sees.

The drop-in LoopHandler (bench_loop_handler.py's synthetic sequence: frame k is a crop of one noise field at (k, 3k))
re-initialises on matchFeatures(last, curr) + removeOutliers(20) of consecutive frames, i.e. correspondences that
are one pure image translation apart, plus mismatches.  getFRANSAC and findEssentialMat on such lists are far more
degenerate than the two-view scenes of bench_geometry.py.  This probe times both host calls on (a) those lists and
(b) a bench_geometry two-view scene of the same size, so the difference is the data, not the code.

    python tools/reinit_probe.py [--pairs 4] [--reps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

import ya_vo_amd as yv  # noqa: E402
from ya_vo_amd.synth import synth_frame  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return r, round(1e3 * float(np.median(ts)), 4)


def probe_list(ctx, m, reps, rng):
    n = len(m)
    samples = rng.integers(0, n, size=(400, 8)).astype(np.int32)
    (fo, _, finl), f_ms = timed(lambda: ctx.f_ransac(m, samples), reps)
    prev = np.c_[m["pt1"]["x"], m["pt1"]["y"]].astype(np.float32)
    curr = np.c_[m["pt2"]["x"], m["pt2"]["y"]].astype(np.float32)
    (eo, _, mask), e_ms = timed(lambda: ctx.find_essential(curr, prev), reps)
    d = curr - prev
    return {"matches": n, "f_ransac_ms": f_ms, "f_inliers": finl, "find_essential_ms": e_ms,
            "essential_inliers": int(mask.sum()), "same_shift_frac": float(np.mean(np.all(d == np.median(d, 0), 1)))}


def loop_handler_lists(ctx, pairs, H=376, W=1241):
    """matchFeatures + removeOutliers(20) of `pairs` consecutive-frame pairs of bench_loop_handler.py's sequence (crops
    one (1, 3) px step apart), as the LoopHandler's re-initialisation sees them.  ctx needs the BRIEF offsets."""
    out = []
    for j in range(pairs):
        kps = []
        for k in (37 * j, 37 * j + 1):
            img = synth_frame(2024, k, 3 * k, H, W)
            rc, _, _ = ctx.detect(img)
            kps.append(ctx.describe(img, rc))
        out.append(ctx.filter_matches(ctx.match_features(kps[0], kps[1]), 20))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    ctx = yv.Context(0)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8))
    rng = np.random.default_rng(0)
    out = {"loop_handler_lists": [], "two_view_scene": None}
    for m in loop_handler_lists(ctx, a.pairs):
        out["loop_handler_lists"].append(probe_list(ctx, m, a.reps, rng))
    # bench_geometry's list: a two-view scene with 20% gross outliers as match records
    from epipolar_scene import two_view_scene
    p1, p2, _, _ = two_view_scene(1935, outlier_frac=0.2, seed=500, angle=0.02)
    m = np.zeros(len(p1), dtype=yv.MATCH_DTYPE)
    m["pt1"]["x"], m["pt1"]["y"] = p1[:, 0], p1[:, 1]
    m["pt2"]["x"], m["pt2"]["y"] = p2[:, 0], p2[:, 1]
    out["two_view_scene"] = probe_list(ctx, m, a.reps, rng)
    ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
