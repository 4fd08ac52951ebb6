"""What the oracle's two libm substitutions move: g2o's pow(2 rho - 1, 3) is
restated as a correctly rounded cube (or_cube) and Sophus' std::sin / std::cos as fdlibm's kernels; the GPU kernels
share both, so the bit-exact tests cannot see them.  The oracle's libm flavour 1 calls the host C library instead, as
the reference's g2o / Sophus build does.  CPU only (the oracle on this host's glibc).

    python tools/libm_flavour_report.py [--problems 2048] [--frames 200] [--out profiles/r04/libm_flavour.json]

* pose LM (optimizePoseOnly, src/LoopHandler.cc:730-861): `--problems` bench-shaped problems (1920 edges, 0.5 px
  noise, 10% gross outliers, perturbed prior), kernel sum order, flavour 0 vs 1;
* the configs[2] front end (tests/sequence_chain.py: track + map + sliding-window BA) over `--frames` synthetic
  stereo frames, flavour 0 vs 1."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)


def compare(a, b):
    a, b = np.asarray(a), np.asarray(b)
    differ = ~np.all(a == b, axis=1)
    d = a - b
    return {"poses": int(len(a)), "poses_differing": int(differ.sum()),
            "max_abs_diff": float(np.abs(d).max()) if len(a) else 0.0,
            "translation_rmse": float(np.sqrt(np.mean(np.sum(d[:, 4:] ** 2, axis=1)))) if len(a) else 0.0}


def pose_lm_leg(orc, n, threads):
    import ya_vo_amd as yv
    from ya_vo_amd import scene
    probs = [scene.random_scene(1920, seed=5000 + i, noise_px=0.5, outlier_frac=0.1) for i in range(n)]
    priors = [scene.perturb(p[2], np.random.default_rng(i)) for i, p in enumerate(probs)]
    mode = yv.lm_sum_mode()
    out = {}
    for flav in (0, 1):
        orc.set_libm_flavour(flav)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(lambda i: orc.pose_lm(probs[i][0], probs[i][1], scene.K_KITTI, priors[i], mode), range(n)))
        out[flav] = (np.array([r[0] for r in res]), np.array([r[2] for r in res]), time.perf_counter() - t0)
    orc.set_libm_flavour(0)
    r = compare(out[0][0], out[1][0])
    r["inlier_counts_differing"] = int(np.sum(out[0][1] != out[1][1]))
    r["what"] = (f"{n} pose-only LM problems (1920 edges, 0.5 px noise, 10% gross outliers, perturbed prior), "
                 "kernel sum order, oracle flavour 0 (restated pow / sin / cos = the GPU's) vs 1 (host glibc)")
    return r


def sequence_leg(orc, offsets, n, threads):
    from sequence_chain import oracle_sequence
    from ya_vo_amd import scene
    from ya_vo_amd.synth import synth_sequence
    frames = synth_sequence(71, n, stereo=True)
    res = {}
    for flav in (0, 1):
        orc.set_libm_flavour(flav)
        traj, _, log = oracle_sequence(orc, frames, 20, scene.K_KITTI, T_RIGHT, offsets, threads=threads)
        res[flav] = (traj, log)
    orc.set_libm_flavour(0)
    r = compare(res[0][0], res[1][0])
    r["ba_logs_identical"] = bool(res[0][1] == res[1][1])
    r["what"] = (f"configs[2] front end over {n} synthetic stereo frames (chunks of 20, BA windows of 22 poses; "
                 "tests/sequence_chain.py), trajectory T_wc, oracle flavour 0 vs 1")
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=2048)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import oracle_bind
    orc = oracle_bind.Oracle()
    offsets = np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8).reshape(256, 4)
    rep = {"host_libc": os.confstr("CS_GNU_LIBC_VERSION") if hasattr(os, "confstr") else None}
    # the cube alone: how often glibc's pow(t, 3) differs from the correctly rounded cube over the LM's arguments
    rng = np.random.default_rng(0)
    t = rng.uniform(-1, 1, 1_000_000)
    rep["cube_vs_pow_differing_fraction"] = float(np.mean(orc.cube(t, 0) != orc.cube(t, 1)))
    if args.problems:
        rep["pose_lm"] = pose_lm_leg(orc, args.problems, args.threads)
    if args.frames:
        rep["sequence"] = sequence_leg(orc, offsets, args.frames, args.threads)
    s = json.dumps(rep, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
