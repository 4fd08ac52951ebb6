#!/usr/bin/env python3
"""Compare a pose dump (tools/pose_dump.py) with the oracle's pose LM in the kernel's sum order and in the
reference's sequential order (sum_mode 0); lists the frames whose GPU pose is not bit-identical.

    python tools/pose_diff.py gpurun_out/pose_dump.npz
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import oracle_bind
    from ya_vo_amd import scene
    z = np.load(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pose_dump.npz"))
    ec, eX, euv, P, mode = z["ec"], z["eX"], z["euv"], z["poses"], int(z["sum_mode"])
    orc = oracle_bind.Oracle()
    prior = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)

    def one(k):
        X, uv = eX[k, :ec[k]], euv[k, :ec[k]]
        g = orc.pose_lm(X, uv, scene.K_KITTI, prior, mode)
        s = orc.pose_lm(X, uv, scene.K_KITTI, prior, 0)
        return g[0], g[2], s[0], s[2]

    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(one, range(len(ec))))
    g = np.array([r[0] for r in res])
    s = np.array([r[2] for r in res])
    bad = np.nonzero(np.any(g != P, axis=1))[0]
    print(f"{len(ec)} frames, sum_mode {mode}: {len(bad)} not bit-identical to the oracle in the kernel's order")
    for k in bad[:20]:
        print(f"  frame {k}: edges {ec[k]} inliers gpu {z['inl'][k]} oracle {res[k][1]} seq {res[k][3]}  "
              f"max|d| {np.abs(g[k] - P[k]).max():.3e}")
    d = P - s
    print("RMSE(t) vs sum_mode 0:", float(np.sqrt(np.mean(np.sum(d[:, 4:] ** 2, 1)))),
          "max|d|:", float(np.abs(d).max()), "at frame", int(np.argmax(np.abs(d).max(1))))
    if "poses_all" in z.files:
        pa = z["poses_all"]
        print("GPU poses identical across dumped steps:", [bool(np.array_equal(p, P)) for p in pa])


if __name__ == "__main__":
    main()
