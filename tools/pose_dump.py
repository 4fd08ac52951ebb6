#!/usr/bin/env python3
"""Dump one bench step's PnP problems (edges) and the GPU's poses / outlier flags for offline comparison with the
oracle (tools/pose_diff.py).  Runs the bench's shard (512 frames, overlap mode 1 by default) for `--steps` steps.

    python tools/pose_dump.py [--frames B] [--steps K] [--overlap-mode M] [--out gpurun_out/pose_dump.npz]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--overlap-mode", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pose_dump.npz"))
    a = ap.parse_args()
    import torch
    import ya_vo_amd as yv
    from ya_vo_amd import scene
    from ya_vo_amd.sharding import FrameShard, shard_images
    from ya_vo_amd.synth import synth_stereo_batch
    T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
    offsets = np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8)
    ctx = yv.Context(0)
    ctx.set_brief_offsets(offsets)
    B = a.frames
    fr = synth_stereo_batch(1234, B + 1, start=0)
    images = shard_images(fr[2:], fr[0])
    d = torch.from_numpy(images).to("cuda:0")
    sh = FrameShard(ctx, B, 1, scene.K_KITTI, T_RIGHT, halo=True, overlap_mode=a.overlap_mode)
    runs = []
    for i in range(a.steps):
        sh.step(d.data_ptr())
        sh.drain()
        v = sh.batch.view()
        NT = sh.n_tracks
        ec = ctx.download(v.edge_count, np.int32, NT)
        eX = ctx.download(v.edge_X, np.float64, NT * 2000 * 3).reshape(NT, 2000, 3)
        euv = ctx.download(v.edge_uv, np.float64, NT * 2000 * 2).reshape(NT, 2000, 2)
        inl = ctx.download(v.track_inliers, np.int32, NT)
        runs.append((ec, eX, euv, inl, sh.poses().copy()))
    ec, eX, euv, inl, P = runs[-1]
    same = [bool(np.array_equal(r[4], P)) for r in runs]
    same_e = [bool(np.array_equal(r[1], eX)) for r in runs]
    print("poses equal across steps:", same, "edges equal across steps:", same_e, "lm_sum_mode", yv.lm_sum_mode())
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    m = int(ec.max())
    np.savez_compressed(a.out, ec=ec, eX=eX[:, :m], euv=euv[:, :m], inl=inl, poses=P,
                        poses_all=np.stack([r[4] for r in runs]), sum_mode=yv.lm_sum_mode())
    sh.close()
    ctx.close()


if __name__ == "__main__":
    main()
