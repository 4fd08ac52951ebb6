"""Phase breakdown of the batched pose LM (pose_lm_kernel) from a YAVO_LM_PROFILE build.

    make -C ya_vo_amd/csrc prof && python tools/lm_profile.py [--frames 64]

Runs the bench's pipeline (detect .. track) on synthetic stereo frames with lib/libyavo_prof.so and prints
the mean shader-clock cycles per workgroup spent in each phase of the LM kernel."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import ya_vo_amd as yv  # noqa: E402
from ya_vo_amd import scene  # noqa: E402
from ya_vo_amd.synth import synth_stereo_batch  # noqa: E402

PHASES = ["edge compute (lane 0's share)", "tree reduce proper", "lane-0 exp/mul", "accept + barriers",
          "classify/compact", "iteration setup", "lane-0 T backup + LDLT", "lane-0 system copy (iteration)", "wait for other waves' edges", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--plain", action="store_true", help="use the product library (for PMC runs), no phase timers")
    ap.add_argument("--lib", default="", help="with --plain: this library instead of lib/libyavo.so")
    args = ap.parse_args()
    lib = yv.load_library(args.lib if (args.plain and args.lib) else
                          os.path.join(ROOT, "ya_vo_amd", "lib", "libyavo.so" if args.plain else "libyavo_prof.so"))
    if not args.plain:
        lib.yv_debug_lm_prof.argtypes = [ctypes.c_void_p]
    H, W, B = 376, 1241, args.frames
    ctx = yv.Context(0)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8))
    d = torch.from_numpy(synth_stereo_batch(1234, B)).to("cuda:0")
    b = yv.Batch(ctx, 2 * B, H, W, 2000, 2 * B)
    pairs, tracks = [], []
    for k in range(B):
        pairs += [(2 * B if k == 0 else 2 * (k - 1), 2 * k), (2 * k, 2 * k + 1)]
        tracks.append((2 * k + 1, 2 * k))
    b.set_pairs(pairs)
    b.set_tracks(tracks, scene.K_KITTI, [0, 0, 0, 1, 0, -0.54, 0])
    prior = torch.from_numpy(np.tile(np.array([0, 0, 0, 1, 0, 0, 0.]), (B, 1))).to("cuda:0")
    pose = torch.zeros_like(prior)
    for _ in range(2):
        b.run(d.data_ptr(), 2 * B, W, H * W, 20, carry_from=2 * (B - 1))
        b.track(prior.data_ptr(), pose.data_ptr())
    b.enable_timing(True)
    b.run(d.data_ptr(), 2 * B, W, H * W, 20, carry_from=2 * (B - 1))
    b.track(prior.data_ptr(), pose.data_ptr())
    ctx.sync()
    ms, _ = b.stage_times()
    if args.plain:
        print(f"track_pose {ms[6]:.4f} ms, track_edges {ms[5]:.4f} ms, frames {B}")
        return
    prof = np.zeros((1024, 10), np.uint64)
    assert lib.yv_debug_lm_prof(prof.ctypes.data) == 0
    p = prof[1:B].astype(np.float64)  # track 0 reads the carry slot
    tot = p[:, :9].sum(1)
    print(f"track_pose {ms[6]:.4f} ms, frames {B}; mean cycles per workgroup: total {tot.mean():.0f}")
    for i in range(9):
        print(f"  {PHASES[i]:32s} {p[:, i].mean():12.0f}  ({100 * p[:, i].mean() / tot.mean():5.1f}%)")
    print(f"  passes per problem: mean {p[:, 9].mean():.1f}, max {p[:, 9].max():.0f}; "
          f"cycles per pass {tot.mean() / max(p[:, 9].mean(), 1):.0f}")
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
