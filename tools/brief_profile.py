"""Phase breakdown of brief_kernel (lane 0 of each workgroup, shader-clock cycles) from the profiling build.

    make -C ya_vo_amd/csrc prof && python tools/brief_profile.py [--frames 512]"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import ya_vo_amd as yv  # noqa: E402
from ya_vo_amd.synth import synth_stereo_batch  # noqa: E402

PHASES = ["keypoint list scan", "band staging", "descriptors + records", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--lib", default=os.path.join(ROOT, "ya_vo_amd", "lib", "libyavo_prof.so"))
    args = ap.parse_args()
    lib = yv.load_library(args.lib)
    lib.yv_debug_brief_prof.argtypes = [ctypes.c_void_p]
    H, W, B = 376, 1241, args.frames
    ctx = yv.Context(0)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8))
    d = torch.from_numpy(synth_stereo_batch(1234, B)).to("cuda:0")
    b = yv.Batch(ctx, 2 * B, H, W, 2000, 0)
    buf = np.zeros((16384, 6), np.uint64)
    for _ in range(2):
        b.run(d.data_ptr(), 2 * B, W, H * W, 20)
    ctx.sync()
    b.enable_timing(True)
    b.run(d.data_ptr(), 2 * B, W, H * W, 20)
    ctx.sync()
    ms, _ = b.stage_times()
    assert lib.yv_debug_brief_prof(buf.ctypes.data) == 0
    wgs = min(((H + 31) // 32) * 2 * B, 16384)
    per = buf[:wgs, :2].astype(np.float64).mean(0)
    print(f"brief {ms[2]:.4f} ms for {2 * B} images, {wgs} workgroups; mean cycles per workgroup (lane 0): "
          f"{per.sum():.0f}")
    for name, v in zip(("list scan + band staging", "descriptors + records"), per):
        print(f"  {name:30s} {v:9.0f}  ({100 * v / max(per.sum(), 1):5.1f}%)")
    # residency: workgroups per CU over time (s_memrealtime, 100 MHz; CU = (XCC, SE, SH, CU) of HW_ID)
    t0 = buf[:wgs, 2].astype(np.int64)
    t1 = buf[:wgs, 3].astype(np.int64)
    hw = buf[:wgs, 4].astype(np.int64)
    xcc = (buf[:wgs, 5] & np.uint64(0xF)).astype(np.int64)
    cu = xcc * 4096 + ((hw >> 8) & 0xF) + 16 * ((hw >> 12) & 1) + 32 * ((hw >> 13) & 7)
    span = t1.max() - t0.min()
    busy = {}
    for c in np.unique(cu):
        m = cu == c
        ev = sorted([(a, 1) for a in t0[m]] + [(b, -1) for b in t1[m]])
        cur = mx = 0
        for _, d in ev:
            cur += d
            mx = max(mx, cur)
        busy[int(c)] = (int(m.sum()), mx, float((t1[m] - t0[m]).sum()) / span)
    v = np.array(list(busy.values()), np.float64)
    print(f"  span {span / 100:.1f} us over {len(busy)} CUs; workgroups per CU mean {v[:, 0].mean():.1f}; max resident "
          f"per CU: mean {v[:, 1].mean():.2f} max {v[:, 1].max():.0f}; mean resident over the span {v[:, 2].mean():.2f}; "
          f"mean workgroup life {(t1 - t0).mean() / 100:.2f} us")
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
