"""Phase breakdown of detect_kernel (lane 0 of each workgroup, shader-clock cycles) from the profiling build.

    make -C ya_vo_amd/csrc prof && python tools/det_profile.py [--frames 256]"""
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

PHASES = ["stage tile (loads + LDS)", "FAST phase 1 (pretest)", "FAST phase 2 (full test)",
          "blur horizontal (+ atomic)", "Harris", "blur vertical + stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    args = ap.parse_args()
    lib = yv.load_library(os.path.join(ROOT, "ya_vo_amd", "lib", "libyavo_prof.so"))
    lib.yv_debug_det_prof.argtypes = [ctypes.c_void_p]
    H, W, B = 376, 1241, args.frames
    ctx = yv.Context(0)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8))
    d = torch.from_numpy(synth_stereo_batch(1234, B)).to("cuda:0")
    b = yv.Batch(ctx, 2 * B, H, W, 2000, 0)
    buf = np.zeros((131072, 6), np.uint64)
    for _ in range(2):
        b.run(d.data_ptr(), 2 * B, W, H * W, 20)
    ctx.sync()
    b.enable_timing(True)
    b.run(d.data_ptr(), 2 * B, W, H * W, 20)
    ctx.sync()
    ms, _ = b.stage_times()
    assert lib.yv_debug_det_prof(buf.ctypes.data) == 0
    wgs = ((W + 63) // 64) * ((H + 55) // 56) * 2 * B  # 64 x 56 tiles (kFastTileW x kFastTileH)
    per = buf[:min(wgs, 131072)].astype(np.float64).mean(0)
    print(f"detect {ms[0]:.4f} ms for {2 * B} images, {wgs} workgroups; mean cycles per workgroup (lane 0): "
          f"{per.sum():.0f}")
    for name, v in zip(PHASES, per):
        print(f"  {name:30s} {v:9.0f}  ({100 * v / per.sum():5.1f}%)")
    b.close()
    ctx.close()


if __name__ == "__main__":
    main()
