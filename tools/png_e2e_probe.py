"""Where the PNG end-to-end step's time goes (bench.py png_end_to_end, GPU decode): host seconds per call
(upload of the B frames, the halo frame, shard.step) and the step's wall time.  python tools/png_e2e_probe.py"""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import ya_vo_amd as yv
    from ya_vo_amd import map as ymap
    from ya_vo_amd import scene
    from ya_vo_amd.io import PngDecoder, Sequence
    from ya_vo_amd.sharding import FrameShard, shard_images
    from ya_vo_amd.synth import synth_stereo_batch
    B = int(os.environ.get("PROBE_FRAMES", "1024"))
    steps = int(os.environ.get("PROBE_STEPS", "6"))
    thr = bench.cpu_threads_available()
    offsets = np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8)
    ctx = yv.Context(0)
    ctx.set_brief_offsets(offsets)
    fr = synth_stereo_batch(1234, B + 1, start=0)
    images = shard_images(fr[2:], fr[0], None)
    halo_right = fr[1].copy()
    max_kf = ymap.max_keyframes(B, 1, 4)
    shard = FrameShard(ctx, B, 1, scene.K_KITTI, bench.T_RIGHT, halo=True, world=1, rank=0, backend="nccl",
                       kf_every=4, max_kf=max_kf, overlap_mode=1, tracker="match")
    tmp = tempfile.mkdtemp(prefix="yavo_pe2e_")
    left = [images[2 * B]] + [images[2 * k] for k in range(B)]
    right = [halo_right] + [images[2 * k + 1] for k in range(B)]
    bench.write_png_sequence(tmp, left, right, thr)
    seq = Sequence(tmp, stereo=True)
    H, W = 376, 1241
    img = H * W
    bufs = [torch.empty((2 * B + 2) * img, dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    dec = PngDecoder(ctx, 2 * B + 2, H, W)
    for i in range(steps):
        k = i % 2
        t0 = time.perf_counter()
        dec.upload_frames(seq, list(range(1, B + 1)) + [0], bufs[k].data_ptr(), img, thr)
        t1 = t2 = time.perf_counter()
        shard.step(bufs[k].data_ptr())
        t3 = time.perf_counter()
        print(f"step {i}: upload B {1e3*(t1-t0):.1f} ms, halo {1e3*(t2-t1):.1f} ms, shard.step {1e3*(t3-t2):.1f} ms",
              flush=True)
    shard.drain()
    torch.cuda.synchronize()
    codes, bad = dec.status()
    print("bad", bad)
    dec.close()
    seq.close()
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
