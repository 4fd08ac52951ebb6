"""Split of the GPU PNG path (yv_seq_upload_gpu): host read + gather vs the inflate / unfilter kernels, on a
synthetic stereo sequence written as cv::imwrite does.  python tools/png_gpu_probe.py [--frames 256] [--threads 16]"""
import argparse
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch
    import ya_vo_amd as yv
    from ya_vo_amd.io import PngDecoder, Sequence, png_write_gray
    from ya_vo_amd.synth import synth_stereo_batch
    from concurrent.futures import ThreadPoolExecutor
    H, W, n = 376, 1241, a.frames
    fr = synth_stereo_batch(7, n, start=0)
    tmp = tempfile.mkdtemp(prefix="yavo_pngp_")
    for side in ("image_0", "image_1"):
        os.makedirs(os.path.join(tmp, side))
    with ThreadPoolExecutor(a.threads) as ex:
        list(ex.map(lambda k: png_write_gray(os.path.join(tmp, "image_%d" % (k % 2), "%06d.png" % (k // 2)), fr[k]),
                    range(2 * n)))
    ctx = yv.Context(0)
    seq = Sequence(tmp, stereo=True)
    dec = PngDecoder(ctx, 2 * n, H, W)
    d = torch.zeros(2 * n * H * W, dtype=torch.uint8, device="cuda:0")
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dec.upload_sequence(seq, 0, n, d.data_ptr(), H * W, a.threads)
        t1 = time.perf_counter()
        codes, bad = dec.status()
        t2 = time.perf_counter()
        print(f"rep {rep}: host read+gather+launch {1e3*(t1-t0):.1f} ms, GPU after that {1e3*(t2-t1):.1f} ms, "
              f"total {1e3*(t2-t0):.1f} ms = {n/(t2-t0):.0f} stereo frames/s, bad {bad}")
    assert np.array_equal(d.cpu().numpy().reshape(-1, H, W), fr)
    t0 = time.perf_counter()
    seq.read(0, n, a.threads)
    print(f"host decode of the same files: {1e3*(time.perf_counter()-t0):.1f} ms")
    dec.close()
    seq.close()


if __name__ == "__main__":
    main()
