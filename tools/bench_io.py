"""Frame I/O throughput: KITTI-size (1241 x 376) 8-bit grey PNG frames written to a temporary
sequence directory, then decoded by yv_seq_read (host threads) and by yv_seq_upload (decode into pinned staging +
async copy to HBM).  The reference reads one frame per cv::imread on its tracking thread (src/LoopHandler.cc:919).

    python tools/bench_io.py [--frames 256] [--threads 16]

Prints one JSON object (committed as profiles/r01_io.json)."""
import argparse
import json
import os
import struct
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def encode_png(img, level=6):
    H, W = img.shape
    raw = np.concatenate([np.zeros((H, 1), np.uint8), img], 1).tobytes()  # filter 0 rows

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, 0, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(raw, level)) + chunk(b"IEND", b""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    import torch
    import ya_vo_amd as yv
    from ya_vo_amd import io as yio
    from ya_vo_amd.synth import synth_stereo_batch

    n = args.frames
    imgs = synth_stereo_batch(9, n)[::2]  # left images of n frames
    H, W = imgs.shape[1:]
    out = {"frames": n, "H": int(H), "W": int(W), "threads": args.threads}
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "image_0"))
        size = 0
        for k in range(n):
            data = encode_png(imgs[k])
            size += len(data)
            with open(os.path.join(d, "image_0", f"{k:06d}.png"), "wb") as f:
                f.write(data)
        out["mean_png_bytes"] = round(size / n)
        seq = yio.Sequence(d)
        seq.read(0, min(n, 8), threads=args.threads)  # warm the page cache and the code
        t0 = time.perf_counter()
        host = seq.read(0, n, threads=args.threads)
        t_read = time.perf_counter() - t0
        assert np.array_equal(host, imgs)
        t0 = time.perf_counter()
        seq.read(0, min(n, 32), threads=1)
        t_one = time.perf_counter() - t0
        ctx = yv.Context(0)
        dev = torch.empty((n, H * W), dtype=torch.uint8, device="cuda:0")
        s = torch.cuda.Stream()
        seq.upload(ctx, 0, min(n, 8), dev.data_ptr(), stream=s.cuda_stream)
        s.synchronize()
        chunk = 32
        t0 = time.perf_counter()
        for f0 in range(0, n, chunk):
            m = min(chunk, n - f0)
            seq.upload(ctx, f0, m, dev[f0].data_ptr(), stream=s.cuda_stream)
        s.synchronize()
        t_up = time.perf_counter() - t0
        assert np.array_equal(dev.cpu().numpy().reshape(n, H, W), imgs)
        out.update({"read_frames_per_s": round(n / t_read, 1), "read_1thread_frames_per_s": round(min(n, 32) / t_one, 1),
                    "upload_frames_per_s": round(n / t_up, 1), "upload_chunk_frames": chunk,
                    "decoded_GB_per_s": round(n * H * W / t_up / 1e9, 3)})
        seq.close()
        ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
