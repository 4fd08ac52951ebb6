"""Host side of the PNG path on the GPU box: how fast 16 threads stat / read / gather a KITTI-size stereo PNG sequence
(page cache), separately.  python tools/host_read_probe.py [--frames 1024] [--threads 16]"""
import argparse
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    from ya_vo_amd.io import png_write_gray
    from ya_vo_amd.synth import synth_stereo_batch
    n = a.frames
    tmp = tempfile.mkdtemp(prefix="yavo_hrp_", dir=a.dir)
    fr = synth_stereo_batch(7, min(n, 64), start=0)
    paths = [os.path.join(tmp, "%06d_%d.png" % (k // 2, k % 2)) for k in range(2 * n)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(a.threads) as ex:
        list(ex.map(lambda k: png_write_gray(paths[k], fr[k % len(fr)]), range(2 * n)))
    print(f"dir {tmp}: wrote {2*n} files in {time.perf_counter()-t0:.2f} s", flush=True)
    os.sync()
    sizes = [os.path.getsize(p) for p in paths]
    tot = sum(sizes)
    buf = np.empty(tot + 64 * len(paths), np.uint8)
    offs = np.cumsum([0] + [(s + 63) & ~63 for s in sizes])[:-1]

    def rd(k):
        fd = os.open(paths[k], os.O_RDONLY)
        mv = memoryview(buf)[offs[k]:offs[k] + sizes[k]]
        got = os.readv(fd, [mv])
        os.close(fd)
        return got
    with ThreadPoolExecutor(a.threads) as ex:
        for rep in range(4):
            t0 = time.perf_counter()
            list(ex.map(lambda k: os.stat(paths[k]).st_size, range(2 * n)))
            t1 = time.perf_counter()
            list(ex.map(rd, range(2 * n)))
            t2 = time.perf_counter()
            list(ex.map(lambda k: buf[offs[k]:offs[k] + sizes[k] - 12].__setitem__(slice(None), buf[offs[k] + 12:offs[k] + sizes[k]]), range(2 * n)))
            t3 = time.perf_counter()
            print(f"rep {rep}: stat {1e3*(t1-t0):.1f} ms, read {1e3*(t2-t1):.1f} ms ({tot/(t2-t1)/1e9:.1f} GB/s), "
                  f"memmove {1e3*(t3-t2):.1f} ms ({tot/(t3-t2)/1e9:.1f} GB/s); {tot/1e6:.0f} MB", flush=True)
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
