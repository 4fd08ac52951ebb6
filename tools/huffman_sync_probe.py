"""How fast a deflate decoder started at an arbitrary bit falls onto the true token boundaries (the premise of the
lane-parallel inflate in ya_vo_amd/csrc/yavo_inflate.hip).  A synthetic KITTI-size frame is written as cv::imwrite
does (yv_png_write_gray: Sub rows, zlib level 1, Z_RLE); the first dynamic block is decoded from its start (true token
starts), then from `--starts` random bit offsets until the decoder lands on a true start.  Pure Python (slow, a
few minutes): python tools/huffman_sync_probe.py [--starts 2000]"""
import argparse
import collections
import os
import random
import struct
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LE = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DE = [0, 0, 0, 0] + [k // 2 - 1 for k in range(4, 30)]


class Reader:
    def __init__(self, data):
        self.bits = int.from_bytes(data, "little")
        self.pos = 0

    def get(self, n):
        v = (self.bits >> self.pos) & ((1 << n) - 1)
        self.pos += n
        return v


def canonical(lens):
    cnt = collections.Counter(l for l in lens if l)
    code, nxt = 0, {}
    for l in range(1, 16):
        code = (code + cnt.get(l - 1, 0)) << 1 if l > 1 else 0
        nxt[l] = code
    table = {}
    for s, l in enumerate(lens):
        if l:
            table[(l, nxt[l])] = s
            nxt[l] += 1
    return table


def sym(rd, table):
    code = 0
    for l in range(1, 16):
        code = (code << 1) | rd.get(1)
        if (l, code) in table:
            return table[(l, code)]
    raise ValueError("no code")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--starts", type=int, default=2000)
    a = ap.parse_args()
    from ya_vo_amd.io import png_write_gray
    from ya_vo_amd.synth import synth_stereo_batch
    path = os.path.join(tempfile.mkdtemp(), "f.png")
    png_write_gray(path, synth_stereo_batch(7, 1, start=0)[0])
    b = open(path, "rb").read()
    p, idat = 8, b""
    while p < len(b):
        n, = struct.unpack(">I", b[p:p + 4])
        if b[p + 4:p + 8] == b"IDAT":
            idat += b[p + 8:p + 8 + n]
        p += 12 + n
    rd = Reader(idat[2:])
    rd.get(1)
    assert rd.get(2) == 2, "expected a dynamic block"
    hl, hd, hc = rd.get(5) + 257, rd.get(5) + 1, rd.get(4) + 4
    cl = [0] * 19
    for k in range(hc):
        cl[[16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15][k]] = rd.get(3)
    ct, L = canonical(cl), []
    while len(L) < hl + hd:
        s = sym(rd, ct)
        L += [s] if s < 16 else [L[-1]] * (3 + rd.get(2)) if s == 16 else [0] * (3 + rd.get(3)) if s == 17 \
            else [0] * (11 + rd.get(7))
    lt, dt = canonical(L[:hl]), canonical(L[hl:])

    def token():
        s = sym(rd, lt)
        if s > 256:
            if s - 257 >= 29:
                raise ValueError("length")
            rd.get(LE[s - 257])
            d = sym(rd, dt)
            if d >= 30:
                raise ValueError("distance")
            rd.get(DE[d])
        return s
    starts, first = set(), rd.pos
    while True:
        starts.add(rd.pos)
        if token() == 256:
            break
    end = rd.pos
    random.seed(1)
    res = []
    for _ in range(a.starts):
        o = random.randrange(first + 100, end - 2000)
        rd.pos = o
        try:
            while rd.pos not in starts:
                token()
            res.append(rd.pos - o)
        except ValueError:
            res.append(-1)
    r = np.array(res)
    ok = r[r >= 0]
    print(f"first block: {end - first} bits, {len(starts)} tokens; {a.starts} random starts, {(r < 0).sum()} hit an "
          f"invalid code first; bits to synchronise: mean {ok.mean():.1f}, median {np.median(ok):.0f}, p99 "
          f"{np.percentile(ok, 99):.0f}, max {ok.max()}; > 64: {(ok > 64).mean():.3f}, > 128: {(ok > 128).mean():.4f},"
          f" > 256: {(ok > 256).mean():.4f}")


if __name__ == "__main__":
    main()
