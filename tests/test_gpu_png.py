"""PNG decoding on the GPU (yv_pngdec_*, ya_vo_amd/csrc/yavo_inflate.hip) against the host decoder
(yv_png_decode_gray, itself pinned to PIL in tests/test_io.py): byte for byte on the reference's own KITTI frame
(tests/epilines.png's content, re-encoded), cv::imwrite-style files (Sub rows, deflate level 1, Z_RLE), PIL-written
files (adaptive filters, default level), stored blocks (level 0), fixed-Huffman blocks (tiny images), every filter
type, odd sizes, and a corrupted stream (reported, no fault)."""
import io as _io
import os
import struct
import zlib

import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd.io import PngDecoder, Sequence, png_decode_gray, png_write_gray

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _png(img, filt, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    """8-bit grey PNG with one filter type per row (filt: int or list), zlib at `level`."""
    H, W = img.shape
    a = img.astype(np.int16)
    rows = []
    for r in range(H):
        f = filt[r % len(filt)] if isinstance(filt, (list, tuple)) else filt
        cur = a[r]
        up = a[r - 1] if r else np.zeros(W, np.int16)
        left = np.concatenate([[0], cur[:-1]])
        ul = np.concatenate([[0], up[:-1]])
        if f == 0:
            pred = np.zeros(W, np.int16)
        elif f == 1:
            pred = left
        elif f == 2:
            pred = up
        elif f == 3:
            pred = (left + up) >> 1
        else:
            p = left + up - ul
            pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
        rows.append(bytes([f]) + ((cur - pred) & 0xFF).astype(np.uint8).tobytes())
    c = zlib.compressobj(level, zlib.DEFLATED, 15, 8, strategy)
    z = c.compress(b"".join(rows)) + c.flush()
    return _png_from_z(z, H, W)


def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _png_from_z(z, H, W):
    """A PNG around the zlib stream z, IDAT split over 8 KB chunks as encoders do, every chunk CRC correct."""
    idat = b"".join(_chunk(b"IDAT", z[i:i + 8192]) for i in range(0, len(z), 8192))
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, 0, 0, 0, 0)) + idat +
            _chunk(b"IEND", b""))


def _zstream(f):
    """The zlib stream of a PNG file (its IDAT payloads concatenated)."""
    p, z = 8, b""
    while p < len(f):
        n = struct.unpack(">I", f[p:p + 4])[0]
        if f[p + 4:p + 8] == b"IDAT":
            z += bytes(f[p + 8:p + 8 + n])
        p += 12 + n
    return z


def _decode_gpu(ctx, files, H, W, checks=(1, 1)):
    import torch
    dec = PngDecoder(ctx, len(files), H, W)
    dec.set_checks(*checks)
    d = torch.zeros(len(files) * H * W, dtype=torch.uint8, device="cuda:0")
    dec.decode(files, d.data_ptr(), H * W)
    codes, bad = dec.status()
    out = d.cpu().numpy().reshape(len(files), H, W)
    dec.close()
    return out, codes[:len(files)], bad


def test_gpu_png_matches_host_decoder(ctx):
    from ya_vo_amd.synth import synth_frame
    rng = np.random.default_rng(5)
    H, W = 376, 1241
    frames = [synth_frame(17, k, 3 * k, H, W) for k in range(3)]
    ref = np.array(__import__("PIL.Image", fromlist=["Image"]).open(
        os.path.join(ROOT, "tests", "golden", "png", "epilines_crop.png")))
    files, expect = [], []
    for k, img in enumerate(frames):
        files.append(_png(img, 1, 1, zlib.Z_RLE))          # cv::imwrite style
        files.append(_png(img, [0, 1, 2, 3, 4], 6))       # every filter type, default level
        files.append(_png(img, 4, 9))                     # Paeth, best compression (long matches)
        expect += [img] * 3
    noise = rng.integers(0, 256, (H, W), dtype=np.uint8)
    files.append(_png(noise, 0, 0))                       # stored blocks
    expect.append(noise)
    flat = np.full((H, W), 77, np.uint8)
    files.append(_png(flat, 2, 6))                        # long runs, distance-1 and long-distance matches
    expect.append(flat)
    out, codes, bad = _decode_gpu(ctx, files, H, W)
    assert bad == 0, codes
    for i, (o, e) in enumerate(zip(out, expect)):
        np.testing.assert_array_equal(o, e, err_msg=f"file {i}")
        np.testing.assert_array_equal(png_decode_gray(files[i]), e)  # the host decoder agrees
    # the reference's KITTI crop (PIL-decoded) re-encoded by PIL with its adaptive filters
    from PIL import Image
    buf = _io.BytesIO()
    Image.fromarray(ref).save(buf, format="PNG")
    out2, _, bad2 = _decode_gpu(ctx, [buf.getvalue(), open(os.path.join(ROOT, "tests", "golden", "png",
                                                                         "epilines_crop.png"), "rb").read()], *ref.shape)
    assert bad2 == 0
    np.testing.assert_array_equal(out2[0], ref)
    np.testing.assert_array_equal(out2[1], ref)


@pytest.mark.parametrize("H,W", [(1, 1), (3, 5), (7, 64), (65, 129), (130, 3)])
def test_gpu_png_odd_sizes_fixed_huffman(ctx, H, W):
    """Tiny images compress to fixed-Huffman blocks; odd sizes exercise the last partial 4-byte group and bands of
    fewer than 64 rows."""
    rng = np.random.default_rng(H * 100 + W)
    imgs = [rng.integers(0, 256, (H, W), dtype=np.uint8), np.tile(np.arange(W, dtype=np.uint8), (H, 1))]
    files = [_png(imgs[0], [4, 3, 2, 1, 0], 6), _png(imgs[1], 1, 1, zlib.Z_FIXED)]
    out, codes, bad = _decode_gpu(ctx, files, H, W)
    assert bad == 0, codes
    np.testing.assert_array_equal(out[0], imgs[0])
    np.testing.assert_array_equal(out[1], imgs[1])


@pytest.mark.parametrize("H,W", [(9, 1241), (5, 3000), (4, 4100)])
def test_gpu_png_rowwise_and_wavefront_unfilter(ctx, H, W):
    """None / Sub / Up rows take the row-wise unfilter (64 lanes per row, up to W = 4096); any Average or Paeth row sends
    the image to the wavefront; wider images always take the wavefront."""
    rng = np.random.default_rng(W)
    img = rng.integers(0, 256, (H, W), dtype=np.uint8)
    img[:, W // 3:] = np.cumsum(img[:, W // 3:] & 3, axis=1, dtype=np.uint8)  # some compressible runs
    files = [_png(img, 1, 1, zlib.Z_RLE), _png(img, [2, 1, 0], 6), _png(img, [1, 2, 3], 6), _png(img, [2, 4], 6)]
    out, codes, bad = _decode_gpu(ctx, files, H, W)
    assert bad == 0, codes
    for o in out:
        np.testing.assert_array_equal(o, img)


PNG_ERR_CRC, PNG_ERR_ADLER = 7, 8


def test_gpu_png_reports_corrupt_stream(ctx):
    """cv::imread's integrity checks (libpng: a critical chunk's CRC-32; zlib: the Adler-32 trailer): a damaged IDAT
    chunk is reported by its CRC, a stream whose CRCs were recomputed by its Adler-32 (or a decode error), a wrong or
    missing trailer by its Adler-32; failed images come back zero-filled, the good ones intact."""
    H, W = 40, 50
    img = np.random.default_rng(1).integers(0, 256, (H, W), dtype=np.uint8)
    good = _png(img, 1, 6)
    z = _zstream(good)
    bad = bytearray(good)
    i = bad.index(b"IDAT") + 4 + 40
    for k in range(i, i + 30):
        bad[k] ^= 0x5A  # garbage inside the deflate data, the chunk CRC left as it was
    zb = bytearray(z)
    for k in range(40, 70):
        zb[k] ^= 0x5A   # the same garbage with valid chunk CRCs: zlib's own checks must catch it
    wrong_adler = z[:-4] + bytes([z[-4] ^ 1]) + z[-3:]
    no_trailer = z[:-4]
    files = [good, bytes(bad), good, _png_from_z(bytes(zb), H, W), _png_from_z(wrong_adler, H, W),
             _png_from_z(no_trailer, H, W)]
    out, codes, n_bad = _decode_gpu(ctx, files, H, W)
    np.testing.assert_array_equal(out[0], img)
    np.testing.assert_array_equal(out[2], img)
    assert codes[0] == 0 and codes[2] == 0
    assert codes[1] == PNG_ERR_CRC
    assert codes[3] != 0
    assert codes[4] == PNG_ERR_ADLER and codes[5] == PNG_ERR_ADLER
    assert n_bad == 4
    for k in (1, 3, 4, 5):
        assert not out[k].any(), k  # zero-filled


def test_gpu_png_status_counts_every_decode(ctx):
    """yv_pngdec_status's n_bad covers every decode since the previous query (a bench step decodes twice per status)."""
    import torch
    H, W = 16, 24
    img = np.random.default_rng(3).integers(0, 256, (H, W), dtype=np.uint8)
    good = _png(img, 2, 6)
    bad = bytearray(good)
    bad[bad.index(b"IDAT") + 10] ^= 0xFF
    dec = PngDecoder(ctx, 3, H, W)
    d = torch.zeros(3 * H * W, dtype=torch.uint8, device="cuda:0")
    dec.decode([good, bytes(bad), good], d.data_ptr(), H * W)
    dec.decode([bytes(bad), good, bytes(bad)], d.data_ptr(), H * W)
    codes, n_bad = dec.status()
    assert n_bad == 3
    assert list(codes[:3]) == [PNG_ERR_CRC, 0, PNG_ERR_CRC]  # the codes are the last decode's
    dec.decode([good, good, good], d.data_ptr(), H * W)
    codes, n_bad = dec.status()
    assert n_bad == 0 and not any(codes[:3])
    np.testing.assert_array_equal(d.cpu().numpy().reshape(3, H, W), np.stack([img] * 3))
    dec.close()


def test_gpu_png_sequence_upload(ctx, tmp_path):
    """yv_seq_upload_gpu: a stereo KITTI-layout sequence written as cv::imwrite does (yv_png_write_gray) decodes on the
    GPU to the same images as the host path (yv_seq_read)."""
    import torch
    from ya_vo_amd.synth import synth_stereo_batch
    H, W, n = 376, 1241, 6
    fr = synth_stereo_batch(99, n, start=0)
    for side in ("image_0", "image_1"):
        os.makedirs(tmp_path / side)
    for k in range(n):
        png_write_gray(str(tmp_path / "image_0" / f"{k:06d}.png"), fr[2 * k])
        png_write_gray(str(tmp_path / "image_1" / f"{k:06d}.png"), fr[2 * k + 1])
    seq = Sequence(str(tmp_path), stereo=True)
    dec = PngDecoder(ctx, 2 * n, H, W)
    d = torch.zeros(2 * (n - 1) * H * W, dtype=torch.uint8, device="cuda:0")
    dec.upload_sequence(seq, 1, n - 1, d.data_ptr(), H * W, threads=4)
    codes, bad = dec.status()
    assert bad == 0, codes
    np.testing.assert_array_equal(d.cpu().numpy().reshape(-1, H, W), seq.read(1, n - 1))
    np.testing.assert_array_equal(d.cpu().numpy().reshape(-1, H, W), fr[2:2 * n])
    # a frame list in one decode (a shard's frames, then its halo frame)
    d.zero_()
    dec.upload_frames(seq, [2, 3, 4, 0], d.data_ptr(), H * W, threads=3)
    codes, bad = dec.status()
    assert bad == 0, codes
    np.testing.assert_array_equal(d.cpu().numpy().reshape(-1, H, W)[:8],
                                  np.concatenate([fr[4:10], fr[0:2]]))
    dec.close()
    seq.close()


def test_gpu_png_bad_files_fail_alone(ctx, tmp_path):
    """A missing, truncated, RGB or wrong-size file in a GPU-decoded batch fails alone with code 9 (its image zero-filled,
    counted), as cv::imread fails per file; the batch's other images decode as the host decoder does."""
    import torch
    from PIL import Image
    from ya_vo_amd.synth import synth_stereo_batch
    H, W, n = 376, 1241, 8
    fr = synth_stereo_batch(5, n // 2, start=0).reshape(n, H, W)
    os.makedirs(tmp_path / "image_0")
    for k in range(n):
        png_write_gray(str(tmp_path / "image_0" / f"{k:06d}.png"), fr[k])
    seq = Sequence(str(tmp_path), stereo=False)
    p = lambda k: str(tmp_path / "image_0" / f"{k:06d}.png")  # noqa: E731
    data = open(p(2), "rb").read()
    open(p(2), "wb").write(data[:len(data) // 2])                                         # truncated
    Image.fromarray(np.stack([fr[4]] * 3, -1)).save(p(4))                                  # RGB
    png_write_gray(p(5), fr[5][:, :W - 1].copy())                                          # wrong size
    os.remove(p(6))                                                                        # missing (listed already)
    dec = PngDecoder(ctx, n, H, W)
    d = torch.full((n * H * W,), 7, dtype=torch.uint8, device="cuda:0")
    dec.upload_sequence(seq, 0, n, d.data_ptr(), H * W, threads=3)
    codes, bad = dec.status()
    assert list(codes) == [0, 0, 9, 0, 9, 9, 9, 0] and bad == 4
    out = d.cpu().numpy().reshape(n, H, W)
    for k in range(n):
        np.testing.assert_array_equal(out[k], fr[k] if codes[k] == 0 else np.zeros((H, W), np.uint8))
    dec.close()
    seq.close()


def test_gpu_png_randomized_streams_match_zlib(ctx):
    """Differential fuzz of the lane-parallel inflate: random sizes, row filters, zlib levels and strategies (every
    block type, short and long matches, far distances, chunks capped by highly compressible rows); then the same
    streams with random bytes flipped inside the deflate data: with the chunk CRCs left as they were every damaged file
    is reported by its CRC; with the CRCs recomputed every damaged file that zlib rejects (decode error or Adler-32) is
    reported too, and whenever zlib's raw inflate (no Adler-32 check) yields an image's worth of valid rows, the GPU's
    inflate produced the same bytes, which the Adler-32 then rejects (never a fault)."""
    rng = np.random.default_rng(20261017)
    strategies = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]
    H, W = 61, 203
    files, imgs = [], []
    for k in range(24):
        kind = k % 4
        if kind == 0:
            img = rng.integers(0, 256, (H, W), dtype=np.uint8)
        elif kind == 1:
            img = np.cumsum(rng.integers(0, 3, (H, W)), axis=1).astype(np.uint8)
        elif kind == 2:
            img = np.full((H, W), rng.integers(0, 256), np.uint8)
            img[rng.integers(0, H, 5), :] = rng.integers(0, 256, (5, W), dtype=np.uint8)
        else:
            img = np.tile(rng.integers(0, 256, (1, W), dtype=np.uint8), (H, 1))
        filt = [int(f) for f in rng.integers(0, 5, H)]
        files.append(_png(img, filt, int(rng.integers(0, 10)), strategies[k % len(strategies)]))
        imgs.append(img)
    out, codes, bad = _decode_gpu(ctx, files, H, W)
    assert bad == 0, codes
    for i, (o, e) in enumerate(zip(out, imgs)):
        np.testing.assert_array_equal(o, e, err_msg=f"file {i}")
    # corrupted copies
    bad_files, expect = [], []
    for i, f in enumerate(files):
        b = bytearray(f)
        s = b.index(b"IDAT") + 4 + 2  # past the zlib header of the first IDAT chunk
        for _ in range(1 + i % 3):
            b[s + int(rng.integers(0, min(200, len(b) - s - 20)))] ^= int(rng.integers(1, 256))
        bad_files.append(bytes(b))
        # zlib's raw inflate of the damaged stream (the IDAT payloads gathered; header and Adler trailer dropped)
        p, z = 8, b""
        while p < len(b):
            n = struct.unpack(">I", b[p:p + 4])[0]
            if b[p + 4:p + 8] == b"IDAT":
                z += bytes(b[p + 8:p + 8 + n])
            p += 12 + n
        ref = None
        try:
            d = zlib.decompressobj(-15)
            raw = d.decompress(z[2:]) + d.flush()
            if d.eof and len(raw) == H * (W + 1) and all(raw[r * (W + 1)] <= 4 for r in range(H)):
                ref = raw
        except zlib.error:
            ref = None
        expect.append(ref)
    out, codes, n_bad = _decode_gpu(ctx, bad_files, H, W)
    assert n_bad == len(bad_files) and all(c == PNG_ERR_CRC for c in codes), codes
    # the damaged streams again, in files whose chunk CRCs were recomputed: zlib's decode or its Adler-32 rejects every
    # one of them (checked here), and so does the GPU
    refiled = [_png_from_z(_zstream(b), H, W) for b in bad_files]
    for b in refiled:
        with pytest.raises(zlib.error):
            zlib.decompress(_zstream(b))
    out, codes, n_bad = _decode_gpu(ctx, refiled, H, W)
    assert n_bad == len(refiled) and all(c != 0 for c in codes), codes
    assert not out.any()
    for i, ref in enumerate(expect):
        if ref is not None:  # zlib's raw inflate yields valid rows: the GPU got past inflate and unfilter too
            assert codes[i] == PNG_ERR_ADLER, (i, codes[i])
    # with the checks off (libpng's PNG_CRC_QUIET_USE / PNG_IGNORE_ADLER32), the damaged streams' bytes themselves
    out, codes, _ = _decode_gpu(ctx, bad_files, H, W, checks=(0, 0))
    n_ok = 0
    for i, ref in enumerate(expect):
        if ref is None:
            continue
        n_ok += 1
        assert codes[i] == 0, (i, codes[i])
        # unfilter the reference rows on the host (png_decode_gray on a repaired file would recheck CRCs)
        rows = np.frombuffer(ref, np.uint8).reshape(H, W + 1)
        img = np.zeros((H, W), np.int32)
        for r in range(H):
            f, x = rows[r, 0], rows[r, 1:].astype(np.int32)
            up = img[r - 1] if r else np.zeros(W, np.int32)
            for c in range(W):
                a = img[r, c - 1] if c else 0
                bb = up[c]
                cc = up[c - 1] if c else 0
                if f == 0:
                    pred = 0
                elif f == 1:
                    pred = a
                elif f == 2:
                    pred = bb
                elif f == 3:
                    pred = (a + bb) >> 1
                else:
                    pp = a + bb - cc
                    pa, pb, pc = abs(pp - a), abs(pp - bb), abs(pp - cc)
                    pred = a if (pa <= pb and pa <= pc) else (bb if pb <= pc else cc)
                img[r, c] = (x[c] + pred) & 255
        np.testing.assert_array_equal(out[i], img.astype(np.uint8), err_msg=f"damaged file {i}")
    assert len(expect) == 24 and n_ok >= 5  # (11 of the 24 damaged streams still inflate in zlib)
