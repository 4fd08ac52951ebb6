"""Frame I/O and formats (include/yavo/yavo_io.h): cv::imread(path, 0) on PNG, the sorted KITTI
listing (getFilesInFolder, src/Utils.cc:31-36), calib.txt (getCalibParams / parseCalibString, src/Utils.cc:4-62),
the threaded host decode, and the KITTI pose format.  Fixtures: the reference's own PNGs (tests/epilines.png,
tests/testBresenham.png, copied under tests/golden/png/), its calib.txt (tests/golden/calib_kitti00.txt) and the
parseCalibString case of tests/UtilsTest.cc:4-15.  Expected pixels come from PIL (test infrastructure only) and from
an independent numpy restatement of the PNG filters / colour conversions."""
import os
import struct
import zlib

import numpy as np
import pytest
from PIL import Image

from ya_vo_amd import io as yio
from ya_vo_amd import YavoError

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _png(pixels, ctype, depth, filters=(0,), palette=None):
    """Minimal PNG encoder: rows of `pixels` (already packed per bit depth / channels) with cycling filters."""
    H = pixels.shape[0]
    W = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    ch = W
    width = pixels.shape[1] // ch if depth >= 8 else None
    rows = []
    bpp = max(1, ch * depth // 8)
    prev = None
    for y in range(H):
        raw = pixels[y].astype(np.uint16 if depth == 16 else np.uint8)
        if depth == 16:
            raw = raw.astype(">u2").view(np.uint8)
        raw = raw.astype(np.int32)
        f = filters[y % len(filters)]
        out = raw.copy()
        up = prev if prev is not None else np.zeros_like(raw)
        for i in range(len(raw)):
            a = raw[i - bpp] if i >= bpp else 0
            b = up[i]
            c = up[i - bpp] if i >= bpp else 0
            if f == 1:
                out[i] = raw[i] - a
            elif f == 2:
                out[i] = raw[i] - b
            elif f == 3:
                out[i] = raw[i] - ((a + b) >> 1)
            elif f == 4:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                pred = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                out[i] = raw[i] - pred
        rows.append(bytes([f]) + bytes((out & 0xFF).astype(np.uint8)))
        prev = raw
    data = zlib.compress(b"".join(rows))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    if width is None:
        width = pixels.shape[1] * 8 // depth
    ihdr = struct.pack(">IIBBBBB", width, H, depth, ctype, 0, 0, 0)
    out = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr)
    if palette is not None:
        out += chunk(b"PLTE", bytes(palette.astype(np.uint8).reshape(-1)))
    return out + chunk(b"IDAT", data) + chunk(b"IEND", b"")


def _gray_from_rgb(r, g, b):
    r, g, b = (x.astype(np.int64) for x in (r, g, b))
    v = (9797 * r + 19234 * g + 3737 * b) >> 15
    return np.where((r == g) & (r == b), r, v).astype(np.uint8)


REF_EPILINES = "/root/reference/tests/epilines.png"  # the full KITTI frame (CC BY-NC-SA): read in place, not copied


@pytest.mark.parametrize("name", ["epilines_crop.png", "testBresenham.png"])
def test_reference_pngs_match_pil(name):
    """testBresenham.png is the reference's own fixture; epilines_crop.png is a 256 x 128 crop of its KITTI frame
    (tests/epilines.png) re-encoded by PIL with adaptive filters (only crops are committed)."""
    path = os.path.join(GOLDEN, "png", name)
    got = yio.imread_gray(path)
    ref = np.array(Image.open(path).convert("L"))  # grey / black-and-white: every grey rule agrees
    np.testing.assert_array_equal(got, ref)


@pytest.mark.skipif(not os.path.exists(REF_EPILINES), reason="the reference checkout is not on this host")
def test_reference_kitti_png_matches_pil_and_crops():
    """The reference's own KITTI frame, decoded where it lies (the build container holds the reference)."""
    got = yio.imread_gray(REF_EPILINES)
    np.testing.assert_array_equal(got, np.array(Image.open(REF_EPILINES).convert("L")))
    np.testing.assert_array_equal(got[100:228, 400:656], yio.imread_gray(os.path.join(GOLDEN, "png",
                                                                                       "epilines_crop.png")))
    crops = np.load(os.path.join(GOLDEN, "kitti_crops.npz"))
    c = crops["epilines"]
    h, w = c.shape
    assert any(np.array_equal(got[y:y + h, x:x + w], c) for y in range(0, got.shape[0] - h + 1)
               for x in range(0, got.shape[1] - w + 1, 1) if got[y, x] == c[0, 0])


@pytest.mark.parametrize("filters", [(0,), (1,), (2,), (3,), (4,), (0, 1, 2, 3, 4)])
def test_grey8_all_filters(filters):
    img = np.random.default_rng(len(filters)).integers(0, 256, (23, 37)).astype(np.uint8)
    np.testing.assert_array_equal(yio.png_decode_gray(_png(img, 0, 8, filters)), img)


def test_grey16_high_byte_and_low_depths():
    v = np.random.default_rng(1).integers(0, 65536, (9, 11)).astype(np.uint16)
    np.testing.assert_array_equal(yio.png_decode_gray(_png(v, 0, 16, (0, 4))), (v >> 8).astype(np.uint8))
    for d in (1, 2, 4):
        vals = np.random.default_rng(d).integers(0, 1 << d, (7, 16))
        packed = np.zeros((7, 16 * d // 8), np.uint8)
        per = 8 // d
        for x in range(16):
            packed[:, x // per] |= (vals[:, x] << (8 - d * (x % per + 1))).astype(np.uint8)
        got = yio.png_decode_gray(_png(packed, 0, d, (0, 1, 2)))
        np.testing.assert_array_equal(got, (vals * 255 // ((1 << d) - 1)).astype(np.uint8))


def test_colour_types_to_grey():
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (6, 10, 3)).astype(np.uint8)
    rgb[0, :3] = 77  # r == g == b passes through
    want = _gray_from_rgb(rgb[..., 0], rgb[..., 1], rgb[..., 2])
    np.testing.assert_array_equal(yio.png_decode_gray(_png(rgb.reshape(6, 30), 2, 8, (0, 1, 4))), want)
    rgba = np.concatenate([rgb, rng.integers(0, 256, (6, 10, 1)).astype(np.uint8)], -1)
    np.testing.assert_array_equal(yio.png_decode_gray(_png(rgba.reshape(6, 40), 6, 8, (2, 3))), want)
    ga = np.stack([rgb[..., 0], rgb[..., 1]], -1)
    np.testing.assert_array_equal(yio.png_decode_gray(_png(ga.reshape(6, 20), 4, 8, (4,))), rgb[..., 0])
    pal = rng.integers(0, 256, (16, 3))
    idx = rng.integers(0, 16, (6, 10)).astype(np.uint8)
    np.testing.assert_array_equal(yio.png_decode_gray(_png(idx, 3, 8, (0,), palette=pal)),
                                  _gray_from_rgb(pal[idx, 0], pal[idx, 1], pal[idx, 2]))


def test_png_rejects_garbage_and_interlace():
    with pytest.raises(YavoError):
        yio.png_decode_gray(b"not a png at all, definitely not" * 4)
    data = bytearray(_png(np.zeros((4, 4), np.uint8), 0, 8))
    data[28] = 1  # interlace method in IHDR (crc now wrong too: the decoder does not check CRCs)
    with pytest.raises(YavoError):
        yio.png_decode_gray(bytes(data))


def test_parse_calib_string_reference_case():
    # tests/UtilsTest.cc:4-15
    m = yio.parse_calib_string("P0: 7.1 8.2 8.3 9.3 10.3 11 12 13 14 15 16 17 18 19 20 21")
    assert m[0, 0] == 7.1 and m[0, 2] == 8.3 and m[1, 2] == 12 and m[3, 3] == 21


def _make_sequence(root, n, stereo, H=12, W=20):
    rng = np.random.default_rng(n)
    frames = rng.integers(0, 256, (n, 2, H, W)).astype(np.uint8)
    for side in range(2 if stereo else 1):
        d = os.path.join(root, f"image_{side}")
        os.makedirs(d)
        for k in reversed(range(n)):  # creation order must not matter
            with open(os.path.join(d, f"{k:06d}.png"), "wb") as f:
                f.write(_png(frames[k, side], 0, 8, (k % 5,)))
    with open(os.path.join(GOLDEN, "calib_kitti00.txt")) as src, open(os.path.join(root, "calib.txt"), "w") as dst:
        dst.write(src.read())
    return frames


@pytest.mark.parametrize("stereo", [False, True])
def test_sequence_listing_calib_and_read(tmp_path, stereo):
    frames = _make_sequence(str(tmp_path), 13, stereo)
    seq = yio.Sequence(str(tmp_path), stereo=stereo)
    assert len(seq) == 13 and (seq.H, seq.W) == (12, 20)
    assert [os.path.basename(seq.path(i)) for i in range(13)] == [f"{i:06d}.png" for i in range(13)]
    P0, P1, K0, K1 = seq.calib()
    assert K0[0, 0] == 718.856 and K0[0, 2] == 607.1928 and K0[1, 2] == 185.2157 and K0[2, 2] == 1
    assert P1[0, 3] == -386.1448 and np.all(P0[3] == 0)  # 12 values per line: row 3 reads as zeros
    got = seq.read(2, 9, threads=4)
    want = frames[2:11, :2 if stereo else 1].reshape(-1, 12, 20)
    np.testing.assert_array_equal(got, want)
    with pytest.raises(YavoError):
        seq.read(10, 5)
    seq.close()


def test_sequence_missing_dir(tmp_path):
    with pytest.raises(YavoError):
        yio.Sequence(str(tmp_path / "nope"))


def test_kitti_poses_roundtrip(tmp_path):
    rng = np.random.default_rng(3)
    q = rng.normal(size=(5, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    t = rng.normal(size=(5, 3)) * 10
    poses = np.c_[q, t]  # SE3d::data() of T_cw
    path = str(tmp_path / "poses.txt")
    yio.write_kitti_poses(path, poses)
    M = yio.read_kitti_poses(path)
    assert M.shape == (5, 3, 4)
    for k in range(5):
        x, y, z, w = q[k]
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        np.testing.assert_allclose(M[k, :, :3], R.T, atol=1e-12)
        np.testing.assert_allclose(M[k, :, 3], -R.T @ t[k], atol=1e-10)


def test_png_writer_round_trip(tmp_path):
    """yv_png_write_gray (the bench's and tools' sequence writer, cv::imwrite's format) round-trips through the
    decoder, PIL agrees, and odd sizes / strides take the same path."""
    from PIL import Image
    from ya_vo_amd.io import png_decode_gray, png_write_gray
    rng = np.random.default_rng(3)
    for H, W in [(376, 1241), (1, 1), (7, 13), (64, 3)]:
        img = rng.integers(0, 256, (H, W), dtype=np.uint8)
        p = str(tmp_path / f"w{H}x{W}.png")
        png_write_gray(p, img)
        np.testing.assert_array_equal(np.array(Image.open(p)), img)
        np.testing.assert_array_equal(png_decode_gray(open(p, "rb").read()), img)
