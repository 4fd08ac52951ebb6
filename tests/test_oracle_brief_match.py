"""CPU tests: the oracle's blur / BRIEF / Hamming match / removeOutliers restatement against independent
numpy restatements, the reference's documented semantics and the committed golden fixtures."""
import os

import numpy as np
import pytest

from ya_vo_amd import KEYPOINT_DTYPE, MATCH_DTYPE, DEFAULT_BLUR_KERNEL
from ya_vo_amd.synth import synth_frame

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_gaussian_kernel_opencv_bitexact(oracle):
    # OpenCV getGaussianKernelFixedPoint_ED for ksize 9, sigma 2.5 (error diffusion) / plain rounding
    np.testing.assert_array_equal(oracle.gauss_kernel(9, 2.5, True), [12, 22, 31, 41, 44, 41, 31, 22, 12])
    np.testing.assert_array_equal(oracle.gauss_kernel(9, 2.5, False), [12, 21, 32, 41, 44, 41, 32, 21, 12])
    np.testing.assert_array_equal(DEFAULT_BLUR_KERNEL, oracle.gauss_kernel(9, 2.5, True))
    for n, s in ((3, 0.8), (5, 1.1), (7, 1.5), (9, 2.5), (11, 3.0)):
        assert int(oracle.gauss_kernel(n, s, True).sum()) == 256


def _numpy_blur(img, k):
    H, W = img.shape
    n = len(k)
    h = n // 2
    pad = np.pad(img.astype(np.int64), h, mode="reflect")  # numpy "reflect" == BORDER_REFLECT_101
    hz = sum(int(k[j]) * pad[:, j:j + W] for j in range(n))
    v = sum(int(k[i]) * hz[i:i + H, :] for i in range(n))
    return np.minimum((v + (1 << 15)) >> 16, 255).astype(np.uint8)


@pytest.mark.parametrize("shape", [(376, 1241), (9, 9), (17, 33)])
def test_blur_matches_numpy(oracle, shape):
    img = np.random.default_rng(1).integers(0, 256, shape).astype(np.uint8)
    np.testing.assert_array_equal(oracle.blur(img), _numpy_blur(img, DEFAULT_BLUR_KERNEL))


def test_offsets_restatement_matches_libstdcxx(oracle, offsets):
    # brief_offsets_mt19937_42.bin was produced by tests/golden/gen/gen_brief_offsets.cc with g++ 11
    np.testing.assert_array_equal(oracle.brief_offsets(42), offsets)
    assert offsets.min() >= -8 and offsets.max() <= 8


def _numpy_brief(img, rc, offsets):
    blur = _numpy_blur(img, DEFAULT_BLUR_KERNEL).reshape(-1)
    H, W = img.shape
    out = []
    for i, (r, c) in enumerate(rc):
        if c - 8 < 0 or c + 8 > W or r - 8 < 0 or r + 8 > H:
            continue
        bits = np.zeros(256, np.uint8)
        for j, (a, b, cc, d) in enumerate(offsets):
            i1 = (r + a) * W + (c + b)
            i2 = (r + cc) * W + (c + d)
            p1 = blur[i1] if 0 <= i1 < H * W else 0
            p2 = blur[i2] if 0 <= i2 < H * W else 0
            bits[j] = 1 if p1 > p2 else 0
        out.append((r, c, i, np.packbits(bits, bitorder="little")))
    return out


def test_brief_matches_numpy(oracle, offsets):
    img = synth_frame(11, 0, 0, 60, 90)
    H, W = img.shape
    rc = np.array([[8, 8], [H - 8, W - 8], [30, 45], [7, 20], [20, W - 7], [H - 8, 40], [52, W - 8]], np.int32)
    got = oracle.brief(img, rc, offsets)
    ref = _numpy_brief(img, rc, offsets)
    assert len(got) == len(ref) == 5
    for g, (r, c, i, fv) in zip(got, ref):
        assert (g["x"], g["y"], g["id"], g["matched"]) == (r, c, i, 0)
        np.testing.assert_array_equal(g["featVec"], fv)
        assert not g["_pad"].any()


def _kp(n, rng, bits=None):
    k = np.zeros(n, KEYPOINT_DTYPE)
    k["x"] = rng.integers(0, 376, n)
    k["y"] = rng.integers(0, 1241, n)
    k["id"] = np.arange(n)
    k["featVec"] = rng.integers(0, 256, (n, 32)) if bits is None else bits
    return k


def test_hamming_literal_popcount(oracle):
    rng = np.random.default_rng(2)
    for _ in range(50):
        a = rng.integers(0, 256, 32).astype(np.uint8)
        b = rng.integers(0, 256, 32).astype(np.uint8)
        assert oracle.hamming(a, b) == int(np.unpackbits(a ^ b).sum())


def test_match_first_minimum_wins(oracle):
    rng = np.random.default_rng(3)
    q = _kp(3, rng)
    t = _kp(6, rng)
    # train 1, 3 and 5 are all at distance 0 from query 0: the first (1) must win
    for j in (1, 3, 5):
        t["featVec"][j] = q["featVec"][0]
    m = oracle.match(q, t)
    assert m[0]["distance"] == 0 and m[0]["pt2"]["id"] == 1
    assert m[0]["pt2"]["x"] == t[1]["x"] and m[0]["pt2"]["y"] == t[1]["y"]
    assert not m[0]["pt2"]["featVec"].any() and m[0]["pt2"]["matched"] == 0
    np.testing.assert_array_equal(m["pt1"], q)


def test_match_empty_train(oracle):
    rng = np.random.default_rng(4)
    q = _kp(4, rng)
    m = oracle.match(q, np.zeros(0, KEYPOINT_DTYPE))
    assert np.all(m["distance"] == 2**31 - 1)
    assert np.all(m["pt2"]["x"] == 0) and np.all(m["pt2"]["id"] == 0)


def test_remove_outliers_semantics(oracle):
    m = np.zeros(6, MATCH_DTYPE)
    m["distance"] = [30, 12, 25, 50, 23, 24]
    m["pt1"]["id"] = np.arange(6)
    f = oracle.remove_outliers(m, 20)  # min 12 -> limit max(24, 20) = 24 -> keep d < 24
    assert list(f["distance"]) == [12, 23]
    assert np.all(f["pt1"]["matched"] == 1) and np.all(f["pt2"]["matched"] == 1)
    m["distance"] = [5, 9, 19, 20, 21, 7]  # min 5 -> limit max(10, 20) = 20
    assert list(oracle.remove_outliers(m, 20)["distance"]) == [5, 9, 19, 7]
    m["distance"] = 2**31 - 1  # 2*INT_MAX wraps to -2 in the reference -> limit 20 -> nothing kept
    assert len(oracle.remove_outliers(m, 20)) == 0
    assert len(oracle.remove_outliers(m[:0], 20)) == 0


def test_brief_golden(oracle, offsets):
    g = np.load(os.path.join(GOLDEN, "brief_golden.npz"))
    fg = np.load(os.path.join(GOLDEN, "fast_golden.npz"))
    crops = np.load(os.path.join(GOLDEN, "kitti_crops.npz"))
    for name in ("crop_epilines", "crop_epilinesOpencv"):
        k = oracle.brief(crops[name[5:]], fg[name + "__rc"], offsets)
        np.testing.assert_array_equal(k, g[name])


def test_match_golden(oracle):
    g = np.load(os.path.join(GOLDEN, "match_golden.npz"))
    b = np.load(os.path.join(GOLDEN, "brief_golden.npz"))
    m = oracle.match(b["synth_1234_f0"], b["synth_1234_f1"])
    np.testing.assert_array_equal(m, g["matches"])
    np.testing.assert_array_equal(oracle.remove_outliers(m, 20), g["filtered"])
