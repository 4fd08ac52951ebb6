"""CPU tests of the oracle's cv::calcOpticalFlowPyrLK restatement.  OpenCV is not in
this image and the reference holds no LK fixtures, so parity to the reference binary is unpinned: pyrDown and
Scharr are pinned by independent numpy restatements, LK by recovering known synthetic motion."""
import numpy as np
import pytest

from ya_vo_amd.synth import synth_frame


def _reflect(p, n):
    if n == 1:  # cv::borderInterpolate(REFLECT_101) on a length-1 axis
        return np.zeros_like(p)
    p = np.abs(p)
    return np.where(p >= n, 2 * n - p - 2, p)


def _np_pyr_down(img):
    H, W = img.shape
    w = np.array([1, 4, 6, 4, 1], np.int64)
    ys = np.arange((H + 1) // 2)
    xs = np.arange((W + 1) // 2)
    out = np.zeros((len(ys), len(xs)), np.int64)
    src = img.astype(np.int64)
    for i in range(5):
        rows = src[_reflect(2 * ys + i - 2, H)]
        for j in range(5):
            out += w[i] * w[j] * rows[:, _reflect(2 * xs + j - 2, W)]
    return ((out + 128) >> 8).astype(np.uint8)


def _np_scharr(img):
    H, W = img.shape
    s = img.astype(np.int64)
    up = s[_reflect(np.arange(H) - 1, H)]
    dn = s[_reflect(np.arange(H) + 1, H)]
    t0 = (up + dn) * 3 + s * 10
    t1 = dn - up
    xl, xr = _reflect(np.arange(W) - 1, W), _reflect(np.arange(W) + 1, W)
    dx = t0[:, xr] - t0[:, xl]
    dy = (t1[:, xr] + t1[:, xl]) * 3 + t1 * 10
    return np.stack([dx, dy], -1).astype(np.int16)


@pytest.mark.parametrize("shape", [(376, 1241), (47, 156), (13, 12), (1, 5)])
def test_pyr_down_matches_numpy(oracle, shape):
    img = synth_frame(3, 0, 0, max(shape[0], 1), shape[1]) if shape[0] > 1 else \
        np.random.default_rng(0).integers(0, 256, shape).astype(np.uint8)
    img = img[:shape[0], :shape[1]]
    np.testing.assert_array_equal(oracle.pyr_down(img), _np_pyr_down(img))


@pytest.mark.parametrize("shape", [(376, 1241), (20, 33)])
def test_scharr_matches_numpy(oracle, shape):
    img = synth_frame(4, 0, 0, shape[0], shape[1])
    np.testing.assert_array_equal(oracle.scharr(img), _np_scharr(img))


def test_lk_recovers_motion(oracle):
    """Frame k+1 is frame k shifted by (-1 row, -3 cols): LK from k to k+1 moves every tracked point by
    (dx, dy) = (-3, -1), sub-pixel accurate; both sum orders agree to float rounding."""
    prev, nxt = synth_frame(11, 0, 0), synth_frame(11, 1, 3)
    rng = np.random.default_rng(0)
    pts = np.stack([rng.integers(20, 1220, 400), rng.integers(20, 356, 400)], 1).astype(np.float32)
    p0, st0, e0, lv = oracle.lk(prev, nxt, pts, sum_mode=0)
    assert lv == 3
    assert st0.mean() > 0.95
    d = p0[st0] - pts[st0]
    np.testing.assert_allclose(np.median(d, 0), [-3.0, -1.0], atol=0.02)
    assert np.mean(np.abs(d - [-3.0, -1.0]).max(1) < 0.1) > 0.9
    p1, st1, e1, _ = oracle.lk(prev, nxt, pts, sum_mode=1)
    np.testing.assert_array_equal(st0, st1)
    np.testing.assert_allclose(p1, p0, atol=1e-3)
    # points pushed off the image lose their status; out-of-range starts are rejected at level 0
    far = np.array([[-30.0, 10.0], [1300.0, 100.0]], np.float32)
    _, stf, ef, _ = oracle.lk(prev, nxt, far)
    assert not stf.any() and np.all(ef == 0)
