"""GPU parity of the pyramidal LK row (cv::calcOpticalFlowPyrLK) against the oracle's
restatement in the GPU window-sum order (sum_mode 1): tracked points, status and error bit for bit.  Against
OpenCV's own scalar order (sum_mode 0) the points agree within LK_TOL px (the float window sums round
differently)."""
import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd.synth import synth_frame

pytestmark = pytest.mark.gpu
LK_TOL = 1e-2  # px, GPU vs OpenCV's scalar summation order


def _d2h(ptr, shape, dtype):
    """Copy device memory at a raw pointer (already complete) into a new host array (hipMemcpy D2H)."""
    import ctypes
    out = np.empty(shape, dtype)
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(out.nbytes), 2)
    assert rc == 0, f"hipMemcpy {rc}"
    return out


def _pts(rng, n, H, W, margin=-20):
    return np.stack([rng.uniform(margin, W - 1 - margin, n), rng.uniform(margin, H - 1 - margin, n)], 1).astype(np.float32)


@pytest.mark.parametrize("H,W,win,seed", [(376, 1241, 11, 0), (120, 200, 11, 1), (40, 60, 7, 2), (376, 1241, 21, 3)])
def test_lk_matches_oracle(ctx, oracle, H, W, win, seed):
    prev, nxt = synth_frame(20 + seed, 0, 0, H, W), synth_frame(20 + seed, 1, 3, H, W)
    rng = np.random.default_rng(seed)
    pts = _pts(rng, 500, H, W)
    pts[:3] = [[-30, 5], [W + 40, 10], [5, H + 50]]  # rejected at level 0
    g, gs, ge = ctx.calc_optical_flow_pyr_lk(prev, nxt, pts, win=win)
    o, os_, oe, _ = oracle.lk(prev, nxt, pts, win=win, sum_mode=1)
    np.testing.assert_array_equal(gs, os_)
    np.testing.assert_array_equal(g, o)
    np.testing.assert_array_equal(ge, oe)
    r, rs, _, _ = oracle.lk(prev, nxt, pts, win=win, sum_mode=0)
    both = gs & rs
    assert np.mean(gs == rs) > 0.99
    np.testing.assert_allclose(g[both], r[both], atol=LK_TOL)


def test_lk_negative_fourth_weight(ctx, oracle):
    """Identical frames (zero flow, J sampled at I's positions) with level-0 fractions whose three rounded bilinear
    weights sum past 2^14, so the fourth is -1 (a = 0.49951171875, b = 2^-14 and a = 0.332763671875, b = 3 2^-16):
    the J interpolation must treat it as signed."""
    H, W = 376, 1241
    img = synth_frame(77, 0, 0, H, W)
    xs = np.arange(60, 1180, 37, dtype=np.float64)
    pts = np.concatenate([
        np.stack([xs + 5 + 0.49951171875, np.full_like(xs, 55 + 2.0 ** -14)], 1),
        np.stack([xs + 5 + 0.332763671875, np.full_like(xs, 201 + 3 * 2.0 ** -16)], 1)]).astype(np.float32)
    g, gs, ge = ctx.calc_optical_flow_pyr_lk(img, img, pts)
    o, os_, oe, _ = oracle.lk(img, img, pts, sum_mode=1)
    np.testing.assert_array_equal(gs, os_)
    np.testing.assert_array_equal(g, o)
    np.testing.assert_array_equal(ge, oe)


def test_lk_empty_and_tiny(ctx, oracle):
    """No points (nothing launched, empty outputs), and a 12 x 15 image with win 3 (one pyramid level) whose points
    sit on the corners and just outside: the border paths of the pyramid, the in-window derivatives and the footprints."""
    img = synth_frame(5, 0, 0, 12, 15)
    g, gs, ge = ctx.calc_optical_flow_pyr_lk(img, img, np.zeros((0, 2), np.float32))
    assert g.shape == (0, 2) and gs.shape == (0,) and ge.shape == (0,)
    nxt = synth_frame(5, 1, 1, 12, 15)
    pts = np.array([[0, 0], [14, 0], [0, 11], [14, 11], [7.25, 5.5], [-1.5, 3], [15.5, 6], [3, -0.75]], np.float32)
    for win in (3, 5):
        g, gs, ge = ctx.calc_optical_flow_pyr_lk(img, nxt, pts, win=win, max_level=2)
        o, os_, oe, _ = oracle.lk(img, nxt, pts, win=win, max_level=2, sum_mode=1)
        np.testing.assert_array_equal(gs, os_)
        np.testing.assert_array_equal(g, o)
        np.testing.assert_array_equal(ge, oe)


def test_lk_flat_image_fails_min_eig(ctx, oracle):
    flat = np.full((64, 80), 128, np.uint8)
    pts = np.array([[40.0, 30.0], [10.5, 12.25]], np.float32)
    g, gs, ge = ctx.calc_optical_flow_pyr_lk(flat, flat, pts)
    o, os_, oe, _ = oracle.lk(flat, flat, pts, sum_mode=1)
    assert not gs.any() and not os_.any()
    np.testing.assert_array_equal(g, o)


def test_lk_batch_pairs(ctx, oracle):
    """Several (prev, next) pairs with different point counts in one launch through yv_lk_build / track."""
    import torch
    H, W, n_img = 188, 300, 4
    imgs = np.stack([synth_frame(40, k, 2 * k, H, W) for k in range(n_img)])
    d_img = torch.from_numpy(imgs).to("cuda:0")
    pairs = np.array([[0, 1], [1, 2], [3, 2]], np.int32)
    counts = np.array([300, 17, 0], np.int32)
    stride = 320
    rng = np.random.default_rng(9)
    pts = np.zeros((len(pairs), stride, 2), np.float32)
    for p in range(len(pairs)):
        pts[p, :counts[p]] = _pts(rng, counts[p], H, W, margin=5)
    lk = yv.Lk(ctx, n_img, H, W)
    dev = "cuda:0"
    d_pairs, d_cnt = torch.from_numpy(pairs).to(dev), torch.from_numpy(counts).to(dev)
    d_pts = torch.from_numpy(pts).to(dev)
    d_next = torch.zeros_like(d_pts)
    d_st = torch.zeros((len(pairs), stride), dtype=torch.uint8, device=dev)
    d_err = torch.zeros((len(pairs), stride), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    lk.build(d_img.data_ptr(), n_img, W, H * W)
    lk.track(d_pairs.data_ptr(), len(pairs), d_pts.data_ptr(), d_cnt.data_ptr(), stride, d_next.data_ptr(),
             d_st.data_ptr(), d_err.data_ptr())
    ctx.sync()
    g, gs, ge = d_next.cpu().numpy(), d_st.cpu().numpy().astype(bool), d_err.cpu().numpy()
    for p, (a, b) in enumerate(pairs):
        n = counts[p]
        o, os_, oe, _ = oracle.lk(imgs[a], imgs[b], pts[p, :n], sum_mode=1)
        np.testing.assert_array_equal(gs[p, :n], os_)
        np.testing.assert_array_equal(g[p, :n], o)
        np.testing.assert_array_equal(ge[p, :n], oe)
    lk.close()


@pytest.mark.parametrize("H,W,stride,n_img,win", [(376, 1241, 1241, 2, 11), (376, 1241, 1299, 1, 11),
                                                   (121, 203, 205, 3, 3), (37, 61, 61, 2, 3), (9, 13, 14, 2, 3),
                                                   (64, 1, 1, 1, 3), (1, 40, 40, 1, 3)])
def test_lk_pyramid_and_derivatives_match_oracle(ctx, oracle, H, W, stride, n_img, win):
    """Every level's pyrDown image and Scharr derivatives (yv_lk_level) byte for byte against the oracle, on noise
    images with odd sizes and strides (the border columns and rows take the reflected path)."""
    import torch
    rng = np.random.default_rng(H * 7 + W)
    pitch = stride * H + 3
    flat = rng.integers(0, 256, pitch * n_img, dtype=np.uint8)
    d_flat = torch.from_numpy(flat).to("cuda:0")
    lk = yv.Lk(ctx, n_img, H, W, win=win)
    lk.build(d_flat.data_ptr(), n_img, stride, pitch)
    ctx.sync()
    torch.cuda.synchronize()
    for i in range(n_img):
        ref = np.lib.stride_tricks.as_strided(flat[i * pitch:], (H, W), (stride, 1)).copy()
        for lvl in range(lk.levels + 1):
            d_img, st, d_der, dst, h, w = lk.level(i, lvl)
            assert (h, w) == ref.shape
            if lvl > 0:
                got = _d2h(d_img, (h, st), np.uint8)[:, :w]
                np.testing.assert_array_equal(got, ref, err_msg=f"level {lvl} image {i}")
            np.testing.assert_array_equal(_d2h(d_der, (h, dst, 2), np.int16)[:, :w], oracle.scharr(ref),
                                          err_msg=f"derivatives level {lvl} image {i}")
            ref = oracle.pyr_down(ref)
    lk.close()


def test_lk_level_waits_for_a_build_on_another_stream(ctx, oracle):
    """yv_lk_build on a caller stream (as the batch's LK mode does), then yv_lk_level with no synchronisation in
    between: the level's derivatives must see the finished pyramid (it waits for the build's event)."""
    import torch
    H, W, n_img = 376, 1241, 6
    rng = np.random.default_rng(11)
    flat = rng.integers(0, 256, H * W * n_img, dtype=np.uint8)
    d_flat = torch.from_numpy(flat).to("cuda:0")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    lk = yv.Lk(ctx, n_img, H, W, win=11)
    lk.build(d_flat.data_ptr(), n_img, W, H * W, stream=side.cuda_stream)
    i = n_img - 1  # the last image's levels are written last
    ref = flat[i * H * W:(i + 1) * H * W].reshape(H, W)
    for lvl in range(lk.levels + 1):
        if lvl > 0:
            ref = oracle.pyr_down(ref)
    d_img, st, d_der, dst, h, w = lk.level(i, lk.levels)
    got = _d2h(d_der, (h, dst, 2), np.int16)[:, :w]
    np.testing.assert_array_equal(got, oracle.scharr(ref))
    lk.close()


def test_lk_host_calls_reuse_the_previous_next_image(ctx, oracle):
    """A tracking loop's consecutive calls (f0, f1), (f1, f2), ...: the host call finds f1 (and its pyramid) in the
    slot its previous call left it in and uploads only the new image.  Every call equals the oracle, also when the
    reused buffer's bytes change in place, when prev is not the previous next, and after a size change."""
    H, W = 120, 200
    frames = [synth_frame(31, k, 3 * k, H, W) for k in range(5)]
    rng = np.random.default_rng(4)
    pts = _pts(rng, 300, H, W)

    def check(a, b):
        g, gs, ge = ctx.calc_optical_flow_pyr_lk(a, b, pts)
        o, os_, oe, _ = oracle.lk(a, b, pts, sum_mode=1)
        np.testing.assert_array_equal(gs, os_)
        np.testing.assert_array_equal(g, o)
        np.testing.assert_array_equal(ge, oe)

    buf = frames[0].copy()
    check(buf, frames[1])
    check(frames[1], frames[2])          # prev == the previous next: reused
    check(frames[2].copy(), frames[3])   # equal bytes in another buffer: reused
    mod = frames[3].copy()
    mod[60, 100] ^= 0x55                 # one byte differs from the previous next: uploaded again
    check(mod, frames[4])
    check(frames[0], frames[1])          # not the previous next
    small = [synth_frame(32, k, k, 60, 90) for k in range(2)]
    g, gs, ge = ctx.calc_optical_flow_pyr_lk(small[0], small[1], pts[:50] * 0.4)
    o, os_, oe, _ = oracle.lk(small[0], small[1], pts[:50] * 0.4, sum_mode=1)
    np.testing.assert_array_equal(g, o)
    check(frames[1], frames[2])          # after a size change: nothing to reuse
    check(frames[2], frames[3])
