"""CPU tests: pin the oracle's FAST / Harris / top-K restatement against the reference's own fixtures
(tests/FastDetectorTest.cc, tests/ImageTest.cc, tests/testBresenham.png) and against an independent numpy
restatement.  No GPU needed."""
import json
import os
import re

import numpy as np
import pytest

from ya_vo_amd.synth import synth_frame

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# ring order derived from src/FastDetector.cc:50-112
RING_ORDER = [(0, -3), (1, -3), (2, -2), (3, -1), (3, 0), (3, 1), (2, 2), (1, 3),
              (0, 3), (-1, 3), (-2, 2), (-3, 1), (-3, 0), (-3, -1), (-2, -2), (-1, -3)]


def _fixture_pixels():
    d = json.load(open(os.path.join(GOLDEN, "testBresenham_pixels.json")))
    return {tuple(p) for p in d["pixels"]}


def test_ring_matches_reference_fixture(oracle):
    # FastDetectorTest.BresenhamCircleCheck (tests/FastDetectorTest.cc:6-31): 16 points that, drawn at
    # (25, 25), reproduce testBresenham.png (the PNG also has the centre set).
    ring = oracle.ring(25, 25)
    assert ring.shape == (16, 2)
    pts = {(int(r), int(c)) for r, c in ring}
    assert len(pts) == 16
    fixture = _fixture_pixels() - {(25, 25)}
    # putPixel uses cv::Point(x=row, y=col) -> at(y, x): the drawing is transposed; the ring is symmetric
    assert pts == fixture
    assert {(c, r) for r, c in pts} == fixture


def test_ring_order_literal(oracle):
    ring = oracle.ring(0, 0)
    assert [tuple(map(int, p)) for p in ring] == RING_ORDER
    # the pretest reads indices 0, 7, 4, 12 (src/FastDetector.cc:304-307)
    assert [tuple(map(int, ring[i])) for i in (0, 7, 4, 12)] == [(0, -3), (1, 3), (3, 0), (-3, 0)]


def test_ring_stl_containers_build_the_same_ring(oracle):
    """The literal CPU baseline rebuilds the ring per pixel with the reference's std::vector / std::set containers
    (or_bresenham_ring_stl): the same 16 points in the same order, at any centre."""
    for xc, yc in [(0, 0), (25, 25), (4, 1236), (371, 4), (187, 600)]:
        np.testing.assert_array_equal(oracle.ring(xc, yc, stl=True), oracle.ring(xc, yc))


def test_ring_table_in_kernel_matches_oracle(oracle):
    src = open(os.path.join(ROOT, "ya_vo_amd", "csrc", "yavo_kernels.hip")).read()
    dr = [int(v) for v in re.search(r"#define YV_RING_DR \{([^}]*)\}", src).group(1).split(",")]
    dc = [int(v) for v in re.search(r"#define YV_RING_DC \{([^}]*)\}", src).group(1).split(",")]
    assert list(zip(dr, dc)) == [tuple(map(int, p)) for p in oracle.ring(0, 0)]


def test_image_getpixel_ring(oracle):
    # ImageTest.GetPixelMethod (tests/ImageTest.cc:23-36): every ring pixel of the fixture reads 255
    img = np.zeros((50, 50), np.uint8)
    for r, c in _fixture_pixels():
        img[r, c] = 255
    for r, c in oracle.ring(25, 25):
        assert img[r, c] == 255


def test_contiguous_reference_cases(oracle):
    # FastDetector.CheckContiguosPixels (tests/FastDetectorTest.cc:38-61)
    img = np.zeros((50, 50), np.uint8)
    ring = oracle.ring(25, 25)
    for r, c in ring:
        img[c, r] = 255  # putPixel(cv::Point(x, y)) writes at(y, x)
    img_rc = img.T.copy()  # getPixelVal(x, y) = data[x*cols + y]: index as (x=row, y=col)
    assert oracle.check_contiguous(int(img_rc[25, 25]), ring, img_rc) is True
    img_rc[25, 25] = 255
    assert oracle.check_contiguous(int(img_rc[25, 25]), ring, img_rc) is False
    # FastDetector.CheckDiscontinuous (:64-80): only the first 11 ring pixels set -> false
    img2 = np.zeros((50, 50), np.uint8)
    for r, c in ring[:11]:
        img2[r, c] = 255
    assert oracle.check_contiguous(0, ring, img2) is False


def test_contiguous_no_wraparound(oracle):
    # runs are counted over indices 0..15 with no wrap: 6 at the end + 6 at the start is not 12
    ring = oracle.ring(10, 10)
    img = np.zeros((21, 21), np.uint8)
    for i in list(range(0, 6)) + list(range(10, 16)):
        r, c = ring[i]
        img[r, c] = 200
    assert oracle.check_contiguous(0, ring, img) is False
    for i in range(4, 16):
        r, c = ring[i]
        img[r, c] = 200
    assert oracle.check_contiguous(0, ring, img) is True


def test_threshold_is_strict_40(oracle):
    # checkInBetween: "similar" iff cent > p-40 && cent < p+40, i.e. |c - p| < 40
    ring = oracle.ring(10, 10)
    for delta, expect in ((39, False), (40, True)):
        img = np.full((21, 21), 100, np.uint8)
        for r, c in ring:
            img[r, c] = 100 + delta
        assert oracle.check_contiguous(100, ring, img) is expect


def _numpy_fast_candidates(img, thr=40):
    """Independent vectorised restatement of the candidate test (src/FastDetector.cc:298-320)."""
    H, W = img.shape
    im = img.astype(np.int32)
    cen = im[4:H - 4, 4:W - 4]
    diffs = []
    for dr, dc in RING_ORDER:
        p = im[4 + dr:H - 4 + dr, 4 + dc:W - 4 + dc]
        diffs.append(~((cen > p - thr) & (cen < p + thr)))
    d = np.stack(diffs)
    pre = d[0] & d[7] & (d[4] | d[12])
    run = np.zeros_like(cen)
    best = np.zeros_like(cen)
    for k in range(16):
        run = np.where(d[k], run + 1, 0)
        best = np.maximum(best, run)
    cand = pre & (best >= 12)
    rr, cc = np.nonzero(cand)
    return (rr + 4) * W + (cc + 4)


def _numpy_harris(img, idx):
    H, W = img.shape
    im = np.pad(img.astype(np.int64), 1)
    gx = np.zeros((H, W), np.int64)
    gy = np.zeros((H, W), np.int64)
    # 3x3 Sobel correlation centred at (r, c), zero border
    for k, wk in enumerate((1, 2, 1)):
        gx += wk * (im[k:k + H, 2:W + 2] - im[k:k + H, 0:W])
        gy += wk * (im[2:H + 2, k:k + W] - im[0:H, k:k + W])
    out = []
    for i in idx:
        r, c = divmod(int(i), W)
        sx = gx[r - 1:r + 2, c - 1:c + 2]
        sy = gy[r - 1:r + 2, c - 1:c + 2]
        m = np.array([[np.sum(sx * sx), np.sum(sx * sy)], [np.sum(sx * sy), np.sum(sy * sy)]], np.float64)
        ev = np.linalg.eigvalsh(m)
        out.append(ev[0] * ev[1] - 0.04 * (ev[0] + ev[1]) ** 2)
    return np.array(out)


@pytest.mark.parametrize("case", ["crop_epilines", "crop_epilinesOpencv", "synth"])
def test_candidates_match_numpy_restatement(oracle, case):
    if case == "synth":
        img = synth_frame(1234, 0, 0)
    else:
        img = np.load(os.path.join(GOLDEN, "kitti_crops.npz"))[case.replace("crop_", "")]
    rc, resp, nc, cidx, cresp = oracle.fast(img, 2000, with_candidates=True)
    ref = _numpy_fast_candidates(img)
    assert nc == len(ref)
    np.testing.assert_array_equal(np.sort(cidx), ref)
    # Harris responses: float32 Jacobi path vs a float64 closed form, relative agreement
    sel = cidx[:: max(1, len(cidx) // 200)]
    sresp = cresp[:: max(1, len(cidx) // 200)]
    h64 = _numpy_harris(img, sel)
    scale = np.maximum(np.abs(h64), 1e6)
    assert np.max(np.abs(sresp - h64) / scale) < 1e-4


def test_topk_order_is_canonical(oracle):
    img = synth_frame(99, 0, 0, 200, 300)
    rc, resp, nc, cidx, cresp = oracle.fast(img, 2000, with_candidates=True)
    W = img.shape[1]
    order = sorted(range(nc), key=lambda i: (-float(cresp[i]), int(cidx[i])))[:2000]
    np.testing.assert_array_equal(rc[:, 0] * W + rc[:, 1], cidx[order])
    np.testing.assert_array_equal(resp, cresp[order])
    assert np.all(np.diff(resp) <= 0)


def test_literal_and_efficient_modes_agree(oracle):
    # mode 0 keeps the reference's costs (per-pixel ring rebuild, whole-image products per corner)
    img = synth_frame(5, 10, 20, 48, 96)
    a = oracle.fast(img, 2000, mode=0)
    b = oracle.fast(img, 2000, mode=1)
    assert a[2] == b[2] and a[2] > 0
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_topk_cut_and_empty(oracle):
    img = synth_frame(3, 0, 0, 376, 1241)
    rc, resp, nc = oracle.fast(img, 2000)
    assert nc > 2000 and len(rc) == 2000
    rc5, resp5, _ = oracle.fast(img, 5)
    np.testing.assert_array_equal(rc5, rc[:5])
    flat = np.full((40, 40), 77, np.uint8)
    rc0, resp0, nc0 = oracle.fast(flat, 2000)
    assert nc0 == 0 and len(rc0) == 0


def test_eigen_jacobi_2x2(oracle):
    rng = np.random.default_rng(0)
    for _ in range(200):
        a, d = rng.integers(0, 9_000_000, 2).astype(np.float32)
        b = np.float32(rng.integers(-4_000_000, 4_000_000))
        w = oracle.eigen_jacobi(np.array([[a, b], [b, d]], np.float32))
        ref = np.linalg.eigvalsh(np.array([[a, b], [b, d]], np.float64))[::-1]
        assert w[0] >= w[1]
        np.testing.assert_allclose(w, ref, rtol=1e-5, atol=1.0)
    # |b| <= FLT_EPSILON: no rotation, sorted diagonal
    w = oracle.eigen_jacobi(np.array([[1.0, 0.0], [0.0, 5.0]], np.float32))
    np.testing.assert_array_equal(w, [5.0, 1.0])


@pytest.mark.parametrize("case", ["crop_epilines", "crop_epilinesOpencv", "synth_1234_f0", "synth_1234_f1"])
def test_fast_golden(oracle, case):
    g = np.load(os.path.join(GOLDEN, "fast_golden.npz"))
    if case.startswith("crop_"):
        img = np.load(os.path.join(GOLDEN, "kitti_crops.npz"))[case[5:]]
    else:
        k = int(case[-1])
        img = synth_frame(1234, k, 3 * k)
    rc, resp, nc = oracle.fast(img, 2000)
    assert nc == int(g[case + "__ncand"][0])
    np.testing.assert_array_equal(rc, g[case + "__rc"])
    np.testing.assert_array_equal(resp, g[case + "__resp"])


def test_calib_parse_reference_case(oracle):
    # UtilsCheck.stringParseCheck (tests/UtilsTest.cc:4-15)
    m, nv = oracle.parse_calib("P0: 7.1 8.2 8.3 9.3 10.3 11 12 13 14 15 16 17 18 19 20 21")
    assert nv == 16
    assert m[0, 0] == 7.1 and m[0, 2] == 8.3 and m[1, 2] == 12 and m[3, 3] == 21


def test_calib_kitti00_fixture(oracle):
    # UtilsCheck.checkInstrinsicIntegrity (tests/UtilsTest.cc:18-29) on the committed tests/calib.txt
    lines = open(os.path.join(GOLDEN, "calib_kitti00.txt")).read().splitlines()
    left, nv = oracle.parse_calib(lines[0])
    right, _ = oracle.parse_calib(lines[1])
    assert nv == 12  # KITTI rows hold 12 values; the reference reads 16 (out of bounds), 0 here
    assert abs(left[0, 0] - 718.856) < 1 and abs(right[0, 0] - 718.856) < 1
    assert abs(left[1, 2] - 185.216) < 1 and abs(right[1, 2] - 185.216) < 1


def test_eigen_selfadjoint_flavour(oracle):
    """HAVE_EIGEN's cv::eigen restatement (Eigen 3.4 SelfAdjointEigenSolver<MatrixXf>): eigenvalues of integer
    structure tensors within float rounding of the exact ones, descending; diagonal and zero tensors exact."""
    rng = np.random.default_rng(11)
    for _ in range(2000):
        a, d = float(rng.integers(0, 2 ** 22)), float(rng.integers(0, 2 ** 22))
        b = float(rng.integers(-2 ** 21, 2 ** 21)) if rng.random() > 0.1 else 0.0
        w = oracle.eigen_selfadjoint2(a, b, d)
        ref = np.linalg.eigvalsh(np.array([[a, b], [b, d]]))[::-1]
        assert w[0] >= w[1]
        np.testing.assert_allclose(w, ref, rtol=0, atol=4e-7 * max(abs(ref).max(), 1.0))
    np.testing.assert_array_equal(oracle.eigen_selfadjoint2(5.0, 0.0, 9.0), [9.0, 5.0])
    np.testing.assert_array_equal(oracle.eigen_selfadjoint2(0.0, 0.0, 0.0), [0.0, 0.0])


def test_eigen_flavours_keep_the_candidate_set(oracle):
    """The flavour moves response bits, never the FAST candidate set (an integer test)."""
    from ya_vo_amd.synth import synth_frame
    img = synth_frame(3, 0, 0, 160, 400)
    out = []
    for fl in (0, 1):
        oracle.set_harris_eigen(fl)
        out.append(oracle.fast(img, 100000, with_candidates=True))
    oracle.set_harris_eigen(0)
    np.testing.assert_array_equal(np.sort(out[0][3]), np.sort(out[1][3]))
    assert out[0][2] == out[1][2]


def test_std_sort_diagnostic_matches_canonical_without_ties(oracle):
    """libstdc++ std::sort of the reference's comparator agrees with the canonical order when responses are
    distinct, and keeps a tie group's members (in some order) when they are not."""
    rng = np.random.default_rng(5)
    idx = np.arange(3000, dtype=np.int32)
    resp = rng.permutation(3000).astype(np.float32)
    cut = oracle.std_sort_cut(idx, resp, 100, 2000)
    np.testing.assert_array_equal(cut, np.argsort(-resp, kind="stable")[:2000])
    resp[:50] = 7.0e6  # a tie group above every other response
    cut = oracle.std_sort_cut(idx, resp, 100, 2000)
    assert set(cut[:50].tolist()) == set(range(50))
