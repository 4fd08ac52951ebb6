"""CPU tests of the oracle's geometry rows against ground truth and independent
numpy / scipy restatements.  The reference's own tests hold no assertions for these rows
(tests/3DHandlerTest.cc, tests/OptimizerTest.cc only print), so parity to the reference binary is unpinned;
these tests pin the restated algorithms to their published mathematics."""
import numpy as np
import pytest
import scipy.linalg

from ya_vo_amd import MATCH_DTYPE
from ya_vo_amd import scene


def test_cv_svd_reconstructs(oracle):
    rng = np.random.default_rng(0)
    for n in (3, 9):
        for _ in range(20):
            A = rng.normal(size=(n, n))
            if n == 9:
                A = A.T @ A  # the F-RANSAC use: A^T A
            w, u, vt = oracle.cv_svd(A)
            assert np.all(np.diff(w) <= 0)
            np.testing.assert_allclose(u @ np.diag(w) @ vt, A, atol=1e-10 * np.abs(A).max())
            np.testing.assert_allclose(vt @ vt.T, np.eye(n), atol=1e-12)
            np.testing.assert_allclose(w, np.linalg.svd(A, compute_uv=False), rtol=1e-10, atol=1e-12)


def _np_fundamental(pts):
    """Independent normalised 8-point in numpy, same conventions as src/3DHandler.cc:50-142."""
    x1, y1, x2, y2 = pts.T

    def N(x, y):
        mx, my = x.mean(), y.mean()
        s = np.sqrt(2.0) / np.mean(np.sqrt((x - mx) ** 2 + (y - my) ** 2))
        return np.array([[s, 0, -s * mx], [0, s, -s * my], [0, 0, 1.0]])

    N1, N2 = N(x1, y1), N(x2, y2)
    p1 = (N1 @ np.stack([x1, y1, np.ones_like(x1)])).T
    p2 = (N2 @ np.stack([x2, y2, np.ones_like(x2)])).T
    A = np.stack([p1[:, 0] * p2[:, 0], p1[:, 0] * p2[:, 1], p1[:, 0], p1[:, 1] * p2[:, 0], p1[:, 1] * p2[:, 1],
                  p1[:, 1], p2[:, 0], p2[:, 1], np.ones(len(p1))], 1)
    _, _, vt = np.linalg.svd(A.T @ A)
    F = vt[8].reshape(3, 3)
    u, w, vt3 = np.linalg.svd(F)
    w[2] = 0
    F = N2.T @ (u @ np.diag(w) @ vt3) @ N1
    return F / F[2, 2]


def _match_array(ua, ub):
    m = np.zeros(len(ua), MATCH_DTYPE)
    m["pt1"]["x"] = np.round(ua[:, 0])
    m["pt1"]["y"] = np.round(ua[:, 1])
    m["pt2"]["x"] = np.round(ub[:, 0])
    m["pt2"]["y"] = np.round(ub[:, 1])
    return m


def test_fundamental_8pt_matches_numpy(oracle):
    Ta, Tb, X, ua, ub = scene.two_view_matches(60, seed=1)
    pts = np.concatenate([ua, ub], 1)
    for s in range(5):
        sel = np.random.default_rng(s).choice(len(pts), 8, replace=False)
        ok, F = oracle.fundamental(pts[sel])
        assert ok
        Fn = _np_fundamental(pts[sel])
        np.testing.assert_allclose(F, Fn, rtol=1e-6, atol=1e-9)
        assert F[2, 2] == 1.0 or abs(F[2, 2] - 1.0) < 1e-15
        # the reference's design row [x1x2, x1y2, x1, y1x2, y1y2, y1, x2, y2, 1] (src/3DHandler.cc:108-116)
        # solves p1^T F p2 = 0 while the denormalisation (N2^T F N1) and the inlier test (p2^T F p1) assume
        # the other order; that mismatch is kept literally, so exact data does NOT
        # give a zero epipolar error here -- only agreement with the numpy restatement is asserted.
    ok, _ = oracle.fundamental(pts[:7])
    assert not ok


def test_f_ransac(oracle):
    Ta, Tb, X, ua, ub = scene.two_view_matches(200, seed=2)
    m = _match_array(ua, ub)
    rng = np.random.default_rng(3)
    samples = rng.integers(0, len(m), (400, 8))
    ok, F, inl = oracle.f_ransac(m, samples, 0.1)
    assert ok and 0 < inl <= len(m)
    # the winner is the first hypothesis reaching the maximum (strict >)
    counts = []
    for s in samples:
        pts = np.stack([m["pt1"]["x"], m["pt1"]["y"], m["pt2"]["x"], m["pt2"]["y"]], 1).astype(np.float64)
        _, Fh = oracle.fundamental(pts[s])
        e = (pts[:, 2] * Fh[0, 0] + pts[:, 3] * Fh[1, 0] + Fh[2, 0]) * pts[:, 0] + \
            (pts[:, 2] * Fh[0, 1] + pts[:, 3] * Fh[1, 1] + Fh[2, 1]) * pts[:, 1] + \
            (pts[:, 2] * Fh[0, 2] + pts[:, 3] * Fh[1, 2] + Fh[2, 2])
        counts.append(int(np.sum(np.abs(e) < 0.1)))
    assert inl == max(counts)
    ok, _, _ = oracle.f_ransac(m[:7], samples, 0.1)
    assert not ok


def test_eigen_svd_4x4(oracle):
    rng = np.random.default_rng(4)
    for _ in range(50):
        A = rng.normal(size=(4, 4))
        ok, sv, V = oracle.eigen_svd(A)
        assert ok
        np.testing.assert_allclose(sv, np.linalg.svd(A, compute_uv=False), rtol=1e-12)
        np.testing.assert_allclose(V.T @ V, np.eye(4), atol=1e-13)
        np.testing.assert_allclose(np.linalg.norm(A @ V, axis=0), sv, rtol=1e-12)


def test_triangulation_recovers_points(oracle):
    Ta, Tb, X, ua, ub = scene.two_view_matches(100, seed=5)
    K = scene.K_KITTI
    # the reference feeds (row, col) into pixel2camera as (x - cx)/fx: build matches so that
    # pixel2camera returns the true normalised coordinates (integer pixels as KeyPoint holds them)
    m = _match_array(ua, ub)
    n, Xw, ok = oracle.triangulate_matches(Ta, Tb, K, m)
    # with integer-rounded pixels the DLT is approximate: depth error small relative to depth
    assert n >= 95
    rel = np.linalg.norm(Xw[ok] - X[ok], axis=1) / np.linalg.norm(X[ok], axis=1)
    assert np.median(rel) < 0.05


def _twist_expm(a):
    rho, om = a[:3], a[3:]
    M = np.zeros((4, 4))
    M[:3, :3] = [[0, -om[2], om[1]], [om[2], 0, -om[0]], [-om[1], om[0], 0]]
    M[:3, 3] = rho
    return scipy.linalg.expm(M)


def test_se3_exp_mul_act(oracle):
    rng = np.random.default_rng(6)
    for _ in range(50):
        a = rng.normal(scale=0.3, size=6)
        T = oracle.se3_exp(a)
        E = _twist_expm(a)
        np.testing.assert_allclose(oracle.quat_to_R(T[:4]), E[:3, :3], atol=1e-12)
        np.testing.assert_allclose(T[4:], E[:3, 3], atol=1e-12)
        B = oracle.se3_exp(rng.normal(scale=0.3, size=6))
        C = oracle.se3_mul(T, B)
        EB = _twist_expm(np.zeros(6))
        RB, tB = oracle.quat_to_R(B[:4]), B[4:]
        np.testing.assert_allclose(oracle.quat_to_R(C[:4]), E[:3, :3] @ RB, atol=1e-12)
        np.testing.assert_allclose(C[4:], E[:3, :3] @ tB + E[:3, 3], atol=1e-12)
        p = rng.normal(size=3)
        np.testing.assert_allclose(oracle.se3_act(T, p), E[:3, :3] @ p + E[:3, 3], atol=1e-12)
    # tiny rotations take the Taylor branch (theta^2 < 1e-20)
    T = oracle.se3_exp(np.array([0.1, 0.2, 0.3, 1e-12, 0, 0]))
    np.testing.assert_allclose(T[4:], [0.1, 0.2, 0.3], atol=1e-12)
    for x in np.linspace(-0.78, 0.78, 101):
        assert abs(oracle.lib.or_ksin(x) - np.sin(x)) <= 2.3e-16 and abs(oracle.lib.or_kcos(x) - np.cos(x)) <= 2.3e-16


def test_world2camera(oracle):
    X, uv, T, _ = scene.random_scene(20, seed=7)
    out = oracle.world2camera(X, T, scene.K_KITTI)
    ref = (scene.K_KITTI @ scene.transform(T, X).T).T
    np.testing.assert_allclose(out, ref, rtol=1e-12)
    np.testing.assert_allclose(out[:, :2] / out[:, 2:], uv, rtol=1e-10)


def test_ldlt6(oracle):
    rng = np.random.default_rng(8)
    for variant in (0, 1):
        for _ in range(30):
            J = rng.normal(size=(20, 6))
            H = J.T @ J + 1e-3 * np.eye(6)
            b = rng.normal(size=6)
            pos, x = oracle.ldlt6(H, b, variant)
            assert pos
            np.testing.assert_allclose(x, np.linalg.solve(H, b), rtol=1e-9)
        pos, _ = oracle.ldlt6(-np.eye(6), np.ones(6), variant)
        assert not pos


@pytest.mark.parametrize("sum_mode", [0, 1, 2, 3, 4, 5, 6, 7])
def test_pose_lm_noise_free(oracle, sum_mode):
    X, uv, T_true, _ = scene.random_scene(300, seed=9)
    prior = scene.perturb(T_true, np.random.default_rng(1))
    T, outl, inl = oracle.pose_lm(X, uv, scene.K_KITTI, prior, sum_mode)
    assert inl == 300 and not outl.any()
    np.testing.assert_allclose(scene.project(T, X), uv, atol=1e-6)


@pytest.mark.parametrize("order", [3, 4, 5, 6, 7])
def test_pose_lm_outliers_and_sum_orders(oracle, order):
    X, uv, T_true, gross = scene.random_scene(800, seed=10, noise_px=0.5, outlier_frac=0.1)
    prior = scene.perturb(T_true, np.random.default_rng(2))
    T0, out0, inl0 = oracle.pose_lm(X, uv, scene.K_KITTI, prior, 0)
    T1, out1, inl1 = oracle.pose_lm(X, uv, scene.K_KITTI, prior, order)
    assert np.all(out0[gross])               # every gross outlier (>= 20 px) is flagged
    assert inl0 >= 800 - int(0.1 * 800) - 40  # chi2 > 5.991 also flags some 0.5-px noise tails
    np.testing.assert_array_equal(out0, out1)
    assert inl0 == inl1
    np.testing.assert_allclose(T0, T1, rtol=0, atol=1e-10)
    assert np.linalg.norm(T0[4:] - T_true[4:]) < 0.05


def test_pose_lm_degenerate(oracle):
    X, uv, T_true, _ = scene.random_scene(10, seed=11)
    prior = scene.perturb(T_true, np.random.default_rng(3))
    T, outl, inl = oracle.pose_lm(X[:0], uv[:0], scene.K_KITTI, prior)
    assert inl == 0 and np.array_equal(T, prior)  # no edges: the prior is returned


@pytest.mark.parametrize("sum_mode", [0, 1])
def test_pose_gn(oracle, sum_mode):
    K = scene.K_KITTI
    X, uv, T_true, _ = scene.random_scene(100, seed=12)
    # test.cc's GN projects with cx, cy like the LM edge: identical measurements
    prior = scene.perturb(T_true, np.random.default_rng(4), rot=0.01, trans=0.05)
    T, it = oracle.pose_gn(X, uv, K, prior, sum_mode)
    assert it >= 2
    np.testing.assert_allclose(scene.project(T, X), uv, atol=1e-5)


def test_track_chain_recovers_synthetic_motion(oracle, offsets):
    """The CPU track chain (tests/track_chain.py) on a synthetic stereo pair of frames recovers the known
    motion: frame k-1 is frame k shifted by (+1 row, +3 cols), disparity 8 px at baseline 0.54 m."""
    from ya_vo_amd.synth import synth_frame
    from track_chain import track_pose
    imgs = [synth_frame(77, 0, 0), synth_frame(77, 1, 3), synth_frame(77, 1, 11)]
    kp = [oracle.brief(im, oracle.fast(im, 2000)[0], offsets) for im in imgs]
    T_right = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
    X, uv, q, T, out, inl = track_pose(oracle, kp[0], kp[1], kp[2], scene.K_KITTI, T_right)
    assert len(X) > 500 and inl > 0.8 * len(X)
    np.testing.assert_allclose(X[:, 2], 0.54 * scene.K_KITTI[1, 1] / 8, rtol=1e-6)
    np.testing.assert_allclose(T[4:], [0.0675, 0.2025, 0.0], atol=2e-3)
