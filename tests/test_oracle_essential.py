"""CPU oracle for cv::findEssentialMat (RANSAC) + cv::recoverPose (oracle/yavo_oracle_essential.c; SURVEY.md 8f
row 2).  OpenCV is absent and no reference fixture holds E / R / t, so parity with the reference binary is unpinned;
these tests pin the restatement by its algebra (Durand-Kerner roots, the five-point constraints, exact two-view
scenes) and by an independent Python restatement of the cv::RNG subset stream."""
import numpy as np
import pytest

from oracle_bind import Oracle

from epipolar_scene import K_KITTI, skew, two_view_scene


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def test_solve_poly_real_roots(oracle):
    roots = np.array([-3.5, -2.0, -1.25, -0.5, 0.3, 0.9, 1.7, 2.4, 3.3, 4.1])
    c = np.poly(roots)[::-1]  # ascending
    got, _ = oracle.solve_poly(c)
    assert np.allclose(np.sort(got.real), np.sort(roots), atol=1e-9)
    assert np.all(np.abs(got.imag) < 1e-9)


def test_solve_poly_complex_pairs(oracle):
    roots = np.array([1 + 2j, 1 - 2j, -0.5 + 0.25j, -0.5 - 0.25j, 2.0])
    c = np.real(np.poly(roots))[::-1]
    got, _ = oracle.solve_poly(c)
    for z in roots:
        assert np.min(np.abs(got - z)) < 1e-9


def test_solve_poly_trims_vanishing_leading(oracle):
    c = np.array([2.0, -3.0, 1.0, 0.0, 0.0])  # (x - 1)(x - 2) with two zero leading coefficients
    got, _ = oracle.solve_poly(c)
    assert np.allclose(np.sort(got[:2].real), [1, 2])
    assert np.all(got[2:] == 0)


def _mwc_subsets(count, iters):
    """Independent restatement of cv::RNG((uint64)-1) + getSubset (5 distinct draws)."""
    state = (1 << 64) - 1
    out = []
    for _ in range(iters):
        row = []
        while len(row) < 5:
            state = ((state & 0xFFFFFFFF) * 4164903690 + (state >> 32)) & ((1 << 64) - 1)
            v = (state & 0xFFFFFFFF) % count
            if v not in row:
                row.append(v)
        out.append(row)
    return np.array(out, np.int32)


@pytest.mark.parametrize("count", [6, 7, 50, 2000])
def test_subsets_match_independent_rng(oracle, count):
    idx = oracle.em_subsets(count, 200)
    assert np.array_equal(idx, _mwc_subsets(count, 200))
    assert all(len(set(r)) == 5 for r in idx.tolist())
    assert idx.min() >= 0 and idx.max() < count


def test_em_kernel_exact_five_points(oracle):
    p1, p2, R, t = two_view_scene(5, seed=3, rounded=False)
    f, cx, cy = 718.856, 607.1928, 185.2157
    q1 = (p1 - [cx, cy]) / f
    q2 = (p2 - [cx, cy]) / f
    models = oracle.em_kernel(q1, q2)
    assert 1 <= len(models) <= 10
    E_true = skew(t) @ R
    E_true /= np.linalg.norm(E_true)
    x1 = np.c_[q1, np.ones(5)]
    x2 = np.c_[q2, np.ones(5)]
    best = min(min(np.linalg.norm(E - E_true), np.linalg.norm(E + E_true)) for E in models)
    assert best < 1e-6
    for E in models:  # every (unit-norm) model satisfies the epipolar and the cubic constraints to root precision
        assert np.abs(np.einsum("ij,jk,ik->i", x2, E, x1)).max() < 1e-6
        assert abs(np.linalg.det(E)) < 1e-6
        assert np.abs(2 * E @ E.T @ E - np.trace(E @ E.T) * E).max() < 1e-6


@pytest.mark.parametrize("seed,outl", [(0, 0.0), (1, 0.2), (2, 0.4)])
def test_find_essential_and_recover_pose(oracle, seed, outl):
    n = 600
    p1, p2, R, t = two_view_scene(n, outlier_frac=outl, seed=seed)
    ok, E, mask, st = oracle.find_essential(p1, p2)
    assert ok
    k = int(outl * n)
    assert mask[k:].mean() > 0.95          # true correspondences (pixel-rounded) are inliers
    assert mask[:k].mean() < 0.2 if k else True
    assert st["best"] == mask.sum() and 0 < st["iters"] < 1000
    good, Rr, tr, g = oracle.recover_pose(E, p1, p2, K_KITTI)
    assert good == max(g)
    ang = np.degrees(np.arccos(np.clip((np.trace(Rr.T @ R) - 1) / 2, -1, 1)))
    assert ang < 0.3
    assert np.degrees(np.arccos(np.clip(abs(tr @ t), -1, 1))) < 3.0 and tr @ t > 0
    assert np.isclose(np.linalg.det(Rr), 1.0) and np.isclose(np.linalg.norm(tr), 1.0)


def test_find_essential_small_inputs(oracle):
    p1, p2, _, _ = two_view_scene(5, seed=4, rounded=False)
    ok, E, mask, st = oracle.find_essential(p1[:4], p2[:4])
    assert not ok
    ok, E, mask, st = oracle.find_essential(p1, p2)  # count == modelPoints: runKernel on the list itself
    assert ok and mask.all() and st["iters"] == 1 and abs(np.linalg.norm(E) - 1) < 1e-12


def test_find_essential_is_deterministic(oracle):
    p1, p2, _, _ = two_view_scene(300, outlier_frac=0.3, seed=5)
    a = oracle.find_essential(p1, p2)
    b = oracle.find_essential(p1, p2)
    assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]
