"""CPU oracle for the sliding-window bundle adjustment (oracle/yavo_oracle_ba.c; BASELINE.json config 5, SURVEY.md
8d-8e).  g2o is absent and the reference holds no multi-pose BA fixture (its Optimizer::partialBA is a pose-only
stub), so parity with a g2o build is unpinned; these tests pin the restatement by its algebra: the LDLT against
numpy, exact recovery of a noise-free window, chi2 monotonicity of LM, the gauge (fixed poses untouched) and the
degenerate graphs."""
import numpy as np
import pytest

from oracle_bind import Oracle
from ya_vo_amd import scene


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def _spd(n, seed, cond=1e3):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    d = np.geomspace(1.0, cond, n)
    return (Q * d) @ Q.T


@pytest.mark.parametrize("n,seed", [(1, 0), (6, 1), (30, 2), (114, 3)])
def test_ldlt_solves_spd(oracle, n, seed):
    H = _spd(n, seed)
    b = np.random.default_rng(seed + 100).normal(size=n)
    x, pos = oracle.ldlt_solve(H, b)
    assert pos
    np.testing.assert_allclose(H @ x, b, rtol=0, atol=1e-9 * np.abs(b).max() * 1e3)


def test_ldlt_pivots_and_flags_indefinite(oracle):
    H = np.diag([1.0, -4.0, 2.0, 9.0])
    H[0, 3] = H[3, 0] = 0.5
    b = np.array([1.0, 2.0, 3.0, 4.0])
    x, pos = oracle.ldlt_solve(H, b)
    assert not pos
    np.testing.assert_allclose(H @ x, b, atol=1e-12)


def test_ldlt_zero_matrix(oracle):
    x, pos = oracle.ldlt_solve(np.zeros((3, 3)), np.ones(3))
    assert pos and not x.any()


def _run(oracle, w, n_fixed, iters=10):
    return oracle.ba_lm(w["poses0"], n_fixed, w["X0"], w["ep"], w["el"], w["meas"], scene.K_KITTI, iters)


def test_ba_noise_free_recovers_truth(oracle):
    # two fixed poses fix the gauge, scale included: the truth is the unique minimum
    w = scene.ba_window(n_poses=6, n_landmarks=300, obs=4, noise_px=0.0, seed=1)
    w["poses0"][1] = w["poses_true"][1]
    T, X, it, log = _run(oracle, w, 2, 20)
    assert log[-1] < 1e-12 * log[0]
    np.testing.assert_allclose(T, w["poses_true"], atol=1e-7)
    np.testing.assert_allclose(X, w["X_true"], rtol=2e-5, atol=1e-6)


def test_ba_noisy_chi2_decreases(oracle):
    w = scene.ba_window(n_poses=10, n_landmarks=1000, obs=5, noise_px=1.0, seed=2)
    T, X, it, log = _run(oracle, w, 1, 10)
    assert it >= 1 and np.all(np.diff(log) <= 0)
    E = len(w["ep"])
    dof = 2 * E - 6 * 9 - 3 * 1000
    assert 0.8 < log[-1] / dof < 1.2  # sigma = 1 px: chi2 ~ the degrees of freedom
    np.testing.assert_array_equal(T[0], w["poses0"][0])


def test_ba_fixed_poses_untouched_and_landmarks_only(oracle):
    w = scene.ba_window(n_poses=5, n_landmarks=200, obs=3, noise_px=0.5, seed=3)
    w["poses0"] = w["poses_true"].copy()
    T, X, it, log = _run(oracle, w, 5, 10)
    np.testing.assert_array_equal(T, w["poses_true"])
    assert log[-1] < 0.05 * log[0]


def test_ba_all_free(oracle):
    w = scene.ba_window(n_poses=4, n_landmarks=150, obs=4, noise_px=0.3, seed=4)
    T, X, it, log = _run(oracle, w, 0, 8)
    assert np.all(np.diff(log) <= 0) and log[-1] < log[0]


def test_ba_empty_graph(oracle):
    poses = scene.ba_window(n_poses=3, n_landmarks=1, obs=1, seed=5)["poses0"]
    T, X, it, log = oracle.ba_lm(poses, 1, np.zeros((0, 3)), np.zeros(0, np.int32), np.zeros(0, np.int32),
                                 np.zeros((0, 2)), scene.K_KITTI, 5)
    np.testing.assert_array_equal(T, poses)
    assert it == 1 and log[0] == 0.0
