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


# ---- g2o's own summation orders (or_ba_lm mode 1): the CPU reference the device trajectory is measured against ----

def _run_mode(oracle, w, n_fixed, iters, mode):
    return oracle.ba_lm(w["poses0"], n_fixed, w["X0"], w["ep"], w["el"], w["meas"], scene.K_KITTI, iters, mode=mode)


def test_ba_g2o_order_noise_free_recovers_truth(oracle):
    w = scene.ba_window(n_poses=6, n_landmarks=300, obs=4, noise_px=0.0, seed=1)
    w["poses0"][1] = w["poses_true"][1]
    T, X, it, log = _run_mode(oracle, w, 2, 20, 1)
    assert log[-1] < 1e-12 * log[0]
    np.testing.assert_allclose(T, w["poses_true"], atol=1e-7)
    np.testing.assert_allclose(X, w["X_true"], rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("n_fixed", [0, 1, 2])
def test_ba_g2o_order_is_a_different_order_with_the_same_solution(oracle, n_fixed):
    """The two orders are different arithmetic (some bit of the result differs) converging to the same minimum: poses
    within 1e-9, chi2 logs within 1e-9 relative, chi2 non-increasing in both."""
    w = scene.ba_window(n_poses=8, n_landmarks=800, obs=4, noise_px=1.0, seed=7)
    T0, X0, it0, log0 = _run_mode(oracle, w, n_fixed, 10, 0)
    T1, X1, it1, log1 = _run_mode(oracle, w, n_fixed, 10, 1)
    assert it0 == it1
    assert np.all(np.diff(log1) <= 0)
    assert not (np.array_equal(T0, T1) and np.array_equal(X0, X1) and np.array_equal(log0, log1))
    np.testing.assert_allclose(T1, T0, rtol=0, atol=1e-9)
    np.testing.assert_allclose(log1, log0, rtol=1e-9)
    np.testing.assert_array_equal(T1[:n_fixed], w["poses0"][:n_fixed])


def _dense_lm_step(oracle, w, n_fixed):
    """One damped step of the full (unreduced) normal equations in numpy -- an order-free restatement of what an
    accepted first LM trial does: H = J^T J over all free variables, lambda = 1e-5 max diag, (H + lambda I) x =
    -J^T e, T_p <- exp(x_p) T_p, X_l <- X_l + x_l."""
    K = scene.K_KITTI
    P, L = len(w["poses0"]), len(w["X0"])
    npz = P - n_fixed
    n = 6 * npz + 3 * L
    H = np.zeros((n, n))
    b = np.zeros(n)
    for e, (p, l) in enumerate(zip(w["ep"], w["el"])):
        T, X = w["poses0"][p], w["X0"][l]
        pc = oracle.se3_act(T, X)
        R = oracle.quat_to_R(T[:4])
        uvw = np.asarray(K) @ pc
        err = w["meas"][e] - uvw[:2] / uvw[2]
        fx, fy = K[0][0], K[1][1]
        x, y, z = pc
        Jp = np.array([[-fx / z, 0, fx * x / z ** 2, fx * x * y / z ** 2, -fx - fx * x * x / z ** 2, fx * y / z],
                       [0, -fy / z, fy * y / z ** 2, fy + fy * y * y / z ** 2, -fy * x * y / z ** 2, -fy * x / z]])
        Jl = Jp[:, :3] @ R
        J = np.zeros((2, n))
        if p >= n_fixed:
            J[:, 6 * (p - n_fixed):6 * (p - n_fixed) + 6] = Jp
        J[:, 6 * npz + 3 * l:6 * npz + 3 * l + 3] = Jl
        H += J.T @ J
        b -= J.T @ err
    lam = 1e-5 * np.max(np.abs(np.diag(H)))
    x = np.linalg.solve(H + lam * np.eye(n), b)
    T = w["poses0"].copy()
    for p in range(n_fixed, P):
        T[p] = oracle.se3_mul(oracle.se3_exp(x[6 * (p - n_fixed):6 * (p - n_fixed) + 6]), T[p])
    return T, w["X0"] + x[6 * npz:].reshape(L, 3)


@pytest.mark.parametrize("mode", [0, 1])
def test_ba_first_step_equals_dense_normal_equations(oracle, mode):
    """The Schur-complement step (both orders) equals the dense solve of the unreduced system (numpy, its own
    order) when the first trial is accepted: an independent check of H_pp / H_pl / H_ll, the Schur complement,
    b_schur and the back-substitution."""
    w = scene.ba_window(n_poses=4, n_landmarks=60, obs=3, noise_px=0.5, seed=11)
    T_ref, X_ref = _dense_lm_step(oracle, w, 1)
    T, X, it, log = _run_mode(oracle, w, 1, 1, mode)
    assert log[1] < log[0]  # accepted
    np.testing.assert_allclose(T, T_ref, rtol=0, atol=1e-10)
    np.testing.assert_allclose(X, X_ref, rtol=0, atol=1e-9)
