"""GPU parity of the sliding-window bundle adjustment (yv_ba, ya_vo_amd/csrc/yavo_ba.hip; BASELINE.json config 5)
with the CPU oracle (oracle/yavo_oracle_ba.c or_ba_lm): poses, landmarks, the chi2 log and the iteration count, bit
for bit, from small windows to the config-5 size (20 keyframes, 10k landmarks, 5 observations each)."""
import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd import scene

pytestmark = pytest.mark.gpu


def _both(ctx, oracle, w, n_fixed, iters, ba=None):
    P, L, E = len(w["poses0"]), len(w["X0"]), len(w["ep"])
    ba = ba or yv.BundleAdjuster(ctx, P, max(L, 1), max(E, 1))
    ba.set_problem(P, n_fixed, L, w["ep"], w["el"], w["meas"], scene.K_KITTI)
    T, X, log, it = ba.solve(w["poses0"], w["X0"], iters)
    oT, oX, oit, olog = oracle.ba_lm(w["poses0"], n_fixed, w["X0"], w["ep"], w["el"], w["meas"], scene.K_KITTI, iters)
    assert it == oit
    np.testing.assert_array_equal(log, olog)
    np.testing.assert_array_equal(T, oT)
    np.testing.assert_array_equal(X, oX)
    return T, X, log


@pytest.mark.parametrize("P,L,obs,noise,nf,iters,seed", [
    (5, 200, 3, 1.0, 1, 10, 0),
    (6, 300, 4, 0.0, 2, 20, 1),
    (10, 1000, 5, 1.0, 1, 10, 2),
    (4, 150, 4, 0.3, 0, 8, 3),     # no fixed pose
    (5, 200, 3, 0.5, 5, 10, 4),    # all poses fixed: landmarks only (no reduced system)
    (44, 2000, 6, 1.0, 2, 6, 5),   # reduced system 252 x 252: more than one LDLT pass per thread
])
def test_ba_matches_oracle(ctx, oracle, P, L, obs, noise, nf, iters, seed):
    w = scene.ba_window(n_poses=P, n_landmarks=L, obs=obs, noise_px=noise, seed=seed)
    if noise == 0.0:
        w["poses0"][:nf] = w["poses_true"][:nf]
    _, _, log = _both(ctx, oracle, w, nf, iters)
    assert log[-1] <= log[0]


def test_ba_config5_matches_oracle(ctx, oracle):
    """BASELINE.json config 5: 20-keyframe window, 10k landmarks, 5 observations each, 10 LM iterations."""
    w = scene.ba_window(n_poses=20, n_landmarks=10000, obs=5, noise_px=1.0, seed=0)
    _, _, log = _both(ctx, oracle, w, 1, 10)
    assert log[-1] < 0.05 * log[0]


@pytest.mark.parametrize("on_device", [True, False])
def test_ba_control_modes_match_oracle(ctx, oracle, on_device):
    """The LM control on the device (default: the host enqueues every iteration, one read-back per solve; iterations
    whose first damping trial is rejected suspend and resume) and on the host (one read-back per trial): both bit for
    bit the oracle's, with a poor start (rejected trials) and an exact one (rho = 0 ends the run)."""
    for kw, nf, iters in [(dict(noise_px=2.0, init_rot=0.05, init_trans=0.5, init_point=1.0, seed=21), 1, 12),
                          (dict(noise_px=0.0, seed=22), 2, 25)]:
        w = scene.ba_window(n_poses=7, n_landmarks=300, obs=4, **kw)
        if kw["noise_px"] == 0.0:
            w["poses0"][:nf] = w["poses_true"][:nf]
        ba = yv.BundleAdjuster(ctx, 7, 300, 1200)
        ba.set_control(on_device)
        _both(ctx, oracle, w, nf, iters, ba)
        ba.close()


def test_ba_reuse_and_shrink(ctx, oracle):
    """One workspace, several graphs of different sizes (the structure rebuilt per set_problem)."""
    ba = yv.BundleAdjuster(ctx, 20, 3000, 15000)
    for P, L, obs, seed in [(20, 3000, 5, 10), (6, 100, 2, 11), (12, 2500, 6, 12)]:
        w = scene.ba_window(n_poses=P, n_landmarks=L, obs=obs, noise_px=1.0, seed=seed)
        _both(ctx, oracle, w, 1, 5, ba)


def test_ba_empty_graph(ctx, oracle):
    poses = scene.ba_window(n_poses=3, n_landmarks=1, obs=1, seed=5)["poses0"]
    w = dict(poses0=poses, X0=np.zeros((0, 3)), ep=np.zeros(0, np.int32), el=np.zeros(0, np.int32),
             meas=np.zeros((0, 2)))
    T, _, log = _both(ctx, oracle, w, 1, 5)
    np.testing.assert_array_equal(T, poses)


def test_ba_rejects_bad_graph(ctx):
    ba = yv.BundleAdjuster(ctx, 4, 10, 20)
    ep = np.array([0, 4], np.int32)  # pose 4 out of range
    el = np.array([0, 1], np.int32)
    with pytest.raises(yv.YavoError):
        ba.set_problem(4, 1, 10, ep, el, np.zeros((2, 2)), scene.K_KITTI)
    with pytest.raises(yv.YavoError):
        ba.set_problem(5, 1, 10, ep, el, np.zeros((2, 2)), scene.K_KITTI)  # more poses than the workspace
    with pytest.raises(yv.YavoError):
        ba.set_problem(4, 5, 10, np.array([0, 1], np.int32), el, np.zeros((2, 2)), scene.K_KITTI)


@pytest.mark.timeout(300)
def test_ba_size_limits(ctx):
    """640 poses is the largest window (6 x 640 rows of the reduced system fit the LDLT's 64 KB of LDS): 641 is refused
    up front, and so is a debug LDLT above 3840 rows; 3840 itself still launches and solves."""
    with pytest.raises(yv.YavoError):
        yv.BundleAdjuster(ctx, 641, 10, 20)
    yv.BundleAdjuster(ctx, 640, 10, 20).close()
    with pytest.raises(yv.YavoError):
        ctx.ba_ldlt(np.eye(3841), np.ones(3841))
    n = 3840  # a diagonal system: the pivoted LDLT's L is I and D the diagonal, so x = b / d, each one division
    d = np.linspace(1.0, 2.0, n)
    b = np.arange(n, dtype=np.float64) + 0.5
    x, ok = ctx.ba_ldlt(np.diag(d), b)
    assert ok
    np.testing.assert_array_equal(x, b / d)


def _spd(n, seed, cond=1e3):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    H = (Q * np.geomspace(1.0, cond, n)) @ Q.T
    return np.tril(H) + np.tril(H, -1).T  # bitwise symmetric, as the Schur kernel writes S


def _block_tridiagonal(nb, seed):
    """The configs[2] window's reduced system: 6 x 6 pose blocks coupled to their neighbours only."""
    rng = np.random.default_rng(seed)
    n = 6 * nb
    J = np.zeros((3 * n, n))
    for p in range(nb):
        J[18 * p:18 * p + 18, 6 * p:6 * p + 6] = rng.normal(size=(18, 6))
        if p + 1 < nb:
            J[18 * p:18 * p + 18, 6 * p + 6:6 * p + 12] = 0.3 * rng.normal(size=(18, 6))
    H = J.T @ J + 1e-3 * np.eye(n)
    return np.tril(H) + np.tril(H, -1).T


def _ldlt_cases():
    cases = [(f"spd{n}", _spd(n, n)) for n in (1, 2, 5, 6, 60, 63, 64, 65, 114, 120, 127, 128, 129, 200)]
    cases.append(("window120", _block_tridiagonal(20, 7)))
    cases.append(("window126", _block_tridiagonal(21, 8)))
    tie = _spd(24, 9)
    np.fill_diagonal(tie, 5.0)  # every pivot tied: the scan-and-swap replay
    cases.append(("ties", tie))
    part = _spd(40, 10)
    part[3, 3] = part[17, 17] = part[30, 30]  # a few tied diagonals among distinct ones
    cases.append(("some_ties", part))
    z = np.zeros((12, 12))
    z[1, 0] = z[0, 1] = 1.0  # zero diagonal: the first pivot is zero (factorisation stops)
    cases.append(("zero_first_pivot", z))
    cases.append(("zero_matrix", np.zeros((7, 7))))
    later = np.array([[4.0, 2.0, 1.0], [2.0, 1.0, 3.0], [1.0, 3.0, 2.5]])  # D(1) = 0 after the first step
    cases.append(("zero_later_pivot", later))
    ind = _spd(30, 11)
    ind[np.arange(0, 30, 4), np.arange(0, 30, 4)] *= -1.0  # indefinite: isPositive false
    cases.append(("indefinite", ind))
    nan_off = _spd(16, 12)
    nan_off[9, 2] = nan_off[2, 9] = np.nan
    cases.append(("nan_offdiag", nan_off))
    nan_diag = _spd(16, 13)
    nan_diag[5, 5] = np.nan
    cases.append(("nan_diag", nan_diag))
    return cases


@pytest.mark.parametrize("name,S", _ldlt_cases(), ids=[c[0] for c in _ldlt_cases()])
def test_ba_ldlt_matches_oracle(ctx, oracle, name, S):
    """The reduced-system solver alone (n <= 128: registers + LDS column hand-offs; above: global memory) against the
    oracle's or_ldlt_solve, bit for bit, including the pivot replay on ties, zero and NaN pivots and the flag."""
    b = np.random.default_rng(len(S)).normal(size=len(S))
    x, ok = ctx.ba_ldlt(S, b)
    ox, ook = oracle.ldlt_solve(S, b)
    assert ok == ook
    np.testing.assert_array_equal(x, ox)
