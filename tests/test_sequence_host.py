"""CPU tests of the sequence front end's host logic (ya_vo_amd/sequence.py) and of its oracle restatement
(tests/sequence_chain.py) on a short synthetic stereo sequence with a known trajectory (BASELINE configs[2]
in miniature; the GPU run is tests/test_gpu_sequence.py)."""
import numpy as np
import pytest

import sequence_chain as chain
from sequence_chain import front_end, ground_truth, oracle_sequence, rmse_translation, sequence_from_tracks
from ya_vo_amd import scene
from ya_vo_amd.sequence import FrameRecord, apply_window, frame_records_from_block, se3_inverse, window_problem
from ya_vo_amd.synth import synth_frame

T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)


def test_se3_inverse(oracle):
    rng = np.random.default_rng(0)
    for _ in range(5):
        T = oracle.se3_exp(rng.normal(0, 0.5, 6))
        np.testing.assert_allclose(oracle.se3_mul(T, se3_inverse(T)), [0, 0, 0, 1, 0, 0, 0], atol=1e-12)
        np.testing.assert_allclose(se3_inverse(se3_inverse(T)), T, atol=1e-12)
        # the window assembly's inverse is the oracle's (Sophus SE3d::inverse) bit for bit
        np.testing.assert_array_equal(se3_inverse(T), oracle.se3_inverse(T))
        Tn = T.copy()
        Tn[:4] *= 1.0 + 1e-9  # an SE3 built from a not-quite-unit quaternion: the SO3 constructor renormalises
        np.testing.assert_array_equal(se3_inverse(Tn), oracle.se3_inverse(Tn))


def _records(oracle, n_frames, n_pts, noise, seed):
    """Exact per-frame landmarks of a random scene seen by cameras moving along x, with noisy poses."""
    rng = np.random.default_rng(seed)
    K = scene.K_KITTI
    truth = [np.concatenate([[0, 0, 0, 1.0], [0.5 * g, 0.0, 0.0]]) for g in range(n_frames)]  # T_wc
    recs = {}
    for g in range(n_frames):
        pc = np.stack([rng.uniform(-8, 8, n_pts), rng.uniform(-3, 3, n_pts), rng.uniform(8, 30, n_pts)], 1)
        Xw = np.array([oracle.se3_act(truth[g], p) for p in pc])
        own = scene.project(se3_inverse(truth[g]), Xw, K)
        prev = scene.project(se3_inverse(truth[g - 1]), Xw, K) if g else own
        T0 = truth[g].copy()
        if g >= 2:
            T0[4:] += rng.normal(0, noise, 3)
        recs[g] = FrameRecord(T0, np.arange(n_pts), Xw + rng.normal(0, noise, Xw.shape), prev, own)
    return recs, truth


def test_window_problem_layout(oracle):
    recs, _ = _records(oracle, 4, 10, 0.0, 1)
    poses, X, ep, el, meas, owners = window_problem(recs, [1, 2, 3], 1)
    assert poses.shape == (3, 7) and X.shape == (20, 3)  # frame 1's predecessor is outside the window
    assert owners == [(1, 0), (2, 10), (3, 10)]
    assert list(ep[:10]) == [1] * 10 and list(ep[10:20]) == [0] * 10 and list(el[:10]) == list(range(10))
    np.testing.assert_array_equal(meas[:10], recs[2].uv_own)
    np.testing.assert_array_equal(meas[10:20], recs[2].uv_prev)


def test_window_assembly_equals_the_tests_restatement(oracle):
    """The product's host window assembly (ya_vo_amd.sequence.window_problem / apply_window, the device window's
    checked restatement) equals tests/sequence_chain.py's own (assemble_window / write_back) bit for bit, for windows
    that start at frame 0, mid-sequence, and hold frames without landmarks."""
    recs, _ = _records(oracle, 7, 12, 0.01, 5)
    recs[4].edge, recs[4].X = recs[4].edge[:0], recs[4].X[:0]
    recs[4].uv_prev, recs[4].uv_own = recs[4].uv_prev[:0], recs[4].uv_own[:0]
    for frames, n_fixed in (([0, 1, 2, 3], 2), ([2, 3, 4, 5, 6], 1), ([5, 6], 1)):
        a = window_problem(recs, frames, n_fixed)
        mine = {g: chain.Rec(r.T_wc.copy(), r.edge, r.X.copy(), r.uv_prev, r.uv_own) for g, r in recs.items()}
        b = chain.assemble_window(oracle, mine, frames, n_fixed)
        for x, y in zip(a[:5], b[:5]):
            assert x.dtype == y.dtype
            np.testing.assert_array_equal(x, y)
        assert [n for _, n in a[5]] == b[5]
        P, Xo, it, log = oracle.ba_lm(a[0], n_fixed, a[1], a[2], a[3], a[4], scene.K_KITTI, 3)
        prod = {g: FrameRecord(r.T_wc.copy(), r.edge, r.X.copy(), r.uv_prev, r.uv_own) for g, r in recs.items()}
        apply_window(prod, frames, P, Xo, a[5])
        chain.write_back(oracle, mine, frames, P, Xo, b[5])
        for g in recs:
            np.testing.assert_array_equal(prod[g].T_wc, mine[g].T_wc)
            np.testing.assert_array_equal(prod[g].X, mine[g].X)


def test_block_records_equal_the_tests_restatement(oracle):
    """frame_records_from_block (the product's block parser) and sequence_chain.records_from_block (the layout of
    include/yavo/yavo_map.h restated with struct offsets) read the same records from an oracle map block."""
    rng = np.random.default_rng(3)
    n, kp = 4, 50
    rel = np.array([oracle.se3_exp(rng.normal(0, 0.05, 6)) for _ in range(n)])
    ec = rng.integers(0, kp, n).astype(np.int32)
    eX = rng.normal(0, 5, (n, kp, 3))
    eo = (rng.random((n, kp)) < 0.2).astype(np.uint8)
    block = oracle.map_chunk(rel, 40, 1, ec, eX, eo, kp, n)
    placed, _, _ = oracle.map_place(block, 1, len(block), np.array([0, 0, 0, 1, 1.0, 2.0, 3.0]))
    uv = rng.normal(0, 100, (n, kp, 2))
    q = rng.integers(0, kp, (n, kp)).astype(np.int32)
    own = rng.integers(0, 1000, (n, kp, 2)).astype(np.int32)
    a = frame_records_from_block(np.ascontiguousarray(placed), uv, q, own)
    b = chain.records_from_block(placed, uv, q, own)
    assert sorted(a) == sorted(b) == list(range(40, 40 + n))
    for g in a:
        for f in ("T_wc", "edge", "X", "uv_prev", "uv_own"):
            x, y = getattr(a[g], f), getattr(b[g], f)
            assert x.dtype == y.dtype
            np.testing.assert_array_equal(x, y)


def test_window_ba_recovers_truth(oracle):
    recs, truth = _records(oracle, 6, 60, 0.02, 2)
    frames = list(range(6))
    poses, X, ep, el, meas, owners = window_problem(recs, frames, 2)
    P, Xo, it, log = oracle.ba_lm(poses, 2, X, ep, el, meas, scene.K_KITTI, 20)
    assert log[-1] < 1e-3 * log[0]
    apply_window(recs, frames, P, Xo, owners)
    for g in frames:
        np.testing.assert_allclose(recs[g].T_wc[4:], truth[g][4:], atol=1e-3)


def test_oracle_sequence_follows_ground_truth(oracle, offsets):
    n, chunk = 8, 4
    frames = np.stack([np.stack([synth_frame(61, k, 3 * k), synth_frame(61, k, 3 * k + 8)]) for k in range(n)])
    traj, records, ba_log = oracle_sequence(oracle, frames, chunk, scene.K_KITTI, T_RIGHT,
                                            offsets.reshape(256, 4), threads=8)
    assert traj.shape == (n, 7) and len(ba_log) == 2
    assert all(last_chi2 <= first_chi2 for _, _, first_chi2, last_chi2 in ba_log)
    gt = ground_truth(n, scene.K_KITTI)
    assert rmse_translation(traj, gt) < 0.02
    assert sum(len(r.edge) for r in records.values()) > 1000


def test_oracle_sequence_g2o_order_within_tolerance(oracle, offsets):
    """The same front end with the BA in g2o's loop orders (or_ba_lm mode 1): within north_star's 1e-4 trajectory
    tolerance of the kernel-order loop (the device's), and on the ground truth."""
    n, chunk = 8, 4
    frames = np.stack([np.stack([synth_frame(61, k, 3 * k), synth_frame(61, k, 3 * k + 8)]) for k in range(n)])
    tracks = front_end(oracle, frames, chunk, scene.K_KITTI, T_RIGHT, offsets.reshape(256, 4), threads=8)
    t0, _, l0 = sequence_from_tracks(oracle, tracks, chunk, scene.K_KITTI)
    t1, _, l1 = sequence_from_tracks(oracle, tracks, chunk, scene.K_KITTI, ba_mode=1)
    assert [x[:2] for x in l0] == [x[:2] for x in l1]
    assert rmse_translation(t0, t1) < 1e-6
    assert rmse_translation(t1, ground_truth(n, scene.K_KITTI)) < 0.02


def test_device_window_cap_is_checked_up_front():
    """chunk + n_fixed above the device window's pose capacity fails in the constructor with a clear message, before
    any device work (it used to fail at the first BA with YV_ERR_INVALID)."""
    import pytest
    from ya_vo_amd import sequence
    with pytest.raises(ValueError, match="at most 128 poses"):
        sequence.SequenceFrontend(None, 127, np.eye(3), np.array([0, 0, 0, 1, 0, -0.54, 0.0]), n_fixed=2)


def test_shard_range_overlaps_by_one_frame():
    from ya_vo_amd.sequence import shard_range
    assert [shard_range(r, 4, 100) for r in range(4)] == [(0, 100), (99, 199), (198, 298), (297, 397)]
    with pytest.raises(ValueError):
        shard_range(2, 2, 100)
    with pytest.raises(ValueError):
        shard_range(0, 1, 1)
