"""GPU parity of the full front end over a sequence (BASELINE configs[2] in miniature): detect / describe /
match / PnP / shared map / local BA through libyavo (ya_vo_amd.sequence.SequenceFrontend) against the same loop
over the CPU oracle (tests/sequence_chain.py): trajectories and refined landmarks bit for bit (the metric's "RMSE
vs CPU ref" is 0), and the trajectory follows the synthetic ground truth."""
import os

import numpy as np
import pytest

from sequence_chain import ground_truth, oracle_sequence, rmse_translation
from ya_vo_amd import scene
from ya_vo_amd.sequence import SequenceFrontend, se3_inverse
from ya_vo_amd.synth import synth_sequence

pytestmark = pytest.mark.gpu

T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)


@pytest.mark.parametrize("n,chunk", [(8, 4), (12, 6)])
def test_sequence_matches_oracle(ctx, oracle, offsets, n, chunk, tmp_path):
    import torch
    from ya_vo_amd import io as yio
    frames = synth_sequence(71, n, stereo=True)  # [n, 2, H, W]
    fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT)
    d = torch.from_numpy(frames.reshape(2 * n, *frames.shape[2:])).to("cuda:0")
    for c in range(n // chunk):
        fe.process_chunk(d[2 * c * chunk:2 * (c + 1) * chunk])
    traj = fe.trajectory()
    ref, rec, log = oracle_sequence(oracle, frames, chunk, scene.K_KITTI, T_RIGHT, offsets, threads=8)
    assert [x[:2] for x in fe.ba_log] == [x[:2] for x in log]
    np.testing.assert_array_equal(np.array([x[2:] for x in fe.ba_log]), np.array([x[2:] for x in log]))
    np.testing.assert_array_equal(traj, ref)
    for g, r in rec.items():
        np.testing.assert_array_equal(fe.records[g].edge, r.edge)
        np.testing.assert_array_equal(fe.records[g].X, r.X)
    assert rmse_translation(traj, ref) == 0.0
    assert rmse_translation(traj, ground_truth(n, scene.K_KITTI)) < 0.02
    # the KITTI pose file of the trajectory (T_wc rows) reads back
    path = str(tmp_path / "poses.txt")
    yio.write_kitti_poses(path, np.stack([se3_inverse(T) for T in traj]))
    back = yio.read_kitti_poses(path)
    np.testing.assert_allclose(back[:, :, 3], traj[:, 4:], atol=1e-9)
    fe.close()


def _threads():
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else min(n, 16)


@pytest.mark.timeout(900)
def test_sequence_200_frames_matches_oracle(ctx, oracle, offsets):
    """BASELINE configs[2] at its stated size: the first 200 frames of a sequence in chunks of 20 (10 BA windows of
    22 poses), trajectory and BA logs bit-identical to the oracle loop (RMSE vs CPU ref = 0), and within 2 cm of the
    synthetic ground truth."""
    import torch
    n, chunk = 200, 20
    frames = synth_sequence(71, n, stereo=True)
    fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT)
    d = torch.from_numpy(frames.reshape(2 * n, *frames.shape[2:])).to("cuda:0")
    for c in range(n // chunk):
        fe.process_chunk(d[2 * c * chunk:2 * (c + 1) * chunk])
    traj = fe.trajectory()
    ba_log = list(fe.ba_log)
    fe.close()
    del d
    ref, _, log = oracle_sequence(oracle, frames, chunk, scene.K_KITTI, T_RIGHT, offsets, threads=_threads())
    assert [x[:2] for x in ba_log] == [x[:2] for x in log]
    np.testing.assert_array_equal(np.array([x[2:] for x in ba_log]), np.array([x[2:] for x in log]))
    np.testing.assert_array_equal(traj, ref)
    assert rmse_translation(traj, ground_truth(n, scene.K_KITTI)) < 0.02


@pytest.mark.timeout(600)
def test_sequence_window_solves_that_suspend_match_oracle(ctx, oracle, offsets):
    """Window solves whose device LM suspends (an iteration's first damping trial rejected: at 40 iterations the
    synthetic windows get there) and is resumed from the host: the finish and write-back enqueued with the solve are
    skipped on the device and rerun after the resume, and the result is still the oracle loop's bit for bit."""
    import torch
    n, chunk, iters = 60, 20, 40
    frames = synth_sequence(71, n, stereo=True)
    fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT, ba_iters=iters)
    d = torch.from_numpy(frames.reshape(2 * n, *frames.shape[2:])).to("cuda:0")
    for c in range(n // chunk):
        fe.process_chunk(d[2 * c * chunk:2 * (c + 1) * chunk])
    traj = fe.trajectory()
    ba_log = list(fe.ba_log)
    resumes = fe.ba.resumes()
    fe.close()
    del d
    assert resumes > 0  # the resume path ran (2 on this sequence, tools/ba_resume_probe.py)
    ref, _, log = oracle_sequence(oracle, frames, chunk, scene.K_KITTI, T_RIGHT, offsets, ba_iters=iters,
                                  threads=_threads())
    assert [x[:2] for x in ba_log] == [x[:2] for x in log]
    np.testing.assert_array_equal(np.array([x[2:] for x in ba_log]), np.array([x[2:] for x in log]))
    np.testing.assert_array_equal(traj, ref)


def test_sequence_device_window_equals_host_assembly(ctx):
    """The BA window recorded, assembled and written back on the device (yv_ba_window_*) gives the host assembly's
    (window_problem / yv_ba_set_problem / apply_window) trajectory, BA logs and frame records bit for bit."""
    import torch
    n, chunk = 60, 20
    frames = synth_sequence(71, n, stereo=True)
    d = torch.from_numpy(frames.reshape(2 * n, *frames.shape[2:])).to("cuda:0")
    out = []
    for device_window in (True, False):
        fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT, device_window=device_window)
        for c in range(n // chunk):
            fe.process_chunk(d[2 * c * chunk:2 * (c + 1) * chunk])
        out.append((fe.trajectory(), fe.records, list(fe.ba_log)))
        fe.close()
    (t_dev, r_dev, l_dev), (t_host, r_host, l_host) = out
    assert len(l_dev) == n // chunk - 1 + 1 and l_dev == l_host
    np.testing.assert_array_equal(t_dev, t_host)
    assert sorted(r_dev) == sorted(r_host)
    for g in r_host:
        np.testing.assert_array_equal(r_dev[g].T_wc, r_host[g].T_wc)
        np.testing.assert_array_equal(r_dev[g].edge, r_host[g].edge)
        np.testing.assert_array_equal(r_dev[g].X, r_host[g].X)
        np.testing.assert_array_equal(r_dev[g].uv_own, r_host[g].uv_own)
        np.testing.assert_array_equal(r_dev[g].uv_prev, r_host[g].uv_prev)


@pytest.mark.gpu
def test_window_solve_begin_end_guards(ctx):
    """yv_ba_window_solve_begin / _end (the sequence's asynchronous window solve): while a solve is pending the window
    refuses reads, records, a second begin and a second end (YV_ERR_INVALID), and after the end it reads the refined
    records."""
    import torch
    n, chunk = 40, 20
    frames = synth_sequence(73, n, stereo=True)
    d = torch.from_numpy(frames.reshape(2 * n, *frames.shape[2:])).to("cuda:0")
    fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT, device_window=True)
    try:
        fe.process_chunk(d[:2 * chunk])
        assert fe._ba_pending  # the chunk's window solve was begun and not collected
        with pytest.raises(RuntimeError):
            fe.win.read(0)
        with pytest.raises(RuntimeError):
            fe.win.solve_begin(0, chunk, 2, scene.K_KITTI, 10)
        solved, log, it = fe.win.solve_end()
        fe._ba_pending = False
        assert solved and it >= 1 and len(log) == it + 1
        with pytest.raises(RuntimeError):
            fe.win.solve_end()
        T, e, X, uo, up = fe.win.read(chunk - 1)
        assert np.all(np.isfinite(T))
    finally:
        fe.close()
