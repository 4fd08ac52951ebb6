"""The frame-sharded sequence front end (BASELINE configs[3] / [4] on N GPUs in miniature): ONE
synthetic stereo sequence split over two ranks (ya_vo_amd.sequence.SequenceShard; shards overlap by one frame), each
a fresh child process with the whole device front end (detect .. pose LM, shared map, local BA windows), the shards'
map blocks all-gathered (gloo: both ranks share the test box's one GPU; RCCL at world 1 below) and placed after each
other. Checked against the CPU oracle loop (tests/sequence_chain.py) over each shard's frames: the shard's
trajectory and BA log bit for bit, and the placed trajectory / landmarks as the oracle's SE3 products of the anchor
chain A_0 = I, A_{r+1} = A_r C_r. Reference: src/LoopHandler.cc:139,156 (serial pose chaining), src/Map.cc:9-40."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from sequence_chain import ground_truth, oracle_sequence, rmse_translation
from ya_vo_amd import map as ymap
from ya_vo_amd import scene
from ya_vo_amd.sequence import shard_range
from ya_vo_amd.synth import synth_sequence

pytestmark = pytest.mark.gpu

TESTS = os.path.dirname(os.path.abspath(__file__))
T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(world, n, chunk, seed, tmp_path, backend="gloo"):
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(TESTS, "sequence_shard_worker.py"), str(r), str(world),
                               str(port), str(n), str(chunk), str(seed), str(tmp_path / f"rank{r}.npz"), backend],
                              env=env) for r in range(world)]
    try:
        for p in procs:
            assert p.wait(timeout=240) == 0
    finally:
        for p in procs:  # a rank that failed leaves its peer inside a collective: end both
            if p.poll() is None:
                p.kill()
                p.wait()
    return [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]


@pytest.mark.timeout(600)
def test_two_rank_sequence_shards_match_oracle(oracle, offsets, tmp_path):
    world, n, chunk, seed = 2, 40, 20, 71
    res = _spawn(world, n, chunk, seed, tmp_path)
    total = world * (n - 1) + 1
    frames = synth_sequence(seed, total, stereo=True)
    A = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
    want_T, want_lm = [], {}
    for r in range(world):
        first, end = shard_range(r, world, n)
        ref, rec, log = oracle_sequence(oracle, frames[first:end], chunk, scene.K_KITTI, T_RIGHT, offsets, threads=8)
        # the shard is the one-rank loop over its own frames, bit for bit
        np.testing.assert_array_equal(res[r]["local"], ref)
        np.testing.assert_array_equal(res[r]["ba_log"], np.array(log, np.float64).reshape(-1, 4))
        # placement: T_wc = A_r T, X_w = A_r X (oracle SE3 products), shard r > 0 without its first frame
        for k in range(0 if r == 0 else 1, n):
            want_T.append(oracle.se3_mul(A, ref[k]))
            for e, X in zip(rec[k].edge, rec[k].X):
                want_lm[((first + k) << 16) | int(e)] = oracle.se3_act(A, X)
        A = oracle.se3_mul(A, ref[-1])
    for r in range(world):  # every rank holds the same placed map
        np.testing.assert_array_equal(res[r]["placed"], res[0]["placed"])
    np.testing.assert_array_equal(res[0]["trajectory"], np.array(want_T))
    m = ymap.Map()
    m.insert_blocks(res[0]["placed"], world, res[0]["placed"].shape[1])
    assert sorted(m.frames) == list(range(total))
    assert sorted(m.landmarks) == sorted(want_lm) and len(want_lm) > 10000
    for i in want_lm:
        np.testing.assert_array_equal(m.landmarks[i], want_lm[i])
    # the shard boundary carries the sequence's motion: the placed trajectory follows the ground truth
    assert rmse_translation(res[0]["trajectory"], ground_truth(total, scene.K_KITTI)) < 0.02


@pytest.mark.timeout(300)
def test_sequence_shard_rccl_world1_equals_one_rank(ctx, tmp_path):
    """The RCCL leg: a 1-rank "nccl" group gathers the shard's block through all_gather_into_tensor and places it; the
    trajectory is the plain SequenceFrontend run's, bit for bit."""
    import torch
    from ya_vo_amd.sequence import SequenceFrontend
    n, chunk, seed = 40, 20, 71
    res = _spawn(1, n, chunk, seed, tmp_path, backend="nccl")
    frames = synth_sequence(seed, n, stereo=True)
    d = torch.from_numpy(frames.reshape(2 * n, *frames.shape[2:])).to("cuda:0")
    fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT)
    for c in range(n // chunk):
        fe.process_chunk(d[2 * c * chunk:2 * (c + 1) * chunk])
    traj = fe.trajectory()
    fe.close()
    np.testing.assert_array_equal(res[0]["local"], traj)
    np.testing.assert_array_equal(res[0]["trajectory"], traj)


def test_window_export_block_guards(ctx):
    """yv_ba_window_export_block refuses what it cannot write: frames never recorded, a landmark stride below the
    window's, more frames than keyframe slots, and an export while a window solve is pending."""
    import torch
    from ya_vo_amd import map as ymap
    from ya_vo_amd.sequence import SequenceFrontend
    n, chunk = 40, 20
    frames = synth_sequence(73, n, stereo=True)
    d = torch.from_numpy(frames.reshape(2 * n, *frames.shape[2:])).to("cuda:0")
    fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT, expected_frames=n)
    blk = torch.zeros(ymap.block_bytes(n, 2000), dtype=torch.uint8, device="cuda:0")
    try:
        fe.process_chunk(d[:2 * chunk])
        with pytest.raises(RuntimeError):  # the chunk's window solve is pending
            fe.win.export_block(0, chunk, chunk - 1, 0, blk.data_ptr(), n, 2000)
        fe.flush()
        with pytest.raises(RuntimeError):  # frames 20 .. 39 are not recorded yet
            fe.win.export_block(0, n, n - 1, 0, blk.data_ptr(), n, 2000)
        with pytest.raises(RuntimeError):  # landmark stride below the window's 2000 slots
            fe.win.export_block(0, chunk, chunk - 1, 0, blk.data_ptr(), n, 1000)
        with pytest.raises(RuntimeError):  # more frames than keyframe slots
            fe.win.export_block(0, chunk, chunk - 1, 0, blk.data_ptr(), chunk - 1, 2000)
        fe.win.export_block(0, chunk, chunk - 1, 100, blk.data_ptr(), n, 2000)
        ctx.sync()
        h, kfs, lms = ymap.parse_block(blk.cpu().numpy())
        assert int(h["placed"]) == 2 and int(h["n_kf"]) == chunk and int(h["first_frame"]) == 100
        traj = fe.trajectory()
        np.testing.assert_array_equal(np.array(kfs["T"]), traj)
        np.testing.assert_array_equal(np.array(h["chunk"]), traj[-1])
        for j, lm in enumerate(lms):
            assert np.all((lm["id"] >> 16) == 100 + j)
            np.testing.assert_array_equal(lm["X"], fe.records[j].X)
    finally:
        fe.close()
