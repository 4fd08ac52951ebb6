"""The multi-rank product path shards ONE sequence (BASELINE configs[3] in miniature): two ranks, each
a fresh child process running ya_vo_amd.sharding.FrameShard on its chunk with the 1-frame halo, all-gather their
shared-map blocks (gloo here: both ranks share the test box's one GPU; the bench uses RCCL) and place them with the
serial anchor chain.  The result must be the 1-rank run of the same frames: every relative pose bit for bit (the
halo gives rank 1's first temporal pair the same keypoints the 1-rank run's carry slot does) and the placed map
(keyframe poses, landmark ids and world points) within 1e-12 absolute + 1e-13 relative -- the chunked anchor chain
A_1 * L_k re-associates the 1-rank left fold rel_0 * ... * rel_k.  The last case is BASELINE
configs[3]'s length (KITTI sequence 00: 4541 frames) on two ranks.  RCCL itself needs a GPU per rank, so its leg
runs at world 1 here (test_rccl_exchange_world1_equals_local).  Reference: the serial chaining of
src/LoopHandler.cc:139,156."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from ya_vo_amd import map as ymap
from ya_vo_amd import scene
from ya_vo_amd.sharding import FrameShard, shard_images
from ya_vo_amd.synth import synth_stereo_batch

pytestmark = pytest.mark.gpu

TESTS = os.path.dirname(os.path.abspath(__file__))
T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _one_rank(ctx, n, kf_every, seed):
    import torch
    fr = synth_stereo_batch(seed, n + 1, start=0)
    d = torch.from_numpy(shard_images(fr[2:], fr[0])).to("cuda:0")
    shard = FrameShard(ctx, n, 1, scene.K_KITTI, T_RIGHT, halo=True, kf_every=kf_every,
                       max_kf=ymap.max_keyframes(n, 1, kf_every))
    for _ in range(2):  # as the workers: the placement base advances by the sequence's span every step
        shard.step(d.data_ptr())
    shard.drain()
    out = shard.poses(), shard.placed_map()
    shard.close()
    return out


def _map(placed):
    m = ymap.Map()
    m.insert_blocks(placed, placed.shape[0], placed.shape[1])
    return m


# (2270, 4): BASELINE configs[3]'s length -- KITTI sequence 00 has 4541 frames = the halo frame 0 + 2 x 2270
@pytest.mark.timeout(900)
@pytest.mark.parametrize("B,kf_every", [(4, 1), (6, 2), (2270, 4)])
def test_two_rank_shards_equal_one_rank(ctx, tmp_path, B, kf_every):
    world, seed = 2, 91
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(TESTS, "shard_worker.py"), str(r), str(world), str(port),
                               str(B), str(kf_every), str(seed), str(tmp_path / f"rank{r}.npz")], env=env)
             for r in range(world)]
    for p in procs:
        assert p.wait(timeout=110 if B < 100 else 600) == 0
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    ref_poses, ref_placed = _one_rank(ctx, world * B, kf_every, seed)

    # relative poses: bit for bit, including rank 1's first frame (its predecessor comes from the halo)
    np.testing.assert_array_equal(np.concatenate([r["poses"] for r in res]), ref_poses)
    assert all(int(r["edge_count"][0]) > 1000 for r in res), "the halo pair must produce PnP edges"
    # every rank holds the same placed map
    np.testing.assert_array_equal(res[0]["placed"], res[1]["placed"])
    got, ref = _map(res[0]["placed"]), _map(ref_placed)
    assert sorted(got.frames) == sorted(ref.frames) == list(range(kf_every, world * B + 1, kf_every))
    assert sorted(got.landmarks) == sorted(ref.landmarks)
    # the re-association error grows with the chain: 1e-12 absolute on short sequences, plus 1e-13 relative at the
    # full sequence length (4540 chained frames, ~920 m of synthetic trajectory)
    for g in ref.frames:
        np.testing.assert_allclose(got.frames[g], ref.frames[g], rtol=1e-13, atol=1e-12)
    gl = np.array([got.landmarks[i] for i in sorted(ref.landmarks)])
    rl = np.array([ref.landmarks[i] for i in sorted(ref.landmarks)])
    np.testing.assert_allclose(gl, rl, rtol=1e-13, atol=1e-12)
    # the rank boundary carries the sequence's real motion (the synthetic camera moves 0.21 m per frame), not the
    # identity an empty or stale predecessor would give
    assert np.linalg.norm(res[1]["poses"][0][4:]) > 0.1


@pytest.mark.timeout(300)
def test_rccl_exchange_world1_equals_local(ctx, tmp_path):
    """The RCCL leg of the shared-map exchange (all_gather_into_tensor on the communication stream, sharding.py) on
    the box's one GPU: a 1-rank "nccl" process group gathers the block into its own buffer and places it from there.
    Poses and the placed map must be the no-collective run's, bit for bit."""
    B, kf_every, seed = 6, 2, 91
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = tmp_path / "rank0.npz"
    p = subprocess.Popen([sys.executable, os.path.join(TESTS, "shard_worker.py"), "0", "1", str(port), str(B),
                          str(kf_every), str(seed), str(out), "nccl"], env=env)
    assert p.wait(timeout=240) == 0
    res = np.load(out)
    ref_poses, ref_placed = _one_rank(ctx, B, kf_every, seed)
    np.testing.assert_array_equal(res["poses"], ref_poses)
    np.testing.assert_array_equal(res["placed"], ref_placed)
    assert sorted(_map(res["placed"]).frames) == list(range(kf_every, B + 1, kf_every))
