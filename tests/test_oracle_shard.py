"""The frame-sharded front end on CPU (GPU counterpart tests/test_gpu_shard.py): a world-2 gloo job in
which every rank runs the oracle chain (detect / describe / match / removeOutliers / triangulation / pose LM,
tests/track_chain.py) over its own chunk of ONE sequence, recomputing its predecessor frame (the 1-frame halo), builds
its shared-map block (oracle map_chunk), all-gathers the blocks and places them (oracle map_place).  The placed map
must equal the 1-rank run of the same frames: relative poses bit for bit, placement within 1e-12 (re-association of
the anchor chain).  A shard that skips the halo (empty predecessor) must NOT match -- the check that catches an
identity pose at the rank boundary."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ya_vo_amd import map as ymap

MAX_KP, H, W = 2000, 160, 320
T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
IDENTITY = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
SEED, EVERY = 33, 2


def _chunk(oracle, offsets, first, n, halo=True):
    """Oracle chain over frames [first, first + n) (predecessor = frame first - 1 when halo, else none)
    -> (rel [n, 7], edge_count, edge_X, edge_outlier)."""
    from track_chain import track_pose
    from ya_vo_amd import scene
    from ya_vo_amd.synth import synth_stereo_batch
    fr = synth_stereo_batch(SEED, n + 1, start=first - 1, h=H, w=W)

    def kp(img):
        return oracle.brief(img, oracle.fast(img, MAX_KP)[0], offsets)

    prev = kp(fr[0]) if halo else kp(np.zeros((H, W), np.uint8))  # zero image: no corners, no keypoints
    rel = np.zeros((n, 7))
    ec = np.zeros(n, np.int32)
    eX = np.zeros((n, MAX_KP, 3))
    eo = np.zeros((n, MAX_KP), np.uint8)
    for k in range(n):
        kl, kr = kp(fr[2 + 2 * k]), kp(fr[3 + 2 * k])
        X, _, _, T, out, _ = track_pose(oracle, prev, kl, kr, scene.K_KITTI, T_RIGHT)
        rel[k], ec[k] = T, len(X)
        eX[k, :len(X)], eo[k, :len(X)] = X, out
        prev = kl
    return rel, ec, eX, eo


def _place(oracle, blocks, world, bb):
    placed, _, _ = oracle.map_place(blocks, world, bb, IDENTITY)
    m = ymap.Map()
    m.insert_blocks(placed, world, bb)
    return m


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, halo, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_bind import Oracle
    oracle = Oracle()
    offsets = np.fromfile(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "brief_offsets_mt19937_42.bin"), np.int8).reshape(256, 4)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first = 1 + rank * B
    rel, ec, eX, eo = _chunk(oracle, offsets, first, B, halo)
    max_kf = max(ymap.max_keyframes(B, 1 + r * B, EVERY) for r in range(world))
    blk = oracle.map_chunk(rel, first, EVERY, ec, eX, eo, MAX_KP, max_kf)
    gathered = ymap.gather_map_blocks(torch.from_numpy(blk), world).numpy()
    m = _place(oracle, gathered, world, len(blk))
    q.put((rank, rel.tolist(), {g: T.tolist() for g, T in m.get_frames().items()},
           {i: X.tolist() for i, X in m.get_mps().items()}))
    dist.barrier()
    dist.destroy_process_group()


def _run_world2(B, halo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, halo, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_halo_sharding_equals_one_rank_gloo_world2(oracle, offsets):
    B = 3
    res = _run_world2(B, halo=True)
    rel1, ec, eX, eo = _chunk(oracle, offsets, 1, 2 * B)
    blk = oracle.map_chunk(rel1, 1, EVERY, ec, eX, eo, MAX_KP, ymap.max_keyframes(2 * B, 1, EVERY))
    ref = _place(oracle, blk, 1, len(blk))
    np.testing.assert_array_equal(np.array(res[0][0] + res[1][0]), rel1)  # relative poses, bit for bit
    assert res[0][1:] == res[1][1:]  # every rank holds the same placed map
    frames, mps = res[0][1], res[0][2]
    assert sorted(frames) == sorted(ref.get_frames()) and sorted(mps) == sorted(ref.get_mps())
    for g, T in ref.get_frames().items():
        np.testing.assert_allclose(frames[g], T, rtol=0, atol=1e-12)
    for i, X in ref.get_mps().items():
        np.testing.assert_allclose(mps[i], X, rtol=0, atol=1e-12)
    assert np.linalg.norm(rel1[B][4:]) > 0.1  # the boundary pose carries real motion


def test_missing_halo_is_detected_gloo_world2(oracle, offsets):
    """Without the halo, rank 1's first frame has no predecessor: its pose is the prior (identity) and every later
    keyframe of rank 1 is placed off the 1-rank trajectory."""
    B = 3
    res = _run_world2(B, halo=False)
    rel1, *_ = _chunk(oracle, offsets, 1, 2 * B)
    rel_boundary = np.array(res[1][0][0])
    np.testing.assert_array_equal(rel_boundary, IDENTITY)
    assert not np.allclose(rel_boundary, rel1[B])
