"""CPU tests of the shared map (include/yavo/yavo_map.h): the oracle's chunk blocks and placement
(oracle/yavo_oracle_map.c), the host-side block layout and Map tables (ya_vo_amd/map.py), and the all-gather of
blocks over a world-2 gloo job (the GPU run uses RCCL). Reference: Map::insertKeyFrame / insertMapPoint
(src/Map.cc:9-40); the reference has no map tests, so the chunked map is checked against the same sequence built
as one chunk (parity unpinned against the reference binary)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ya_vo_amd import map as ymap

MAX_KP = 64


def _sequence(oracle, n, seed):
    """n relative poses (small random twists), per-track edges with some outliers."""
    rng = np.random.default_rng(seed)
    rel = np.stack([oracle.se3_exp(np.concatenate([rng.normal(0, 0.3, 3), rng.normal(0, 0.05, 3)]))
                    for _ in range(n)])
    ec = rng.integers(0, MAX_KP + 1, n).astype(np.int32)
    ec[n // 2] = 0  # a frame without edges
    eX = rng.normal(0, 5, (n, MAX_KP, 3))
    eX[..., 2] = np.abs(eX[..., 2]) + 1
    eo = (rng.random((n, MAX_KP)) < 0.2).astype(np.uint8)
    return rel, ec, eX, eo


def test_block_layout_agrees(oracle):
    for max_kf, stride in [(1, 1), (3, 2000), (64, 2000), (7, 13)]:
        bb = ymap.block_bytes(max_kf, stride)
        assert bb == oracle.map_block_bytes(max_kf, stride)
        assert bb % 256 == 0 and ymap.landmark_offset(max_kf) % 256 == 0
    with pytest.raises(ValueError):
        ymap.block_bytes(0, 5)
    assert oracle.map_block_bytes(0, 5) == -1


@pytest.mark.parametrize("first,n,every", [(0, 10, 1), (0, 10, 3), (7, 9, 4), (5, 1, 5), (6, 0, 2), (1, 3, 5)])
def test_max_keyframes(first, n, every):
    assert ymap.max_keyframes(n, first, every) == sum(1 for g in range(first, first + n) if g % every == 0)


def test_chunk_records(oracle):
    n, first, every = 12, 5, 2
    rel, ec, eX, eo = _sequence(oracle, n, 3)
    max_kf = ymap.max_keyframes(n, first, every)
    blk = oracle.map_chunk(rel, first, every, ec, eX, eo, MAX_KP, max_kf)
    h, kfs, lms = ymap.parse_block(blk)
    assert (int(h["n_frames"]), int(h["n_kf"]), int(h["first_frame"]), int(h["placed"])) == (n, max_kf, first, 0)
    L = rel[0].copy()
    chain = [L.copy()]
    for k in range(1, n):
        L = oracle.se3_mul(L, rel[k])
        chain.append(L.copy())
    np.testing.assert_array_equal(h["chunk"], chain[-1])
    j = 0
    for k in range(n):
        g = first + k
        if g % every:
            continue
        assert int(kfs[j]["frame_id"]) == g
        np.testing.assert_array_equal(kfs[j]["T"], chain[k])
        keep = [e for e in range(ec[k]) if eo[k, e] == 0]
        assert int(kfs[j]["n_landmarks"]) == len(keep)
        np.testing.assert_array_equal(lms[j]["id"], [(g << 16) | e for e in keep])
        np.testing.assert_array_equal(lms[j]["X"], eX[k, keep])
        j += 1
    assert j == max_kf


def test_max_kf_caps_keyframes(oracle):
    rel, ec, eX, eo = _sequence(oracle, 6, 4)
    h, kfs, _ = ymap.parse_block(oracle.map_chunk(rel, 0, 1, ec, eX, eo, MAX_KP, 2))
    assert int(h["n_kf"]) == 2 and list(kfs["frame_id"]) == [0, 1]


def _chunks(oracle, rel, ec, eX, eo, bounds, every):
    max_kf = max(max(ymap.max_keyframes(b - a, a, every) for a, b in bounds), 1)
    return [oracle.map_chunk(rel[a:b], a, every, ec[a:b], eX[a:b], eo[a:b], MAX_KP, max_kf) for a, b in bounds], max_kf


@pytest.mark.parametrize("bounds", [[(0, 5), (5, 11), (11, 16)], [(0, 8), (8, 8), (8, 16)], [(0, 16)]])
def test_place_matches_one_chunk(oracle, bounds):
    """Sharded chunks placed by the anchor chain = the same sequence built and placed as one chunk."""
    n, every = 16, 3
    rel, ec, eX, eo = _sequence(oracle, n, 11)
    base = oracle.se3_exp(np.array([1.0, -2.0, 0.5, 0.1, 0.2, -0.3]))
    blocks, max_kf = _chunks(oracle, rel, ec, eX, eo, bounds, every)
    bb = len(blocks[0])
    placed, end, anchors = oracle.map_place(np.concatenate(blocks), len(blocks), bb, base)
    one, one_kf = _chunks(oracle, rel, ec, eX, eo, [(0, n)], every)
    ref, ref_end, _ = oracle.map_place(one[0], 1, len(one[0]), base)
    np.testing.assert_array_equal(anchors[0], base)
    np.testing.assert_allclose(end, ref_end, atol=1e-12)
    m, mref = ymap.Map(), ymap.Map()
    m.insert_blocks(placed, len(blocks), bb)
    mref.insert_blocks(ref, 1, len(one[0]))
    assert sorted(m.get_frames()) == sorted(mref.get_frames()) == [g for g in range(n) if g % every == 0]
    assert sorted(m.get_mps()) == sorted(mref.get_mps())
    for g, T in mref.get_frames().items():
        np.testing.assert_allclose(m.get_frames()[g], T, atol=1e-12)
    for i, X in mref.get_mps().items():
        np.testing.assert_allclose(m.get_mps()[i], X, atol=1e-10)
    if len(bounds) == 1:
        np.testing.assert_array_equal(placed, ref)


def test_place_world_coordinates(oracle):
    """A placed landmark is T_wc(k) * X with T_wc(k) = base * rel_0 * ... * rel_k."""
    n = 5
    rel, ec, eX, eo = _sequence(oracle, n, 5)
    base = oracle.se3_exp(np.array([0.5, 0.0, 0.0, 0.0, 0.3, 0.0]))
    blk = oracle.map_chunk(rel, 0, 1, ec, eX, eo, MAX_KP, n)
    placed, _, _ = oracle.map_place(blk, 1, len(blk), base)
    h, kfs, lms = ymap.parse_block(placed)
    assert int(h["placed"]) == 1
    T = base.copy()
    for k in range(n):
        T = oracle.se3_mul(T, rel[k])
        np.testing.assert_allclose(kfs[k]["T"], T, atol=1e-12)
        for rec in lms[k][:5]:
            e = int(rec["id"]) & 0xFFFF
            np.testing.assert_allclose(rec["X"], oracle.se3_act(T, eX[k, e]), atol=1e-10)


def test_unplaced_block_rejected(oracle):
    rel, ec, eX, eo = _sequence(oracle, 3, 6)
    blk = oracle.map_chunk(rel, 0, 1, ec, eX, eo, MAX_KP, 3)
    with pytest.raises(ValueError):
        ymap.Map().insert_blocks(blk, 1, len(blk))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle_bind import Oracle
    from ya_vo_amd.sharding import shard_frames
    oracle = Oracle()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, every = 13, 2
    rel, ec, eX, eo = _sequence(oracle, n, 21)  # every rank draws the same sequence, keeps its own chunk
    s = shard_frames(n, world, rank)
    max_kf = max(ymap.max_keyframes(len(shard_frames(n, world, r).frames), shard_frames(n, world, r).start, every)
                 for r in range(world))
    a, b = s.start, s.end
    blk = oracle.map_chunk(rel[a:b], a, every, ec[a:b], eX[a:b], eo[a:b], MAX_KP, max_kf)
    gathered = ymap.gather_map_blocks(torch.from_numpy(blk), world).numpy()
    placed, end, _ = oracle.map_place(gathered, world, len(blk), np.array([0, 0, 0, 1, 0, 0, 0], np.float64))
    m = ymap.Map()
    m.insert_blocks(placed, world, len(blk))
    q.put((rank, {g: T.tolist() for g, T in m.get_frames().items()}, len(m.get_mps()), end.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_and_place_gloo_world2(oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    frames, n_mps, end = res[0]
    # the same sequence as one chunk in this process
    n, every = 13, 2
    rel, ec, eX, eo = _sequence(oracle, n, 21)
    one = oracle.map_chunk(rel, 0, every, ec, eX, eo, MAX_KP, ymap.max_keyframes(n, 0, every))
    ref, ref_end, _ = oracle.map_place(one, 1, len(one), np.array([0, 0, 0, 1, 0, 0, 0], np.float64))
    mref = ymap.Map()
    mref.insert_blocks(ref, 1, len(one))
    assert sorted(frames) == sorted(mref.get_frames()) and n_mps == len(mref.get_mps())
    for g, T in mref.get_frames().items():
        np.testing.assert_allclose(frames[g], T, atol=1e-12)
    np.testing.assert_allclose(end, ref_end, atol=1e-12)


def test_parse_block_views_are_read_only(oracle):
    """parse_block parses a uint8 buffer in place: its views alias the buffer, so writes through them are refused and
    a later reuse of the buffer shows through (ya_vo_amd/map.py docstring)."""
    rel, ec, eX, eo = _sequence(oracle, 3, 6)
    blk = oracle.map_chunk(rel, 0, 1, ec, eX, eo, MAX_KP, 3)
    h, kfs, lms = ymap.parse_block(blk)
    with pytest.raises(ValueError):
        lms[0]["X"][0] = 1.0
    with pytest.raises(ValueError):
        kfs["T"][0] = 0.0
    before = kfs["frame_id"].copy()
    blk[128:136] = 0xFF  # the caller reuses its buffer: the view follows it
    assert kfs["frame_id"][0] != before[0]
    assert blk.flags.writeable  # the caller's own array stays writable


def _shard_block(rng, oracle, first, n, max_kf, stride):
    """A sequence shard's export (yv_ba_window_export_block layout, placed = 2) built on the host: its own T_wc per
    frame (frame 0 of the shard at identity), X_w in the shard's frame, C = its last T_wc."""
    bb = ymap.block_bytes(max_kf, stride)
    raw = np.zeros(bb, np.uint8)
    T = [np.array([0, 0, 0, 1, 0, 0, 0], np.float64)]
    for _ in range(n - 1):
        T.append(oracle.se3_mul(T[-1], oracle.se3_exp(rng.normal(0, 0.05, 6))))
    h = raw[:128].view(ymap.HEADER_DTYPE)
    h["chunk"], h["first_frame"], h["n_frames"], h["n_kf"] = T[-1], first, n, n
    h["kf_every"], h["lm_stride"], h["max_kf"], h["placed"] = 1, stride, max_kf, 2
    kfs = raw[128:128 + 72 * max_kf].view(ymap.KEYFRAME_DTYPE)
    lmo = ymap.landmark_offset(max_kf)
    for j in range(n):
        c = int(rng.integers(0, stride))
        kfs[j]["frame_id"], kfs[j]["T"], kfs[j]["n_landmarks"] = first + j, T[j], c
        lm = raw[lmo + 32 * j * stride:lmo + 32 * (j * stride + c)].view(ymap.LANDMARK_DTYPE)
        lm["id"] = ((first + j) << 16) + np.arange(c)
        lm["X"] = rng.normal(0, 10, (c, 3))
    return raw


def test_place_sequence_shards(oracle):
    """yv_map_place on sequence-shard exports (placed = 2, SequenceShard): A_0 = base, A_{r+1} = A_r C_r, keyframes
    T_wc = A_r T, landmarks X_w = A_r X (the shard's own world frame, not a camera frame); placed becomes 3."""
    rng = np.random.default_rng(8)
    max_kf, stride = 6, 9
    blocks = [_shard_block(rng, oracle, 0, 6, max_kf, stride), _shard_block(rng, oracle, 6, 5, max_kf, stride),
              _shard_block(rng, oracle, 11, 4, max_kf, stride)]
    bb = len(blocks[0])
    base = oracle.se3_exp(rng.normal(0, 0.3, 6))
    placed, new_base, anchors = oracle.map_place(np.concatenate(blocks), 3, bb, base)
    A = base
    for r, raw in enumerate(blocks):
        h0, kf0, lm0 = ymap.parse_block(raw)
        h1, kf1, lm1 = ymap.parse_block(placed[r * bb:(r + 1) * bb])
        np.testing.assert_array_equal(anchors[r], A)
        assert int(h1["placed"]) == 3
        for j in range(int(h0["n_kf"])):
            np.testing.assert_array_equal(kf1[j]["T"], oracle.se3_mul(A, kf0[j]["T"]))
            np.testing.assert_array_equal(lm1[j]["id"], lm0[j]["id"])
            for a, b in zip(lm0[j]["X"], lm1[j]["X"]):
                np.testing.assert_array_equal(b, oracle.se3_act(A, a))
        A = oracle.se3_mul(A, h0["chunk"])
    np.testing.assert_array_equal(new_base, A)
    m = ymap.Map()
    m.insert_blocks(placed, 3, bb)  # a placed shard export reads as placed
    assert sorted(m.frames) == list(range(15))
