"""GPU parity of the shared map (include/yavo/yavo_map.h): the chunk block yv_batch_track_map writes after the
pose LM and the placement yv_map_place runs after the all-gather, byte for byte against the oracle
(oracle/yavo_oracle_map.c) fed with the GPU's own edges and poses (whose parity tests/test_gpu_track.py holds)."""
import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd import map as ymap
from ya_vo_amd import scene
from ya_vo_amd.synth import synth_frame

pytestmark = pytest.mark.gpu

H, W, MAX_KP = 376, 1241, 2000
T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
IDENTITY = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)


def _setup(ctx, n_frames):
    b = yv.Batch(ctx, 2 * n_frames, H, W, MAX_KP, 2 * n_frames)
    carry = 2 * n_frames
    pairs, tracks = [], []
    for k in range(n_frames):
        pairs.append((carry if k == 0 else 2 * (k - 1), 2 * k))
        pairs.append((2 * k, 2 * k + 1))
        tracks.append((2 * k + 1, 2 * k))
    b.set_pairs(pairs)
    b.set_tracks(tracks, scene.K_KITTI, T_RIGHT)
    return b


def _edges(ctx, b, n):
    v = b.view()
    ec = ctx.download(v.edge_count, np.int32, n)
    eX = ctx.download(v.edge_X, np.float64, n * MAX_KP * 3).reshape(n, MAX_KP, 3)
    eo = ctx.download(v.edge_outlier, np.uint8, n * MAX_KP).reshape(n, MAX_KP)
    return ec, eX, eo


@pytest.mark.parametrize("overlap", [0, 1, 2, 3])
def test_map_blocks_and_place_match_oracle(ctx, oracle, overlap):
    import torch
    n, every = 4, 2
    b = _setup(ctx, n)
    b.set_track_overlap(overlap)
    max_kf = 2
    bb = ymap.block_bytes(max_kf, MAX_KP)
    assert bb == ctx.lib.yv_map_block_bytes(max_kf, MAX_KP)
    d_prior = torch.from_numpy(np.tile(IDENTITY, (n, 1))).to("cuda:0")
    d_pose = torch.zeros((n, 7), dtype=torch.float64, device="cuda:0")
    side = torch.cuda.Stream()
    blocks, copies = [], []
    d_block = torch.zeros(bb, dtype=torch.uint8, device="cuda:0")
    for run in range(2):
        first = 1 + run * n  # frame 0 is the carry slot's predecessor: chunks start at 1, 5
        frames = np.stack([im for k in range(first, first + n) for im in (synth_frame(52, k, 3 * k),
                                                                           synth_frame(52, k, 3 * k + 8))])
        d = torch.from_numpy(frames).to("cuda:0")
        torch.cuda.synchronize()
        b.run(d.data_ptr(), len(frames), W, H * W, 20, carry_from=2 * (n - 1))
        b.track_map(d_prior.data_ptr(), d_pose.data_ptr(), first, every, d_block.data_ptr(), max_kf)
        # a reader on another stream orders itself after the block and releases it for the next write
        b.map_wait(side.cuda_stream)
        with torch.cuda.stream(side):
            copies.append(d_block.clone())
        b.map_release(side.cuda_stream)
        ctx.sync()
        b.track_sync()
        torch.cuda.synchronize()
        ec, eX, eo = _edges(ctx, b, n)
        rel = d_pose.cpu().numpy()
        ref = oracle.map_chunk(rel, first, every, ec, eX, eo, MAX_KP, max_kf)
        got = copies[-1].cpu().numpy()
        h, kfs, lms = ymap.parse_block(got)
        rh, rkfs, rlms = ymap.parse_block(ref)
        np.testing.assert_array_equal(kfs, rkfs, err_msg=f"run {run}: keyframe records")
        for j in range(len(rkfs)):
            np.testing.assert_array_equal(lms[j]["id"], rlms[j]["id"], err_msg=f"run {run}: kf {j} landmark ids")
            np.testing.assert_array_equal(lms[j]["X"], rlms[j]["X"], err_msg=f"run {run}: kf {j} landmark X")
        np.testing.assert_array_equal(np.frombuffer(h.tobytes(), np.uint8), np.frombuffer(rh.tobytes(), np.uint8),
                                      err_msg=f"run {run}: header {h} vs {rh}")
        if run == 0:  # a zeroed block: every byte (later runs leave stale slots past each keyframe's count)
            np.testing.assert_array_equal(got, ref)
        assert int(h["n_kf"]) == ymap.max_keyframes(n, first, every)
        assert sum(len(x) for x in lms) > 0
        blocks.append(got)
    empty = oracle.map_chunk(np.zeros((0, 7)), 9, every, np.zeros(0, np.int32), np.zeros((0, MAX_KP, 3)),
                             np.zeros((0, MAX_KP), np.uint8), MAX_KP, max_kf)
    gathered = np.concatenate([blocks[0], empty, blocks[1]])
    base = oracle.se3_exp(np.array([0.3, -0.1, 2.0, 0.01, 0.02, -0.03]))
    ref, ref_base, ref_anchors = oracle.map_place(gathered, 3, bb, base)
    d_all = torch.from_numpy(gathered).to("cuda:0")
    d_base = torch.from_numpy(base.copy()).to("cuda:0")
    d_anchors = torch.zeros((3, 7), dtype=torch.float64, device="cuda:0")
    ctx.map_place(d_all.data_ptr(), 3, bb, d_base.data_ptr(), d_anchors.data_ptr(),
                  stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_all.cpu().numpy(), ref)
    np.testing.assert_array_equal(d_base.cpu().numpy(), ref_base)
    np.testing.assert_array_equal(d_anchors.cpu().numpy(), ref_anchors)
    m = ymap.Map()
    m.insert_blocks(ref, 3, bb)
    assert sorted(m.get_frames()) == [2, 4, 6, 8]
    b.close()


def test_map_rejects_bad_arguments(ctx):
    import torch
    b = _setup(ctx, 2)
    d = torch.zeros(16, dtype=torch.float64, device="cuda:0")
    with pytest.raises(yv.YavoError):
        b.track_map(d.data_ptr(), d.data_ptr(), 0, 0, d.data_ptr(), 1)  # kf_every < 1
    with pytest.raises(yv.YavoError):
        ctx.map_place(d.data_ptr(), 1, 100, d.data_ptr(), d.data_ptr())  # block size not a 256-B multiple
    b.close()
