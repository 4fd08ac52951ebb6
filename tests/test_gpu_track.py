"""GPU parity of the batch's track stage (yv_batch_set_tracks / yv_batch_track): stereo triangulation of
the kept matches and the per-frame pose LM, bit for bit against the oracle chain in tests/track_chain.py,
over two chained runs (the first track of each run reads the carry slot)."""
import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd import scene
from ya_vo_amd.synth import synth_frame

from track_chain import IDENTITY, track_pose

pytestmark = pytest.mark.gpu

H, W = 376, 1241
T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)  # right camera 0.54 m along the column axis


def _setup(ctx, n_frames):
    b = yv.Batch(ctx, 2 * n_frames, H, W, 2000, 2 * n_frames)
    carry = 2 * n_frames
    pairs, tracks = [], []
    for k in range(n_frames):
        pairs.append((carry if k == 0 else 2 * (k - 1), 2 * k))  # temporal L_{k-1} -> L_k
        pairs.append((2 * k, 2 * k + 1))                          # stereo L_k -> R_k
        tracks.append((2 * k + 1, 2 * k))
    b.set_pairs(pairs)
    b.set_tracks(tracks, scene.K_KITTI, T_RIGHT)
    return b, carry


@pytest.mark.parametrize("overlap", [0, 1, 2, 3])
def test_track_matches_oracle(ctx, oracle, offsets, overlap):
    import torch
    n_frames = 3
    b, carry = _setup(ctx, n_frames)
    b.set_track_overlap(overlap)
    seq = [(synth_frame(51, k, 3 * k), synth_frame(51, k, 3 * k + 8)) for k in range(2 * n_frames)]
    d_prior = torch.from_numpy(np.tile(IDENTITY, (n_frames, 1))).to("cuda:0")
    d_pose = torch.zeros((n_frames, 7), dtype=torch.float64, device="cuda:0")
    kps = {}
    prev_left = None
    b.enable_timing(True)
    for run in range(2):
        frames = np.stack([im for k in range(run * n_frames, (run + 1) * n_frames) for im in seq[k]])
        d = torch.from_numpy(frames).to("cuda:0")
        torch.cuda.synchronize()
        b.run(d.data_ptr(), len(frames), W, H * W, 20, carry_from=2 * (n_frames - 1))
        b.track(d_prior.data_ptr(), d_pose.data_ptr())
        ctx.sync()
        b.track_sync()
        v = b.view()
        assert v.n_tracks == n_frames
        for i, img in enumerate(frames):
            kps[i] = oracle.brief(img, oracle.fast(img, 2000)[0], offsets)
        cnt = ctx.download(v.edge_count, np.int32, n_frames)
        inl = ctx.download(v.track_inliers, np.int32, n_frames)
        P = d_pose.cpu().numpy()
        for k in range(n_frames):
            kq = (prev_left if prev_left is not None else kps[0][:0]) if k == 0 else kps[2 * (k - 1)]
            X, uv, q, T, out, oinl = track_pose(oracle, kq, kps[2 * k], kps[2 * k + 1], scene.K_KITTI, T_RIGHT,
                                                n_tracks=n_frames)
            assert cnt[k] == len(X), (run, k)
            base = k * 2000
            gX = ctx.download(v.edge_X + base * 24, np.float64, 3 * cnt[k]).reshape(-1, 3)
            guv = ctx.download(v.edge_uv + base * 16, np.float64, 2 * cnt[k]).reshape(-1, 2)
            gq = ctx.download(v.edge_query + base * 4, np.int32, cnt[k])
            gout = ctx.download(v.edge_outlier + base, np.uint8, cnt[k]).astype(bool)
            np.testing.assert_array_equal(gq, q)
            np.testing.assert_array_equal(gX, X)
            np.testing.assert_array_equal(guv, uv)
            assert inl[k] == oinl
            np.testing.assert_array_equal(gout, out)
            np.testing.assert_array_equal(P[k], T)
            if len(X) >= 100:
                # the synthetic motion: frame k-1 is frame k's content shifted by (+1 row, +3 cols); the
                # stereo disparity is 8 px, so every point lies at Z = 0.54 fy / 8 and the pose of frame
                # k-1 in frame k is the translation (Z / fx, 3 Z / fy, 0) = (0.0675, 0.2025, 0)
                np.testing.assert_allclose(T[4:], [0.0675, 0.2025, 0.0], atol=2e-3)
                np.testing.assert_allclose(np.abs(T[3]), 1.0, atol=1e-4)
        prev_left = kps[2 * (n_frames - 1)]
    ms, nruns = b.stage_times()
    assert nruns == 2 and np.all(ms > 0)  # every stage, incl. track_edges / track_pose, was timed
    b.close()


def test_track_rejects_inconsistent_pairs(ctx):
    b = yv.Batch(ctx, 4, H, W, 2000, 4)
    b.set_pairs([(0, 1), (2, 3)])
    with pytest.raises(yv.YavoError):
        b.set_tracks([(0, 1)], scene.K_KITTI, T_RIGHT)  # stereo query 0 != temporal train 3
    with pytest.raises(yv.YavoError):
        b.set_tracks([(0, 5)], scene.K_KITTI, T_RIGHT)  # pair index out of range
    b.close()


@pytest.mark.parametrize("build_async", ["1", "0"])
def test_track_overlap_pipelined(ctx, oracle, offsets, monkeypatch, build_async):
    """Overlap mode without any host synchronization between steps: four run + track steps back to back
    (the LM of step i beside the kernels of step i + 1, the three edge buffers wrapping; with build_async the
    edge build of step i also runs beside step i + 1's detect and the carry-slot copy waits for it); every
    step's poses, read after one final sync, equal the oracle chain's."""
    import torch
    monkeypatch.setenv("YAVO_BUILD_ASYNC", build_async)  # read by yv_batch_set_track_overlap
    n_frames, steps = 2, 4
    b, carry = _setup(ctx, n_frames)
    b.set_track_overlap(True)
    seq = [(synth_frame(61, k, 3 * k), synth_frame(61, k, 3 * k + 8)) for k in range(n_frames * steps)]
    d_prior = torch.from_numpy(np.tile(IDENTITY, (n_frames, 1))).to("cuda:0")
    d_poses = [torch.zeros((n_frames, 7), dtype=torch.float64, device="cuda:0") for _ in range(steps)]
    frames = [np.stack([im for k in range(i * n_frames, (i + 1) * n_frames) for im in seq[k]]) for i in range(steps)]
    d_frames = [torch.from_numpy(f).to("cuda:0") for f in frames]
    torch.cuda.synchronize()
    for i in range(steps):
        b.run(d_frames[i].data_ptr(), 2 * n_frames, W, H * W, 20, carry_from=2 * (n_frames - 1))
        b.track(d_prior.data_ptr(), d_poses[i].data_ptr())
    ctx.sync()
    b.track_sync()
    kp = [[oracle.brief(im, oracle.fast(im, 2000)[0], offsets) for im in f] for f in frames]
    for i in range(steps):
        P = d_poses[i].cpu().numpy()
        for k in range(n_frames):
            if k == 0:
                kq = kp[i - 1][2 * (n_frames - 1)] if i > 0 else kp[0][0][:0]
            else:
                kq = kp[i][2 * (k - 1)]
            T = track_pose(oracle, kq, kp[i][2 * k], kp[i][2 * k + 1], scene.K_KITTI, T_RIGHT, n_tracks=n_frames)[3]
            np.testing.assert_array_equal(P[k], T)
    b.close()


def test_track_lk_mode_matches_oracle(ctx, oracle, offsets):
    """LK tracking mode (the reference's trackLastFrame): frame k-1's stereo map points tracked into frame k by
    calcOpticalFlowPyrLK, then the pose LM; edges and poses bit for bit against tests/track_chain.py."""
    import torch
    from track_chain import lk_track_pose
    n_frames = 3
    b = yv.Batch(ctx, 2 * n_frames, H, W, 2000, 2 * n_frames)
    carry = 2 * n_frames
    pairs = []
    for k in range(n_frames):
        pairs.append((carry if k == 0 else 2 * (k - 1), 2 * k))
        pairs.append((2 * k, 2 * k + 1))
    b.set_pairs(pairs)
    b.set_track_lk(2)
    tracks = [(2 * (k - 1) + 1, 2 * k) for k in range(1, n_frames)]  # {stereo pair of k-1, image of L_k}
    b.set_tracks(tracks, scene.K_KITTI, T_RIGHT)
    frames = np.stack([im for k in range(n_frames) for im in (synth_frame(71, k, 3 * k), synth_frame(71, k, 3 * k + 8))])
    d = torch.from_numpy(frames).to("cuda:0")
    nt = len(tracks)
    d_prior = torch.from_numpy(np.tile(IDENTITY, (nt, 1))).to("cuda:0")
    d_pose = torch.zeros((nt, 7), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    b.run(d.data_ptr(), len(frames), W, H * W, 20)
    b.track(d_prior.data_ptr(), d_pose.data_ptr())
    ctx.sync()
    v = b.view()
    kps = [oracle.brief(im, oracle.fast(im, 2000)[0], offsets) for im in frames]
    cnt = ctx.download(v.edge_count, np.int32, nt)
    P = d_pose.cpu().numpy()
    for t, k in enumerate(range(1, n_frames)):
        X, uv, q, T, out, inl = lk_track_pose(oracle, frames[2 * (k - 1)], frames[2 * k], kps[2 * (k - 1)],
                                              kps[2 * (k - 1) + 1], scene.K_KITTI, T_RIGHT, n_tracks=nt)
        assert cnt[t] == len(X) > 500
        base = t * 2000
        np.testing.assert_array_equal(ctx.download(v.edge_X + base * 24, np.float64, 3 * cnt[t]).reshape(-1, 3), X)
        np.testing.assert_array_equal(ctx.download(v.edge_uv + base * 16, np.float64, 2 * cnt[t]).reshape(-1, 2), uv)
        np.testing.assert_array_equal(ctx.download(v.edge_query + base * 4, np.int32, cnt[t]), q)
        np.testing.assert_array_equal(P[t], T)
        # frame k is frame k-1 shifted by (1, 3) px, the stereo points sit at Z = 0.54 fy / 8: the pose of frame
        # k in frame k-1's camera is the translation (-Z/fx, -3 Z/fy, 0).  The reference truncates the LK points
        # to int (cv::Point2i(float), src/LoopHandler.cc:395): LK lands within ~0.01 px of the integer truth, so
        # truncation biases the measurements by up to 1 px = 0.07 m at this depth
        np.testing.assert_allclose(T[4:], [-0.0675, -0.2025, 0.0], atol=0.07)
    b.close()


def test_frame_shard_lk_halo_tracks_the_boundary_pair(ctx, oracle, offsets):
    """FrameShard in LK mode with a halo: the halo frame's stereo pair seeds track 0 (halo frame -> first frame), so
    a multi-rank LK trajectory loses no pose at a rank boundary; every track bit for bit against lk_track_pose."""
    import torch
    from track_chain import lk_track_pose
    from ya_vo_amd.sharding import FrameShard, shard_images
    B, first = 3, 5
    seq = [(synth_frame(81, k, 3 * k), synth_frame(81, k, 3 * k + 8)) for k in range(first - 1, first + B)]
    images = shard_images(np.stack([im for fr in seq[1:] for im in fr]), seq[0][0], seq[0][1])
    shard = FrameShard(ctx, B, first, scene.K_KITTI, T_RIGHT, halo=True, tracker="lk", overlap_mode=0)
    assert shard.n_tracks == B and shard.n_images == 2 * B + 2
    d = torch.from_numpy(images).to("cuda:0")
    torch.cuda.synchronize()
    shard.step(d.data_ptr())
    shard.drain()
    P = shard.poses()
    kps = [(oracle.brief(L, oracle.fast(L, 2000)[0], offsets), oracle.brief(R, oracle.fast(R, 2000)[0], offsets))
           for L, R in seq]
    for k in range(B):  # track k: frame first + k - 1 (seq[k]) -> frame first + k (seq[k + 1])
        T = lk_track_pose(oracle, seq[k][0], seq[k + 1][0], kps[k][0], kps[k][1], scene.K_KITTI, T_RIGHT,
                          n_tracks=shard.n_tracks)[3]
        np.testing.assert_array_equal(P[k], T, err_msg=f"track {k}")
    shard.close()


def test_lk_overlap_pipelined_matches_serial(ctx):
    """LK mode with the asynchronous build (overlap on): the LK stage of step i runs beside step i + 1's run, its
    stereo points in the other of two point sets; every step's poses equal the serial mode's bit for bit."""
    import torch
    n_frames, steps = 3, 4
    frames = [np.stack([im for k in range(n_frames) for im in (synth_frame(91 + s, k, 3 * k), synth_frame(91 + s, k, 3 * k + 8))])
              for s in range(steps)]
    d = [torch.from_numpy(f).to("cuda:0") for f in frames]
    tracks = [(2 * (k - 1) + 1, 2 * k) for k in range(1, n_frames)]
    nt = len(tracks)
    out = []
    for overlap in (0, 1):
        b = yv.Batch(ctx, 2 * n_frames, H, W, 2000, 2 * n_frames)
        carry = 2 * n_frames
        pairs = []
        for k in range(n_frames):
            pairs.append((carry if k == 0 else 2 * (k - 1), 2 * k))
            pairs.append((2 * k, 2 * k + 1))
        b.set_pairs(pairs)
        b.set_track_lk(2)
        b.set_tracks(tracks, scene.K_KITTI, T_RIGHT)
        b.set_track_overlap(overlap)
        d_prior = torch.from_numpy(np.tile(IDENTITY, (nt, 1))).to("cuda:0")
        poses = [torch.zeros((nt, 7), dtype=torch.float64, device="cuda:0") for _ in range(steps)]
        torch.cuda.synchronize()
        for s in range(steps):
            b.run(d[s].data_ptr(), 2 * n_frames, W, H * W, 20)
            b.track(d_prior.data_ptr(), poses[s].data_ptr())
        b.track_sync()
        ctx.sync()
        torch.cuda.synchronize()
        out.append(np.stack([p.cpu().numpy() for p in poses]))
        b.close()
    assert np.all(np.isfinite(out[0])) and np.abs(out[0][:, :, 4]).max() > 0.01
    np.testing.assert_array_equal(out[1], out[0])
