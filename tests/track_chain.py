"""CPU restatement of the batch's track stage (yv_batch_track) composed from oracle rows -- test
infrastructure, used by tests/test_gpu_track.py and bench.py's cpu_baseline leg as the checker.

Track for frame k: temporal Matches L_{k-1} -> L_k and stereo Matches L_k -> R_k (Brief::matchFeatures +
removeOutliers, src/BriefDescriptor.cc:163-231), stereo triangulation with the left camera as world
(LoopHandler::triangulation + triangulate2View's Z > 0, src/LoopHandler.cc:658-726, 867-885), then
LoopHandler::optimizePoseOnly (src/LoopHandler.cc:730-861) of frame k-1's pose in frame k's camera from
the frame-(k-1) measurements.
"""
import time

import numpy as np

from ya_vo_amd import MATCH_DTYPE, lm_sum_mode, track_lm_sum_mode


def lm_sum_mode_default(n_tracks=None):
    """The batch track LM's edge-sum order for a batch of n_tracks tracks (yv_track_lm_sum_mode: 512-thread
    workgroups up to 256 tracks); None: a batch of more than 256 (yv_lm_sum_mode)."""
    return lm_sum_mode() if n_tracks is None else track_lm_sum_mode(n_tracks)

IDENTITY = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)


def kept_flags(orc, m, thr=20):
    """removeOutliers as per-record keep flags (pt1.id is unique within the query image)."""
    if len(m) == 0:
        return np.zeros(0, bool)
    kept_ids = set(orc.remove_outliers(m, thr)["pt1"]["id"].tolist())
    return np.array([i in kept_ids for i in m["pt1"]["id"].tolist()], bool)


def _tick(timers, key, t0):
    """Accumulate seconds since t0 under `key` (timers None: no timing); returns the new start."""
    t = time.perf_counter()
    if timers is not None:
        timers[key] = timers.get(key, 0.0) + t - t0
    return t


def f_ransac_seconds(orc, matches, iters=400, thr=0.1, seed=0):
    """Seconds of the oracle's getFRANSAC (src/3DHandler.cc:145-195: `iters` hypotheses of 8 draws with replacement,
    |p2^T F p1| < thr) on a kept match list: the reference runs it at (re)initialisation (buildInitMap /
    reinitialize, src/LoopHandler.cc:225,567), not per tracked frame."""
    if len(matches) < 8:
        return 0.0
    samples = np.random.default_rng(seed).integers(0, len(matches), (iters, 8)).astype(np.int32)
    t0 = time.perf_counter()
    orc.f_ransac(matches, samples, thr)
    return time.perf_counter() - t0


def track_edges(orc, kq, kl, kr, K, T_right, thr=20, timers=None, init_timers=None):
    """Edges of one track -> (X [n,3], uv [n,2], query index [n]).  timers: optional dict of per-stage seconds
    ("match": matchFeatures + removeOutliers of both pairs, "triangulate": the stereo triangulation).  init_timers:
    optional dict that gets "f_ransac", the (re)initialisation stage timed on this track's kept temporal matches
    (outside `timers`)."""
    if len(kq) == 0:
        return np.zeros((0, 3)), np.zeros((0, 2)), np.zeros(0, np.int32)
    t0 = time.perf_counter()
    mt = orc.match(kq, kl)
    ms = orc.match(kl, kr) if len(kl) else np.zeros(0, MATCH_DTYPE)
    kt, ks = kept_flags(orc, mt, thr), kept_flags(orc, ms, thr)
    t0 = _tick(timers, "match", t0)
    if init_timers is not None:
        init_timers["f_ransac"] = init_timers.get("f_ransac", 0.0) + f_ransac_seconds(orc, mt[kt])
        t0 = time.perf_counter()
    l_index = {int(i): j for j, i in enumerate(kl["id"].tolist())}
    cand, recs = [], []
    for i in range(len(kq)):
        if not kt[i] or len(kl) == 0:
            continue
        j = l_index[int(mt[i]["pt2"]["id"])]
        if not ks[j]:
            continue
        cand.append(i)
        recs.append(ms[j])
    if not cand:
        return np.zeros((0, 3)), np.zeros((0, 2)), np.zeros(0, np.int32)
    _, X, ok = orc.triangulate_matches(IDENTITY, T_right, K, np.array(recs, MATCH_DTYPE))
    _tick(timers, "triangulate", t0)
    q = np.array(cand, np.int32)[ok]
    uv = np.stack([kq["x"][q], kq["y"][q]], 1).astype(np.float64)
    return X[ok], uv, q


def track_pose(orc, kq, kl, kr, K, T_right, prior=IDENTITY, thr=20, sum_mode=None, timers=None, init_timers=None,
               n_tracks=None):
    """track_edges + optimizePoseOnly in `sum_mode` (None: the GPU kernel's order for a batch of n_tracks tracks,
    lm_sum_mode_default; 0: the reference's sequential order).  timers: as track_edges, plus "pose_lm"; init_timers:
    as track_edges."""
    if sum_mode is None:
        sum_mode = lm_sum_mode_default(n_tracks)
    X, uv, q = track_edges(orc, kq, kl, kr, K, T_right, thr, timers, init_timers)
    t0 = time.perf_counter()
    T, out, inl = orc.pose_lm(X, uv, K, prior, sum_mode)
    _tick(timers, "pose_lm", t0)
    return X, uv, q, T, out, inl


def lk_track_pose(orc, img_prev, img_next, kl, kr, K, T_right, prior=IDENTITY, thr=20, lk_sum_mode=1,
                  lm_sum_mode=None, n_tracks=None):
    """The reference's trackLastFrame + optimizePoseOnly (src/LoopHandler.cc:298-454, 730-861) with frame k-1's
    map points from its stereo pair: kept stereo matches triangulated (left camera = world), tracked by
    calcOpticalFlowPyrLK into frame k, status-1 points at cv::Point2i(next.y, next.x) (truncation).
    lm_sum_mode None: the GPU kernel's order for a batch of n_tracks tracks (lm_sum_mode_default).
    -> (X [n,3], uv [n,2], query index [n], T, outlier, inliers)."""
    if lm_sum_mode is None:
        lm_sum_mode = lm_sum_mode_default(n_tracks)
    if len(kl) == 0:
        e = np.zeros((0, 3)), np.zeros((0, 2)), np.zeros(0, np.int32)
        return (*e, *orc.pose_lm(e[0], e[1], K, prior, lm_sum_mode))
    ms = orc.match(kl, kr) if len(kr) else np.zeros(0, MATCH_DTYPE)
    ks = kept_flags(orc, ms, thr) if len(kr) else np.zeros(len(kl), bool)
    js = np.nonzero(ks)[0]
    X = np.zeros((0, 3))
    q = np.zeros(0, np.int32)
    if len(js):
        _, Xa, ok = orc.triangulate_matches(IDENTITY, T_right, K, ms[js])
        X, q = Xa[ok], js[ok].astype(np.int32)
    pts = np.stack([kl["y"][q], kl["x"][q]], 1).astype(np.float32)  # (x = column, y = row)
    nxt, st, _, _ = orc.lk(img_prev, img_next, pts, sum_mode=lk_sum_mode)
    uv = np.stack([np.trunc(nxt[st, 1]), np.trunc(nxt[st, 0])], 1).astype(np.float64)
    X, q = X[st], q[st]
    T, out, inl = orc.pose_lm(X, uv, K, prior, lm_sum_mode)
    return X, uv, q, T, out, inl
