"""CPU restatement of ya_vo_amd.sequence.SequenceFrontend over the oracle -- test infrastructure only.

The same loop as the device front end (BASELINE configs[2]): per frame the oracle's FAST + BRIEF on L / R, the
temporal and stereo Matches with removeOutliers, stereo triangulation and the pose LM (tests/track_chain.py); per
chunk the oracle's map block and placement (oracle/yavo_oracle_map.c); then the oracle's BA (or_ba_lm) over the
same window, assembled by the same host functions (ya_vo_amd.sequence.window_problem / apply_window).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from track_chain import track_pose
from ya_vo_amd.sequence import IDENTITY, apply_window, frame_records_from_block, window_problem


def oracle_sequence(orc, frames, chunk, K, T_right, offsets, n_fixed=2, ba_iters=10, max_kp=2000, threads=8):
    """frames: [n, 2, H, W] (left, right). -> (trajectory [n, 7] T_wc, records, ba_log)."""
    n_frames = len(frames)
    assert n_frames % chunk == 0

    def describe(img):
        return orc.brief(img, orc.fast(img, max_kp)[0], offsets)

    with ThreadPoolExecutor(threads) as ex:
        kl = list(ex.map(describe, [f[0] for f in frames]))
        kr = list(ex.map(describe, [f[1] for f in frames]))
    empty = kl[0][:0]

    def track(g):
        kq = kl[g - 1] if g > 0 else empty
        X, uv, q, T, out, inl = track_pose(orc, kq, kl[g], kr[g], K, T_right, n_tracks=chunk)  # chunk tracks per batch
        own = np.zeros((max_kp, 2), np.int32)
        if len(kq):
            mt = orc.match(kq, kl[g])
            own[:len(mt), 0] = mt["pt2"]["x"]
            own[:len(mt), 1] = mt["pt2"]["y"]
        return X, uv, q, T, out, own

    with ThreadPoolExecutor(threads) as ex:
        tracks = list(ex.map(track, range(n_frames)))

    records, ba_log = {}, []
    base = IDENTITY.copy()
    window = chunk + n_fixed
    for c in range(n_frames // chunk):
        first = c * chunk
        rel = np.zeros((chunk, 7))
        ec = np.zeros(chunk, np.int32)
        eX = np.zeros((chunk, max_kp, 3))
        eo = np.zeros((chunk, max_kp), np.uint8)
        uv = np.zeros((chunk, max_kp, 2))
        qq = np.zeros((chunk, max_kp), np.int32)
        own = np.zeros((chunk, max_kp, 2), np.int32)
        for k in range(chunk):
            X, u, q, T, out, o = tracks[first + k]
            rel[k] = T
            ec[k] = len(X)
            eX[k, :len(X)] = X
            eo[k, :len(X)] = out
            uv[k, :len(X)] = u
            qq[k, :len(X)] = q
            own[k] = o
        block = orc.map_chunk(rel, first, 1, ec, eX, eo, max_kp, chunk)
        placed, base, _ = orc.map_place(block, 1, len(block), base)
        records.update(frame_records_from_block(placed, uv, qq, own))
        last = first + chunk - 1
        fr = list(range(max(0, last - window + 1), last + 1))
        poses, Xw, ep, el, meas, owners = window_problem(records, fr, n_fixed)
        if len(ep):
            P, Xo, it, log = orc.ba_lm(poses, n_fixed, Xw, ep, el, meas, K, ba_iters)
            apply_window(records, fr, P, Xo, owners)
            ba_log.append((last, it, float(log[0]), float(log[-1])))
            base = records[last].T_wc.copy()
    traj = np.stack([records[g].T_wc for g in sorted(records)])
    return traj, records, ba_log


def rmse_translation(A, B) -> float:
    d = np.asarray(A)[:, 4:] - np.asarray(B)[:, 4:]
    return float(np.sqrt(np.mean(np.sum(d * d, axis=1)))) if len(d) else 0.0


def ground_truth(n_frames, K):
    """The synthetic sequence's trajectory: frame k is the crop at (k, 3k) of one fronto-parallel textured plane at
    Z = 0.54 fy / 8 (stereo disparity 8 px), so T_wc(k) is a pure translation by k (Z / fx, 3 Z / fy, 0)."""
    Z = 0.54 * K[1][1] / 8.0
    step = np.array([Z / K[0][0], 3.0 * Z / K[1][1], 0.0])
    return np.stack([np.concatenate([[0, 0, 0, 1.0], k * step]) for k in range(n_frames)])
