"""CPU restatement of ya_vo_amd.sequence.SequenceFrontend over the oracle -- test infrastructure only.

The same loop as the device front end (BASELINE configs[2]): per frame the oracle's FAST + BRIEF on L / R, the
temporal and stereo Matches with removeOutliers, stereo triangulation and the pose LM (tests/track_chain.py); per
chunk the oracle's map block and placement (oracle/yavo_oracle_map.c); then the oracle's BA (or_ba_lm) over the
same window. The window's host assembly is restated here (records_from_block / assemble_window / write_back, from
include/yavo/yavo_map.h's block layout and the window rule of ya_vo_amd/sequence.py's docstring), not imported from
the product, and SE3 inverses are the oracle's (or_se3_inverse): tests/test_sequence_host.py checks the product's
window_problem / apply_window against these.

ba_mode 0 runs the BA in the kernel's summation order (bit-exact with the device); 1 in g2o's own loop orders
(oracle/yavo_oracle_ba.c), the CPU reference the trajectory tolerance is measured against.
"""
import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from track_chain import track_pose

IDENTITY = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)


class Rec:
    """A frame's share of the map: T_wc and its landmarks (edge index, X_w, observation in frame k-1 / frame k)."""

    def __init__(self, T_wc, edge, X, uv_prev, uv_own):
        self.T_wc, self.edge, self.X, self.uv_prev, self.uv_own = T_wc, edge, X, uv_prev, uv_own


def records_from_block(block, edge_uv, edge_query, own_px):
    """A placed map block (yavo_map.h: 128-B header {chunk[7] f64, first_frame i64, n_frames, n_kf, kf_every,
    lm_stride, max_kf, placed i32}, max_kf 72-B keyframe records {frame_id i64, T[7] f64, n_landmarks i32, pad},
    landmark slots of 32 B {ptID i64, X[3] f64} from the first 256-B boundary after the keyframes, keyframe j's at
    slot j * lm_stride) -> {frame: Rec}. edge_uv [n, max_kp, 2] / edge_query [n, max_kp] per track of the chunk;
    own_px [n, max_kp, 2] = the frame's keypoint its query's temporal match picked (Matches::pt2)."""
    raw = bytes(np.ascontiguousarray(block).view(np.uint8))
    first = struct.unpack_from("<q", raw, 56)[0]
    n_kf, _, lm_stride, max_kf = struct.unpack_from("<iiii", raw, 68)
    lm0 = (128 + 72 * max_kf + 255) // 256 * 256
    out = {}
    for j in range(n_kf):
        o = 128 + 72 * j
        g = struct.unpack_from("<q", raw, o)[0]
        T = np.array(struct.unpack_from("<7d", raw, o + 8))
        n = struct.unpack_from("<i", raw, o + 64)[0]
        slots = np.frombuffer(raw, np.dtype([("id", "<i8"), ("X", "<f8", 3)]), n, lm0 + 32 * j * lm_stride)
        k = g - first
        edge = (slots["id"] & 0xFFFF).astype(np.int64)
        X = slots["X"].astype(np.float64)
        uv = np.asarray(edge_uv[k])[edge].astype(np.float64)
        own = np.asarray(own_px[k])[np.asarray(edge_query[k])[edge]].astype(np.float64)
        out[g] = Rec(T, edge, X, uv, own)
    return out


def assemble_window(orc, records, frames, n_fixed):
    """The BA problem over consecutive `frames`: pose i = frames[i] as T_cw; for every frame g whose predecessor
    g - 1 is in the window, each of its landmarks, in its record's order, becomes one landmark with two edges --
    (pose of g, its own keypoint), then (pose of g - 1, the PnP measurement). -> (poses, X, ep, el, meas, counts)."""
    poses = np.array([orc.se3_inverse(records[g].T_wc) for g in frames]).reshape(len(frames), 7)
    X, ep, el, meas, counts = [], [], [], [], []
    for i, g in enumerate(frames):
        r = records[g]
        if i == 0 or len(r.edge) == 0:
            counts.append(0)
            continue
        lo = sum(counts)
        for m in range(len(r.edge)):
            X.append(r.X[m])
        ep.extend([i] * len(r.edge) + [i - 1] * len(r.edge))
        el.extend(list(range(lo, lo + len(r.edge))) * 2)
        meas.extend(list(r.uv_own) + list(r.uv_prev))
        counts.append(len(r.edge))
    return (poses, np.array(X, np.float64).reshape(-1, 3), np.array(ep, np.int32), np.array(el, np.int32),
            np.array(meas, np.float64).reshape(-1, 2), counts)


def write_back(orc, records, frames, poses, X, counts):
    """Solved window -> records: T_wc = inverse(T_cw); frame frames[i] takes landmarks [sum(counts[:i]), + counts[i])."""
    lo = 0
    for i, g in enumerate(frames):
        records[g].T_wc = orc.se3_inverse(poses[i])
        if counts[i]:
            records[g].X = X[lo:lo + counts[i]].copy()
            lo += counts[i]


def oracle_sequence(orc, frames, chunk, K, T_right, offsets, n_fixed=2, ba_iters=10, max_kp=2000, threads=8,
                    ba_mode=0, tracks=None):
    """frames: [n, 2, H, W] (left, right). -> (trajectory [n, 7] T_wc, records, ba_log). tracks: the per-frame
    front end of an earlier call (`front_end`), reused."""
    if tracks is None:
        tracks = front_end(orc, frames, chunk, K, T_right, offsets, max_kp, threads)
    return sequence_from_tracks(orc, tracks, chunk, K, n_fixed, ba_iters, max_kp, ba_mode)


def front_end(orc, frames, chunk, K, T_right, offsets, max_kp=2000, threads=8):
    """Per frame: FAST + BRIEF on L / R, the temporal match and the pose LM (tests/track_chain.py)."""
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
        return list(ex.map(track, range(n_frames)))


def sequence_from_tracks(orc, tracks, chunk, K, n_fixed=2, ba_iters=10, max_kp=2000, ba_mode=0):
    """The map blocks, placement and BA windows over the per-frame tracks."""
    n_frames = len(tracks)
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
        records.update(records_from_block(placed, uv, qq, own))
        last = first + chunk - 1
        fr = list(range(max(0, last - window + 1), last + 1))
        poses, Xw, ep, el, meas, counts = assemble_window(orc, records, fr, n_fixed)
        if len(ep):
            P, Xo, it, log = orc.ba_lm(poses, n_fixed, Xw, ep, el, meas, K, ba_iters, mode=ba_mode)
            write_back(orc, records, fr, P, Xo, counts)
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
