"""The full front end over a stereo sequence (BASELINE configs[2]: "full Frontend incl. 3DHandler PnP + local-BA
Optimizer, first 200 frames"), driven the way LoopHandler drives its loop (src/LoopHandler.cc:60-165):

  per chunk of B stereo frames, on the device (one yv_batch, carry slot = the previous chunk's last frame):
    detect + describe L / R, match L_{k-1} -> L_k and L_k -> R_k, removeOutliers(20)  (yv_batch_run)
    stereo triangulation + pose-only LM per frame, the chunk's map block              (yv_batch_track_map)
    placement of the block in world coordinates after the previous chunk             (yv_map_place)
  then the local BA (the keyframe window the reference's Optimizer::partialBA stands for, src/Optimizer.cc:17-60,
  solved as g2o's BlockSolver_6_3 LM would, yv_ba) over the chunk's frames plus the `n_fixed` frames before it
  (held fixed: they were refined with the previous chunk and pin the gauge and the scale): every landmark of frame k
  (its pose-LM inliers, X_w from the map) observed in frame k (its left keypoint) and frame k-1 (the PnP
  measurement); the refined poses replace the trajectory's and the last one anchors the next chunk.

Host logic only (the window assembly and SE3 inversion are numpy); every compute step is a libyavo kernel.
tests/sequence_chain.py restates the same loop over the CPU oracle for the trajectory check.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np

from . import map as ymap

IDENTITY = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)


def se3_inverse(T) -> np.ndarray:
    """Sophus SE3d::inverse on data() = {qx, qy, qz, qw, tx, ty, tz}: SO3(q*) (renormalised by the SO3 constructor,
    |q| summed as Eigen's squaredNorm pairs it) and that rotation applied to -t as Eigen's Quaternion * Vector3 does
    (uv = 2 (q.vec x v); v + w uv + q.vec x uv) -- oracle/yavo_oracle_geom.c or_se3_inverse's arithmetic, in scalar
    IEEE doubles, which the device restatement (yavo_ba.hip se3_inverse_dev, no contraction) repeats bit for bit."""
    x, y, z, w = -float(T[0]), -float(T[1]), -float(T[2]), float(T[3])
    n = math.sqrt((x * x + z * z) + (y * y + w * w))
    x, y, z, w = x / n, y / n, z / n, w / n
    vx, vy, vz = float(T[4]) * -1.0, float(T[5]) * -1.0, float(T[6]) * -1.0
    ux, uy, uz = y * vz - z * vy, z * vx - x * vz, x * vy - y * vx
    ux, uy, uz = ux + ux, uy + uy, uz + uz
    cx, cy, cz = y * uz - z * uy, z * ux - x * uz, x * uy - y * ux
    return np.array([x, y, z, w, vx + w * ux + cx, vy + w * uy + cy, vz + w * uz + cz])


@dataclass
class FrameRecord:
    """One frame's share of the map: T_wc, its landmarks (edge index, X_w) and their two observations."""
    T_wc: np.ndarray
    edge: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    X: np.ndarray = field(default_factory=lambda: np.zeros((0, 3)))
    uv_prev: np.ndarray = field(default_factory=lambda: np.zeros((0, 2)))  # in frame k-1 (the PnP measurement)
    uv_own: np.ndarray = field(default_factory=lambda: np.zeros((0, 2)))   # in frame k (its left keypoint)


def frame_records_from_block(block: np.ndarray, edge_uv: np.ndarray, edge_query: np.ndarray,
                             own_px: np.ndarray) -> Dict[int, FrameRecord]:
    """Placed map block + the chunk's edge arrays -> per-frame records. edge_uv [n, max_kp, 2] and edge_query
    [n, max_kp] per track (track k = frame first_frame + k); own_px [n, max_kp, 2] = the frame-k keypoint the
    query's temporal match selected (Matches::pt2, row / col)."""
    h, kfs, lms = ymap.parse_block(block)
    first = int(h["first_frame"])
    out = {}
    for kf, lm in zip(kfs, lms):
        g = int(kf["frame_id"])
        k = g - first
        e = (lm["id"] & 0xFFFF).astype(np.int64)
        q = edge_query[k, e]
        out[g] = FrameRecord(np.array(kf["T"], np.float64), e, np.array(lm["X"], np.float64),
                             edge_uv[k, e].astype(np.float64), own_px[k, q].astype(np.float64))
    return out


def window_problem(records: Dict[int, FrameRecord], frames: List[int], n_fixed: int):
    """BA problem over consecutive `frames` (oldest first): poses T_cw, landmarks of frames whose predecessor is in
    the window (two observations each), edges (pose index, landmark index, meas). -> (poses, X, ep, el, meas,
    landmark owner [(frame, count)])."""
    index = {g: i for i, g in enumerate(frames)}
    poses = np.stack([se3_inverse(records[g].T_wc) for g in frames])
    Xs, ep, el, meas, owners = [], [], [], [], []
    base = 0
    for g in frames:
        r = records[g]
        n = len(r.edge)
        if g - 1 not in index or n == 0:
            owners.append((g, 0))
            continue
        ids = np.arange(base, base + n, dtype=np.int32)
        Xs.append(r.X)
        ep += [np.full(n, index[g], np.int32), np.full(n, index[g - 1], np.int32)]
        el += [ids, ids]
        meas += [r.uv_own, r.uv_prev]
        owners.append((g, n))
        base += n
    if not Xs:
        return poses, np.zeros((0, 3)), np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros((0, 2)), owners
    return (poses, np.concatenate(Xs), np.concatenate(ep), np.concatenate(el), np.concatenate(meas), owners)


def apply_window(records: Dict[int, FrameRecord], frames: List[int], poses: np.ndarray, X: np.ndarray,
                 owners) -> None:
    """Write a solved window back: T_wc = inverse(T_cw) per frame, refined landmarks per owning frame."""
    for g, T in zip(frames, poses):
        records[g].T_wc = se3_inverse(T)
    base = 0
    for g, n in owners:
        if n:
            records[g].X = X[base:base + n].copy()
            base += n


# poses of one device BA window (yv_ba_window_solve, yavo_ba.hip kWinMaxPoses)
WINDOW_MAX_POSES = 128


class SequenceFrontend:
    """The device front end over a stereo sequence in chunks of `chunk` frames (module docstring)."""

    def __init__(self, ctx, chunk: int, K, T_right, n_fixed: int = 2, ba_iters: int = 10,
                 H: int = 376, W: int = 1241, max_kp: int = 2000, match_thr: int = 20, device_window: bool = True,
                 ba_priority: int = 0, expected_frames: int = 0, ba_stream=None):
        """device_window: the BA window is recorded, assembled and written back on the device (yv_ba_window_*,
        no per-chunk read-back); False: the host assembly below (window_problem / apply_window), kept as the
        restatement the device path is checked against. ba_priority: the BA stream's priority (torch's convention:
        -1 high, 0 default) against the context stream the next chunk's kernels run on. expected_frames: the
        sequence length when known (the device window's record store is sized for it up front instead of growing by
        doubling, which synchronises the device inside the loop)."""
        import torch
        from . import Batch, BaWindow, BundleAdjuster
        if chunk < 2 or n_fixed < 1:
            raise ValueError("bad chunk / n_fixed")
        window = chunk + n_fixed
        if device_window and window > WINDOW_MAX_POSES:
            raise ValueError(f"the device BA window holds at most {WINDOW_MAX_POSES} poses (chunk + n_fixed = {window}); "
                             "use a smaller chunk or device_window=False")
        self.ctx, self.chunk, self.H, self.W, self.max_kp = ctx, chunk, H, W, max_kp
        self.K = np.asarray(K, np.float64)
        self.window, self.n_fixed, self.ba_iters, self.match_thr = window, n_fixed, ba_iters, match_thr
        self.batch = Batch(ctx, 2 * chunk, H, W, max_kp, 2 * chunk)
        carry = 2 * chunk
        pairs, tracks = [], []
        for k in range(chunk):
            pairs.append((carry if k == 0 else 2 * (k - 1), 2 * k))  # temporal L_{k-1} -> L_k
            pairs.append((2 * k, 2 * k + 1))                          # stereo L_k -> R_k
            tracks.append((2 * k + 1, 2 * k))
        self.batch.set_pairs(pairs)
        self.batch.set_tracks(tracks, self.K, T_right)
        dev = torch.device("cuda", ctx.device)
        self.bb = ymap.block_bytes(chunk, max_kp)
        self.d_block = torch.zeros(self.bb, dtype=torch.uint8, device=dev)
        self.d_base = torch.from_numpy(IDENTITY.copy()).to(dev)
        self.d_anchors = torch.zeros((1, 7), dtype=torch.float64, device=dev)
        self.d_prior = torch.from_numpy(np.tile(IDENTITY, (chunk, 1))).to(dev)
        self.d_poses = torch.zeros((chunk, 7), dtype=torch.float64, device=dev)
        # pinned read-back buffers (block, edge uv / query, the temporal pairs' match records): DMA, not staging
        def pinned(nbytes):
            return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()
        self._h_block = pinned(self.bb)
        self._h_uv = pinned(chunk * max_kp * 16)
        self._h_q = pinned(chunk * max_kp * 4)
        self._h_m = pinned(2 * chunk * max_kp * 100)
        self.ba = BundleAdjuster(ctx, window, window * max_kp, 2 * window * max_kp)
        # the BA beside the next chunk's kernels: by default the context's side stream, whose hardware queue is never
        # the context stream's (a fresh torch stream shares it one time in four and the two serialise: yv_side_stream);
        # ba_priority != 0 or ba_stream: a stream of the caller's
        if ba_stream is None and ba_priority == 0:
            ba_stream = torch.cuda.ExternalStream(ctx.side_stream, device=dev)
        self.ba_stream = ba_stream if ba_stream is not None else torch.cuda.Stream(device=dev, priority=ba_priority)
        self.ba.set_stream(self.ba_stream.cuda_stream)
        self._ba_pending = False
        self.device_window = device_window
        self.win = BaWindow(self.ba, max_kp, chunk) if device_window else None
        if self.win is not None and expected_frames > 0:
            self.win.reserve(expected_frames)
        self._records: Dict[int, FrameRecord] = {}
        self.next_frame = 0
        self.ba_log: List[Tuple[int, int, float, float]] = []  # (last frame, iterations, chi2 first, chi2 last)

    def close(self) -> None:
        if self.win is not None:
            self.win.close()
        self.ba.set_stream(0)
        self.ba.close()
        self.batch.close()

    @property
    def records(self) -> Dict[int, FrameRecord]:
        """frame -> FrameRecord (device window: read back from the records in HBM after the pending window solve,
        which the window refuses to be read during)."""
        if self.win is None:
            return self._records
        self.flush()
        out = {}
        for g in range(self.next_frame):
            T, e, X, uo, up = self.win.read(g)
            out[g] = FrameRecord(T, e.astype(np.int64), X, up, uo)
        return out

    def process_chunk(self, d_images, seconds: Dict[str, float] = None) -> None:
        """d_images: device uint8 [2 * chunk, H, W] (L_k, R_k interleaved) of frames next_frame ...

        Pipelined: this chunk's detect .. pose LM is issued on the context stream first, then the previous chunk's
        BA window runs (its own stream, host-driven LM) while the GPU works on this chunk; the refined last pose
        then anchors this chunk's placement. The data flow is the sequential loop's, so results are identical."""
        import time
        ctx, n, kp = self.ctx, self.chunk, self.max_kp
        t0 = time.perf_counter()
        first = self.next_frame
        self.batch.run(d_images.data_ptr(), 2 * n, self.W, self.H * self.W, self.match_thr,
                       carry_from=2 * (n - 1))
        self.batch.track_map(self.d_prior.data_ptr(), self.d_poses.data_ptr(), first, 1, self.d_block.data_ptr(), n)
        if self.win is not None:
            return self._process_chunk_device(first, t0, seconds)
        t1 = time.perf_counter()
        ba_sec = {}
        if self._ba_pending:
            self._local_ba(ba_sec)  # the previous chunk's window, beside this chunk's kernels
        t2 = time.perf_counter()
        ctx.map_place(self.d_block.data_ptr(), 1, self.bb, self.d_base.data_ptr(), self.d_anchors.data_ptr())
        ctx.sync()
        t3 = time.perf_counter()
        v = self.batch.view()
        block = ctx.download(self.d_block.data_ptr(), np.uint8, self.bb, out=self._h_block)
        uv = ctx.download(v.edge_uv, np.float64, n * kp * 2, out=self._h_uv).reshape(n, kp, 2)
        q = ctx.download(v.edge_query, np.int32, n * kp, out=self._h_q).reshape(n, kp)
        m = ctx.download(v.matches, np.uint8, 2 * n * kp * 100, out=self._h_m).reshape(2 * n, kp, 100)[0::2]
        own = m[:, :, 48:56].copy().view(np.int32).reshape(n, kp, 2)  # Matches::pt2.{x, y}
        self._records.update(frame_records_from_block(block, uv, q, own))
        self.next_frame = first + n
        self._ba_pending = True
        t4 = time.perf_counter()
        if seconds is not None:
            for key, dt in (("issue", t1 - t0), ("ba", t2 - t1), ("device_wait", t3 - t2), ("download", t4 - t3)):
                seconds[key] = seconds.get(key, 0.0) + dt
            for key, dt in ba_sec.items():
                seconds[key] = seconds.get(key, 0.0) + dt

    def _process_chunk_device(self, first: int, t0: float, seconds) -> None:
        """process_chunk with the device window: collect the previous window's BA (begun one call earlier, it ran
        beside this chunk's kernels; the anchor lands in d_base), place and record this chunk after it, and begin this
        chunk's window at once, so it runs while the host issues the next chunk -- no read-back but the counts."""
        import time
        ctx, n = self.ctx, self.chunk
        t1 = time.perf_counter()
        if self._ba_pending:
            self._local_ba_device_end()
        t2 = time.perf_counter()
        ctx.map_place(self.d_block.data_ptr(), 1, self.bb, self.d_base.data_ptr(), self.d_anchors.data_ptr())
        v = self.batch.view()
        self.win.add_block(self.d_block.data_ptr(), first, n, v.edge_uv, v.edge_query, v.matches, self.max_kp)
        self.next_frame = first + n
        t3 = time.perf_counter()
        self._local_ba_device_begin()
        t4 = time.perf_counter()
        if seconds is not None:
            for key, dt in (("issue", t1 - t0), ("ba", t2 - t1), ("place_record", t3 - t2), ("ba_begin", t4 - t3)):
                seconds[key] = seconds.get(key, 0.0) + dt

    def _local_ba_device_begin(self) -> None:
        last = self.next_frame - 1
        lo = max(0, last - self.window + 1)
        self._ba_last = last
        self.win.solve_begin(lo, last + 1 - lo, self.n_fixed, self.K, self.ba_iters, self.d_base.data_ptr())
        self._ba_pending = True

    def _local_ba_device_end(self) -> None:
        self._ba_pending = False
        solved, log, it = self.win.solve_end()
        if solved:
            self.ba_log.append((self._ba_last, it, float(log[0]), float(log[-1])))

    def flush(self, seconds: Dict[str, float] = None) -> None:
        """The last chunk's BA window (process_chunk runs each window one chunk late)."""
        import time
        if self._ba_pending and self.win is not None:
            t0 = time.perf_counter()
            self._local_ba_device_end()
            if seconds is not None:
                seconds["ba"] = seconds.get("ba", 0.0) + time.perf_counter() - t0
        elif self._ba_pending:
            t0 = time.perf_counter()
            ba_sec = {}
            self._local_ba(ba_sec)
            if seconds is not None:
                seconds["ba"] = seconds.get("ba", 0.0) + time.perf_counter() - t0
                for key, dt in ba_sec.items():
                    seconds[key] = seconds.get(key, 0.0) + dt

    def _local_ba(self, sec) -> None:
        import time
        self._ba_pending = False
        last = self.next_frame - 1
        frames = list(range(max(0, last - self.window + 1), last + 1))
        if len(frames) <= self.n_fixed:
            return
        t0 = time.perf_counter()
        poses, X, ep, el, meas, owners = window_problem(self._records, frames, self.n_fixed)
        if len(ep) == 0:
            return
        t1 = time.perf_counter()
        self.ba.set_problem(len(frames), self.n_fixed, len(X), ep, el, meas, self.K)
        t2 = time.perf_counter()
        poses, X, log, it = self.ba.solve(poses, X, self.ba_iters)
        t3 = time.perf_counter()
        apply_window(self._records, frames, poses, X, owners)
        sec["ba_assemble"] = t1 - t0 + time.perf_counter() - t3
        sec["ba_set_problem"] = t2 - t1
        sec["ba_solve"] = t3 - t2
        self.ba_log.append((last, it, float(log[0]), float(log[-1])))
        # the next chunk is placed after the refined last pose
        self.ctx.upload(self.d_base.data_ptr(), self._records[last].T_wc)

    def trajectory(self) -> np.ndarray:
        """[n_frames, 7] T_wc in frame order (after the last BA window)."""
        self.flush()
        if self.win is not None:
            return self.win.trajectory(0, self.next_frame)
        return np.stack([self._records[g].T_wc for g in sorted(self._records)])


def shard_range(rank: int, world: int, frames_per_rank: int) -> Tuple[int, int]:
    """[first, end) of the frames rank r runs: contiguous shards of `frames_per_rank` frames overlapping by one frame
    (the 1-frame halo: shard r starts at shard r - 1's last frame, so its first temporal pair is the sequence's own and
    its trajectory can be placed after shard r - 1's). A world of W ranks covers W (n - 1) + 1 frames."""
    if not 0 <= rank < world or frames_per_rank < 2:
        raise ValueError("bad rank / world / frames_per_rank")
    first = rank * (frames_per_rank - 1)
    return first, first + frames_per_rank


class SequenceShard:
    """The frame-sharded form of the sequence front end (BASELINE configs[3] / [4] on N GPUs; SURVEY.md 8e: the
    front end shards with a 1-frame halo, pose chaining is serial): ONE sequence split over `world` ranks
    (shard_range). Rank r runs its frames through its own SequenceFrontend -- detect .. pose LM, the shared map, the
    local BA windows -- with its trajectory starting at identity at its first frame; no collective on the data path.
    finish() exports the shard's frames (rank r > 0 without its first frame, which shard r - 1 owns) as one map block
    (yv_ba_window_export_block), all-gathers the blocks (RCCL over xGMI; gloo for the CPU / shared-GPU rehearsal) and
    places them after each other on every rank (yv_map_place: A_0 = I, A_{r+1} = A_r C_r with C_r the shard's last
    pose; T_wc = A_r T, X_w = A_r X). Each shard's local result is what a one-rank SequenceFrontend run over the same
    frames gives, bit for bit; the BA windows do not straddle shards (replicas)."""

    def __init__(self, ctx, rank: int, world: int, frames_per_rank: int, chunk: int, K, T_right, n_fixed: int = 2,
                 ba_iters: int = 10, H: int = 376, W: int = 1241, max_kp: int = 2000, match_thr: int = 20):
        import torch
        if frames_per_rank % chunk:
            raise ValueError("frames_per_rank must be a multiple of chunk")
        self.ctx, self.rank, self.world, self.n, self.max_kp = ctx, rank, world, frames_per_rank, max_kp
        self.first, self.end = shard_range(rank, world, frames_per_rank)
        self.fe = SequenceFrontend(ctx, chunk, K, T_right, n_fixed=n_fixed, ba_iters=ba_iters, H=H, W=W,
                                   max_kp=max_kp, match_thr=match_thr, expected_frames=frames_per_rank)
        dev = torch.device("cuda", ctx.device)
        self.bb = ymap.block_bytes(frames_per_rank, max_kp)
        self.d_block = torch.zeros(self.bb, dtype=torch.uint8, device=dev)
        import torch.distributed as dist
        self.collective = dist.is_available() and dist.is_initialized()
        if (self.collective and dist.get_world_size() != world) or (world > 1 and not self.collective):
            raise ValueError("world must match the process group (and N > 1 needs one)")
        self.d_gathered = torch.zeros((world, self.bb), dtype=torch.uint8, device=dev) if self.collective \
            else self.d_block.view(1, self.bb)
        self.d_base = torch.zeros(7, dtype=torch.float64, device=dev)
        self.d_anchors = torch.zeros((world, 7), dtype=torch.float64, device=dev)
        self.seconds_exchange = 0.0

    def process_chunk(self, d_images, seconds: Dict[str, float] = None) -> None:
        """d_images: device uint8 [2 * chunk, H, W] of the shard's next chunk (SequenceFrontend.process_chunk)."""
        self.fe.process_chunk(d_images, seconds)

    def finish(self) -> None:
        """The last BA window, the shard's block, the all-gather and the placement (every rank)."""
        import time
        import torch
        import torch.distributed as dist
        fe = self.fe
        if fe.next_frame != self.n:
            raise RuntimeError(f"shard holds {fe.next_frame} of its {self.n} frames")
        fe.flush()
        lo = 0 if self.rank == 0 else 1
        t0 = time.perf_counter()
        fe.win.export_block(lo, self.n - lo, self.n - 1, self.first, self.d_block.data_ptr(), self.n, self.max_kp)
        self.ctx.sync()
        if self.collective and dist.get_backend() == "nccl":
            dist.all_gather_into_tensor(self.d_gathered, self.d_block)
        elif self.collective:  # gloo: list form
            dist.all_gather(list(self.d_gathered.unbind(0)), self.d_block)
        self.d_base.copy_(torch.from_numpy(IDENTITY.copy()))
        torch.cuda.synchronize(self.d_block.device)  # the gathered blocks and the base are in place
        self.ctx.map_place(self.d_gathered.data_ptr(), self.world, self.bb, self.d_base.data_ptr(),
                           self.d_anchors.data_ptr())  # on the context stream
        self.ctx.sync()
        self.seconds_exchange = time.perf_counter() - t0

    def local_trajectory(self) -> np.ndarray:
        """[n, 7] T_wc of the shard's frames relative to its first frame (the one-rank run's trajectory)."""
        return self.fe.trajectory()

    def placed_blocks(self) -> np.ndarray:
        """[world, block_bytes] uint8: every shard's block in world coordinates (the same on every rank)."""
        return self.d_gathered.cpu().numpy().reshape(self.world, self.bb)

    def trajectory(self) -> np.ndarray:
        """[world (n - 1) + 1, 7] T_wc of the whole sequence from the placed blocks."""
        out = []
        for blk in self.placed_blocks():
            _, kfs, _ = ymap.parse_block(blk)
            out.append(np.array(kfs["T"], np.float64))
        return np.concatenate(out)

    def map(self) -> "ymap.Map":
        m = ymap.Map()
        m.insert_blocks(self.placed_blocks(), self.world, self.bb)
        return m

    def close(self) -> None:
        self.fe.close()
