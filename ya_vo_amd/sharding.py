"""Frame sharding across GPUs: one process per GPU, contiguous chunks of the frame
sequence, and the exchange the shared map needs.

* Detect / describe / match are per frame (matching needs frame k-1): every rank owns a contiguous
  chunk [start, end) and recomputes its predecessor frame start-1 (a 1-frame halo), so the data path has
  no collective at all.
* Pose chaining is serial (src/LoopHandler.cc:139,156): the per-frame results are gathered in frame
  order for the host that chains them -- an all-gather of fixed-size per-frame records (12 doubles of
  T_cw per frame, landmark blocks) over RCCL (backend "nccl") on GPUs, gloo in the CPU tests.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional


@dataclass(frozen=True)
class Shard:
    rank: int
    start: int          # first frame this rank reports
    end: int            # one past the last frame
    halo: Optional[int]  # predecessor frame recomputed locally (None for the sequence's first frame)

    @property
    def frames(self) -> range:
        return range(self.start, self.end)

    @property
    def computed(self) -> range:
        """Frames this rank detects / describes (its chunk plus the halo)."""
        return range(self.start if self.halo is None else self.halo, self.end)

    def pairs(self) -> List[tuple]:
        """Temporal match pairs (k-1, k) this rank evaluates: every pair whose second frame it owns."""
        return [(k - 1, k) for k in self.frames if k >= 1]


def shard_frames(n_frames: int, world: int, rank: int) -> Shard:
    """Balanced contiguous chunks: the first n_frames % world ranks get one extra frame."""
    if world <= 0 or not 0 <= rank < world or n_frames < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    end = start + base + (1 if rank < extra else 0)
    halo = start - 1 if start > 0 and end > start else None
    return Shard(rank, start, end, halo)


def gather_frame_records(local, n_frames: int, world: int, rank: int):
    """All-gather per-frame records (torch tensor [n_local, R]) into [n_frames, R] in frame order.

    Uses padded all_gather (chunks may differ by one frame): each rank sends max_chunk rows; the
    receiver trims by the known shard sizes.  Works on the nccl (RCCL) and gloo backends.
    """
    import torch
    import torch.distributed as dist

    shards = [shard_frames(n_frames, world, r) for r in range(world)]
    max_chunk = max(len(s.frames) for s in shards)
    pad = torch.zeros((max_chunk,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return torch.cat([o[: len(s.frames)] for o, s in zip(outs, shards)], dim=0)


def shard_images(stereo, halo_left=None, halo_right=None):
    """Device image layout of one rank's shard: [L_0, R_0, ..., L_{B-1}, R_{B-1}] then, when the shard has a
    predecessor, the halo frame's left image (index 2B) and, for the LK tracker, its right image (index 2B + 1: the
    halo frame's stereo map points seed the shard's first LK track).  `stereo` [B, 2, H, W] or [2B, H, W] uint8."""
    import numpy as np
    s = np.asarray(stereo, np.uint8)
    s = s.reshape(-1, s.shape[-2], s.shape[-1])
    if halo_left is None:
        return np.ascontiguousarray(s)
    extra = [np.asarray(halo_left, np.uint8)[None]]
    if halo_right is not None:
        extra.append(np.asarray(halo_right, np.uint8)[None])
    return np.ascontiguousarray(np.concatenate([s] + extra))


def exchange_summary(gather_ms, place_ms, slack_ms):
    """Summary of a run's shared-map exchanges (FrameShard.collective_stats): per exchange the all-gather's and the
    placement's device time and the slack from the gather's end to the end of the context-stream run it overlapped
    (>= 0: the collective was hidden behind the image kernels)."""
    import numpy as np
    g, pl, sl = (np.asarray(x, np.float64) for x in (gather_ms, place_ms, slack_ms))
    if not len(g):
        return None
    return {"exchanges": int(len(g)), "allgather_ms_mean": round(float(g.mean()), 4),
            "allgather_ms_max": round(float(g.max()), 4), "place_ms_mean": round(float(pl.mean()), 4),
            "hidden_fraction": round(float(np.mean(sl >= 0)), 4), "min_slack_ms": round(float(sl.min()), 4),
            "how": "HIP events on the communication stream around all_gather_into_tensor and map_place; slack = time "
                   "from the gather's end to the end of the context-stream run it overlaps (>= 0: hidden)"}


class FrameShard:
    """One rank's share of a frame-sharded stereo sequence on its GPU: frames
    [first_frame, first_frame + n_frames) and, with `halo`, the predecessor frame first_frame - 1 whose left image is
    detected and described in the same run (image index 2 * n_frames), so the shard's first temporal pair
    L_{first-1} -> L_first needs no communication and gives the same matches a 1-rank run over the whole sequence
    gets from its carry slot.  Without `halo` the first pair reads the batch's carry slot (empty on the first run:
    the sequence's frame 0 has no predecessor, as in the reference's first takeVOStep).  The LK tracker
    (trackLastFrame, src/LoopHandler.cc:327-413) tracks frame k-1's stereo map points into L_k, so with a halo it also
    takes the halo frame's right image (index 2B + 1, `shard_images(..., halo_right)`) and its stereo pair: track 0 is
    then the halo frame -> first_frame, as in match mode, and no pose is lost at a rank boundary.

    Per step (one pass over the shard's resident images, `step`): yv_batch_run (detect / describe L and R, match
    L_{k-1} -> L_k and L_k -> R_k, removeOutliers), then yv_batch_track_map (stereo triangulation + pose-only LM per
    frame, the shard's shared-map block).  With a map, every rank's block is all-gathered (RCCL over xGMI on "nccl",
    list all_gather on gloo) on a communication stream one step behind and placed in world coordinates by the serial
    anchor chain A_{r+1} = A_r * C_r (yavo_map.hip), the reference's pose chaining (src/LoopHandler.cc:139,156)."""

    def __init__(self, ctx, n_frames: int, first_frame: int, K, T_right, *, halo: bool = True, world: int = 1,
                 rank: int = 0, backend: str = "nccl", kf_every: int = 0, max_kf: int = 0, overlap_mode: int = 1,
                 tracker: str = "match", H: int = 376, W: int = 1241, max_kp: int = 2000, match_thr: int = 20):
        import numpy as np
        import torch
        from . import Batch
        from . import map as ymap
        if n_frames < 1 or first_frame < 0 or (halo and first_frame < 1):
            raise ValueError("bad shard: n_frames >= 1 and a halo needs first_frame >= 1")
        if tracker not in ("match", "lk"):
            raise ValueError("tracker must be 'match' or 'lk'")
        self.ctx, self.B, self.first, self.halo = ctx, n_frames, first_frame, halo
        self.world, self.rank, self.backend = world, rank, backend
        self.H, self.W, self.max_kp, self.match_thr = H, W, max_kp, match_thr
        B = n_frames
        lk_halo = halo and tracker == "lk"
        self.n_images = 2 * B + (2 if lk_halo else 1 if halo else 0)
        self.batch = Batch(ctx, self.n_images, H, W, max_kp, 2 * B + (1 if lk_halo else 0))
        prev0 = 2 * B if halo else self.n_images  # the halo image, or the carry slot (index max_images)
        pairs, tracks = [], []
        for k in range(B):
            pairs.append((prev0 if k == 0 else 2 * (k - 1), 2 * k))  # temporal L_{k-1} -> L_k
            pairs.append((2 * k, 2 * k + 1))                          # stereo L_k -> R_k
            if tracker == "match":
                tracks.append((2 * k + 1, 2 * k))                     # PnP of frame k-1 against frame k's map
            elif k > 0:
                tracks.append((2 * (k - 1) + 1, 2 * k))               # LK: frame k-1's stereo map -> L_k
        if lk_halo:
            pairs.append((2 * B, 2 * B + 1))                          # the halo frame's stereo pair (index 2B)
            tracks.insert(0, (2 * B, 0))                              # LK: halo frame's stereo map -> L_0
        self.pairs, self.tracks = pairs, tracks
        self.batch.set_pairs(pairs)
        if tracker == "lk":
            self.batch.set_track_lk(2)  # LK images = the left images 0, 2, 4, ...
        self.batch.set_tracks(tracks, K, T_right)
        self.n_tracks = len(tracks)
        dev = torch.device("cuda", ctx.device)
        identity = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
        self.d_prior = torch.from_numpy(np.tile(identity, (self.n_tracks, 1))).to(dev)
        # the pose LM of step i runs on the batch's side stream beside step i + 1's image kernels; its output buffer
        # alternates so step i + 1 never writes poses step i's LM is still producing
        self.batch.set_track_overlap(overlap_mode)
        self.d_poses = [torch.zeros((self.n_tracks, 7), dtype=torch.float64, device=dev) for _ in range(2)]
        self.calls = 0
        self.use_map = kf_every > 0 and tracker == "match"
        self.kf_every = kf_every
        self._pending = False
        self.collective = False
        if self.use_map:
            self.max_kf = max(max_kf, ymap.max_keyframes(self.n_tracks, first_frame, kf_every), 1)
            self.bb = ymap.block_bytes(self.max_kf, max_kp)
            self.d_block = torch.zeros(self.bb, dtype=torch.uint8, device=dev)
            # the collective runs whenever a process group is up, so RCCL also carries a 1-rank run's block (the
            # same stream / event hand-off as at N > 1); without one the block is placed where it was written
            import torch.distributed as dist
            self.collective = dist.is_available() and dist.is_initialized()
            if (self.collective and dist.get_world_size() != world) or (world > 1 and not self.collective):
                raise ValueError("world must match the process group (and N > 1 needs one)")
            self.d_gathered = torch.zeros((world, self.bb), dtype=torch.uint8, device=dev) if self.collective \
                else self.d_block.view(1, self.bb)
            self.d_base = torch.from_numpy(identity.copy()).to(dev)
            self.d_anchors = torch.zeros((world, 7), dtype=torch.float64, device=dev)
            self.comm = torch.cuda.Stream(device=dev)
        # collective timing (set_collective_timing): per exchange, events around the all-gather and the placement on
        # the communication stream and one on the context stream after the run it overlaps
        self._timing = False
        self._ev = []
        self._ctx_stream = None

    def set_collective_timing(self, on: bool) -> None:
        """Record HIP events around every exchange from now on (collective_stats reads them); off drops them."""
        import torch
        self._timing = bool(on) and self.use_map
        self._ev = []
        if self._timing and self._ctx_stream is None:
            self._ctx_stream = torch.cuda.ExternalStream(self.ctx.stream, device=self.d_prior.device)

    def collective_stats(self):
        """Device times of the recorded exchanges (after drain): the all-gather (comm stream, events around the
        collective call), the placement after it, and whether the gather had finished by the time the context stream
        finished the run it was exchanged beside (the next step's image kernels: then it is off the critical path).
        Only exchanges issued beside a run are recorded (drain's last one has no run to hide behind)."""
        if not self._ev:
            return None
        g = [e0.elapsed_time(e1) for e0, e1, _, _ in self._ev]
        pl = [e1.elapsed_time(e2) for _, e1, e2, _ in self._ev]
        slack = [e1.elapsed_time(er) for _, e1, _, er in self._ev]  # > 0: the run ended after the gather
        return exchange_summary(g, pl, slack)

    def _exchange(self, overlapped: bool = True) -> None:
        """overlapped: issued right after a run, which it overlaps (step); drain's final exchange overlaps nothing,
        so it is not timed -- its slack would be measured against a run that had already finished."""
        import torch
        import torch.distributed as dist
        # the last track_map's block: all-gathered and placed on the communication stream once it is written
        self.batch.map_wait(self.comm.cuda_stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if self._timing and overlapped else None
        with torch.cuda.stream(self.comm):
            if ev:
                ev[0].record(self.comm)
            if self.collective and self.backend == "nccl":
                dist.all_gather_into_tensor(self.d_gathered, self.d_block)
            elif self.collective:  # gloo: list form
                dist.all_gather(list(self.d_gathered.unbind(0)), self.d_block)
            if ev:
                ev[1].record(self.comm)
            self.ctx.map_place(self.d_gathered.data_ptr(), self.world, self.bb, self.d_base.data_ptr(),
                               self.d_anchors.data_ptr(), stream=self.comm.cuda_stream)
            if ev:
                ev[2].record(self.comm)
        if ev:
            ev[3].record(self._ctx_stream)  # the run this exchange was issued beside
            self._ev.append(tuple(ev))
        self.batch.map_release(self.comm.cuda_stream)
        self._pending = False

    def step(self, d_images: int) -> None:
        """One pass over the shard's resident images (device pointer, layout of shard_images)."""
        # overlap modes 2 / 3 launch the previous step's pose LM (and its map block) inside this run, so the previous
        # block is exchanged after it (one step behind: map_wait before the launch would force it early)
        self.batch.run(d_images, self.n_images, self.W, self.H * self.W, self.match_thr, carry_from=-1)
        if self._pending:
            self._exchange()
        d_out = self.d_poses[self.calls & 1]
        if not self.use_map:
            self.batch.track(self.d_prior.data_ptr(), d_out.data_ptr())
        else:
            self.batch.track_map(self.d_prior.data_ptr(), d_out.data_ptr(), self.first, self.kf_every,
                                 self.d_block.data_ptr(), self.max_kf)
            self._pending = True
        self.calls += 1

    def drain(self) -> None:
        """Exchange the last block, then wait for every stream of the shard."""
        import torch
        if self._pending:
            self._exchange(overlapped=False)
        self.ctx.sync()
        self.batch.track_sync()
        torch.cuda.synchronize(self.d_prior.device)

    def poses(self):
        """[n_tracks, 7] relative poses of the last step (SE3d::data()), track k for the frame pair
        (first + k - 1, first + k).  Match tracker: the edges hold frame first + k's stereo points and frame
        first + k - 1's keypoints, so the pose maps frame first + k's camera coordinates into frame first + k - 1's.
        LK tracker (trackLastFrame): frame first + k - 1's stereo points tracked into frame first + k, so the pose maps
        the other way.  Without a halo the LK tracks start at the pair (first, first + 1)."""
        return self.d_poses[(self.calls - 1) & 1].cpu().numpy()

    def placed_map(self):
        """The last placed shared map: [world, block_bytes] uint8 (rank order; every rank holds the same)."""
        return self.d_gathered.cpu().numpy().reshape(self.world, self.bb)

    def close(self) -> None:
        self.batch.close()
