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
