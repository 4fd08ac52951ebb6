"""The shared map (include/yavo/yavo_map.h) on the host side.

The reference keeps one process-wide ``Map`` (include/Map.hpp:9-37): ``insertKeyFrame`` keys frames by
``Frame::frameID`` and ``insertMapPoint`` keys landmarks by ``MapPoint::ptID`` (src/Map.cc:9-40);
``getFrames`` / ``getMPs`` return those tables. Here every rank builds a fixed-size device block for its
frame chunk (``Batch.track_map``), the blocks are all-gathered (RCCL over xGMI, :func:`gather_map_blocks`) and
placed in world coordinates on the device (``Context.map_place``). :class:`Map` reads placed blocks back into the
reference's two tables.

Block layout (256-B aligned sections): header (128 B), ``max_kf`` keyframe records (72 B), then
``max_kf * lm_stride`` landmark slots (32 B) -- keyframe j's landmarks start at slot ``j * lm_stride``.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

HEADER_DTYPE = np.dtype([("chunk", "<f8", 7), ("first_frame", "<i8"), ("n_frames", "<i4"), ("n_kf", "<i4"),
                         ("kf_every", "<i4"), ("lm_stride", "<i4"), ("max_kf", "<i4"), ("placed", "<i4"),
                         ("pad", "<f8", 5)])
KEYFRAME_DTYPE = np.dtype([("frame_id", "<i8"), ("T", "<f8", 7), ("n_landmarks", "<i4"), ("pad", "<i4")])
LANDMARK_DTYPE = np.dtype([("id", "<i8"), ("X", "<f8", 3)])
assert HEADER_DTYPE.itemsize == 128 and KEYFRAME_DTYPE.itemsize == 72 and LANDMARK_DTYPE.itemsize == 32


def _round256(x: int) -> int:
    return (x + 255) & ~255


def landmark_offset(max_kf: int) -> int:
    return _round256(HEADER_DTYPE.itemsize + max_kf * KEYFRAME_DTYPE.itemsize)


def block_bytes(max_kf: int, lm_stride: int) -> int:
    """Bytes of one block (yv_map_block_bytes)."""
    if max_kf < 1 or lm_stride < 1:
        raise ValueError("max_kf and lm_stride must be >= 1")
    return _round256(landmark_offset(max_kf) + max_kf * lm_stride * LANDMARK_DTYPE.itemsize)


def max_keyframes(n_frames: int, first_frame: int, kf_every: int) -> int:
    """Keyframes a chunk [first_frame, first_frame + n_frames) holds under the policy g % kf_every == 0."""
    if n_frames <= 0:
        return 0
    return (first_frame + n_frames - 1) // kf_every - (first_frame - 1) // kf_every


def parse_block(buf) -> Tuple[np.ndarray, np.ndarray, List[np.ndarray]]:
    """(header, written keyframes, per-keyframe written landmarks) of one block (bytes / uint8 array).

    A C-contiguous uint8 array is parsed in place: the results are READ-ONLY views that alias `buf` (no 1+ MB
    copy), so they change when the caller reuses the buffer (ya_vo_amd.sequence reuses one pinned block); copy what
    you keep.  Any other input is copied first."""
    if isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and buf.flags["C_CONTIGUOUS"]:
        raw = buf.reshape(-1).view()
        raw.flags.writeable = False  # the views alias the caller's buffer: writes through them are refused
    else:
        raw = np.frombuffer(bytes(buf) if not isinstance(buf, np.ndarray) else buf.tobytes(), np.uint8)
    h = raw[:HEADER_DTYPE.itemsize].view(HEADER_DTYPE)[0]
    max_kf, stride, n_kf = int(h["max_kf"]), int(h["lm_stride"]), int(h["n_kf"])
    if not 0 <= n_kf <= max_kf:
        raise ValueError(f"corrupt block: n_kf={n_kf} max_kf={max_kf}")
    kfo = HEADER_DTYPE.itemsize
    kfs = raw[kfo:kfo + max_kf * KEYFRAME_DTYPE.itemsize].view(KEYFRAME_DTYPE)[:n_kf]
    lmo = landmark_offset(max_kf)
    lms = []
    for j in range(n_kf):
        base = lmo + j * stride * LANDMARK_DTYPE.itemsize
        n = int(kfs[j]["n_landmarks"])
        lms.append(raw[base:base + n * LANDMARK_DTYPE.itemsize].view(LANDMARK_DTYPE))
    return h, kfs, lms


class Map:
    """The reference's Map tables (include/Map.hpp:12-13) read back from placed blocks.

    ``frames``: frameID -> T_wc (Sophus SE3d::data() = qx, qy, qz, qw, tx, ty, tz);
    ``landmarks``: ptID -> world point. ptID = frameID << 16 | edge index (unique per observation edge).
    """

    def __init__(self):
        self.frames: Dict[int, np.ndarray] = {}
        self.landmarks: Dict[int, np.ndarray] = {}

    def insert_blocks(self, blocks: np.ndarray, world: int, block_bytes_: int) -> None:
        raw = np.ascontiguousarray(blocks).view(np.uint8).reshape(-1)
        for r in range(world):
            h, kfs, lms = parse_block(raw[r * block_bytes_:(r + 1) * block_bytes_])
            if int(h["n_kf"]) and int(h["placed"]) not in (1, 3):  # 1 / 3: placed (a frame chunk / a sequence shard)
                raise ValueError(f"block {r} is not placed in world coordinates")
            for kf, lm in zip(kfs, lms):
                self.insert_keyframe(int(kf["frame_id"]), kf["T"])
                for rec in lm:
                    self.insert_map_point(int(rec["id"]), rec["X"])

    # Map::insertKeyFrame / insertMapPoint (src/Map.cc:9-40): insert keyed by id (the reference's insert keeps
    # an existing entry; ids here are unique per frame / edge, so no key repeats)
    def insert_keyframe(self, frame_id: int, T) -> None:
        self.frames.setdefault(frame_id, np.array(T, np.float64))

    def insert_map_point(self, pt_id: int, X) -> None:
        self.landmarks.setdefault(pt_id, np.array(X, np.float64))

    def get_frames(self) -> Dict[int, np.ndarray]:
        return dict(self.frames)

    def get_mps(self) -> Dict[int, np.ndarray]:
        return dict(self.landmarks)


def gather_map_blocks(block, world: int):
    """All-gather one fixed-size block per rank (uint8 torch tensor [block_bytes]) into [world, block_bytes] in
    rank order: RCCL over xGMI on GPUs (all_gather_into_tensor), gloo on CPU (list all_gather)."""
    import torch
    import torch.distributed as dist

    out = torch.empty((world,) + tuple(block.shape), dtype=block.dtype, device=block.device)
    if block.is_cuda:
        dist.all_gather_into_tensor(out, block)
    else:
        dist.all_gather(list(out.unbind(0)), block)
    return out
