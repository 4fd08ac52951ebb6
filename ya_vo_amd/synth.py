"""Synthetic KITTI-shaped frames.

There is no KITTI data in this container or on the GPU box, so the benchmarks and the parity tests run on
a deterministic blurred-noise field: integer-only splitmix64 noise, separable integer Gaussian (sigma 2),
rescaled to mean 128 / std 64 and clipped to u8.  Frame k of a sequence is the crop at offset (k, 3k) of
one unbounded field (so consecutive frames share texture and produce real matches); the stereo "right"
image is the crop at column + 8.  Every step is integer arithmetic or correctly rounded IEEE double, so
any host produces the same bytes.
"""
from __future__ import annotations

import numpy as np

H_KITTI, W_KITTI = 376, 1241

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
# round(256 * exp(-x^2 / (2 * 2^2))), x = -6..6  (sigma = 2)
_GAUSS13 = np.array([3, 11, 35, 83, 155, 226, 256, 226, 155, 83, 35, 11, 3], dtype=np.int64)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def _noise(seed: int, r0: int, c0: int, h: int, w: int) -> np.ndarray:
    """Integer noise n(R, C) in [-131070, 131070]: sum of the four 16-bit lanes of splitmix64(key)."""
    rows = (np.arange(h, dtype=np.int64) + r0).astype(np.uint64)
    cols = (np.arange(w, dtype=np.int64) + c0).astype(np.uint64)
    key = (rows[:, None] << np.uint64(32)) | cols[None, :]
    with np.errstate(over="ignore"):
        salt = (np.uint64(seed) * np.uint64(0x100000001B3)) & _M64
    z = _splitmix64(key ^ salt)
    m = np.uint64(0xFFFF)
    s = (z & m).astype(np.int64) + ((z >> np.uint64(16)) & m).astype(np.int64) \
        + ((z >> np.uint64(32)) & m).astype(np.int64) + ((z >> np.uint64(48)) & m).astype(np.int64)
    return s - 131070


def synth_frame(seed: int, r0: int, c0: int, h: int = H_KITTI, w: int = W_KITTI) -> np.ndarray:
    """One h x w uint8 crop of the blurred-noise field of `seed`, top-left corner at (r0, c0)."""
    g = _GAUSS13
    half = len(g) // 2
    n = _noise(seed, r0 - half, c0 - half, h + 2 * half, w + 2 * half)
    # separable integer correlation (exact in int64)
    hz = np.zeros((h + 2 * half, w), dtype=np.int64)
    for j, gj in enumerate(g):
        hz += gj * n[:, j:j + w]
    v = np.zeros((h, w), dtype=np.int64)
    for i, gi in enumerate(g):
        v += gi * hz[i:i + h, :]
    # std of v = std(noise) * (sum g^2): var of one 16-bit uniform lane = (65536^2 - 1) / 12, four lanes
    std_noise = np.sqrt(4.0 * (65536.0 * 65536.0 - 1.0) / 12.0)
    std_v = std_noise * float(np.sum(g * g))
    out = np.floor(128.0 + 64.0 * (v.astype(np.float64) / std_v) + 0.5)
    return np.clip(out, 0, 255).astype(np.uint8)


def synth_sequence(seed: int, n_frames: int, stereo: bool = False, h: int = H_KITTI, w: int = W_KITTI,
                   start: int = 0) -> np.ndarray:
    """Frames start..start+n_frames-1 of a sequence: frame k = crop at (k, 3k).  With stereo=True the
    result is [n_frames, 2, h, w] (left, right = crop at column + 8), else [n_frames, h, w]."""
    frames = []
    for k in range(start, start + n_frames):
        left = synth_frame(seed, k, 3 * k, h, w)
        if stereo:
            right = synth_frame(seed, k, 3 * k + 8, h, w)
            frames.append(np.stack([left, right]))
        else:
            frames.append(left)
    return np.stack(frames)


def synth_stereo_batch(seed: int, n_frames: int, start: int = 0, h: int = H_KITTI, w: int = W_KITTI) -> np.ndarray:
    """[n_frames * 2, h, w] images L_k, R_k for k = start..start+n_frames-1, cut from one field (same bytes
    as synth_frame(seed, k, 3k) / synth_frame(seed, k, 3k + 8))."""
    r0, c0 = start, 3 * start
    hh = h + (n_frames - 1)
    ww = w + 3 * (n_frames - 1) + 8
    field = synth_frame(seed, r0, c0, hh, ww)
    out = np.empty((2 * n_frames, h, w), np.uint8)
    for i in range(n_frames):
        out[2 * i] = field[i:i + h, 3 * i:3 * i + w]
        out[2 * i + 1] = field[i:i + h, 3 * i + 8:3 * i + 8 + w]
    return out
