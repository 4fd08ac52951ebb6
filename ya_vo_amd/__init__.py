"""ya_vo_amd -- MI355X-native YA_VO visual-odometry front end (detect / describe / match / PnP hot path).

The product is libyavo.so (gfx950 HIP kernels behind the C ABI in include/yavo/yavo.h).  This module is the ctypes
binding of that ABI (Context, Batch, Lk, Essential, BundleAdjuster); the reference-shaped C++ host classes
(FastDetector, Brief, LoopHandler) live in ya_vo_amd/frontend/.  There is no CPU fallback: if the library or a GPU is
missing, the calls raise.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref
from typing import Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YAVO_LIB") or os.path.join(_HERE, "lib", "libyavo.so")  # YAVO_LIB: experiment builds

YV_OK = 0
YV_ERR_INVALID = -1
YV_ERR_HIP = -2
YV_ERR_NODEVICE = -3
YV_ERR_CAPACITY = -4
YV_NUM_STAGES = 7
STAGE_NAMES = ("detect", "topk", "brief", "match", "finalize", "track_edges", "track_pose")

# byte-identical to KeyPoint (48 B) / Matches (100 B), /root/reference/include/BriefDescriptor.hpp:11-39
KEYPOINT_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("id", "<i4"), ("matched", "u1"),
                           ("featVec", "u1", (32,)), ("_pad", "u1", (3,))])
MATCH_DTYPE = np.dtype([("pt1", KEYPOINT_DTYPE), ("pt2", KEYPOINT_DTYPE), ("distance", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 48 and MATCH_DTYPE.itemsize == 100

# cv::GaussianBlur(Size(9, 9), 2.5) 8U fixed-point kernel (src/BriefDescriptor.cc:90)
DEFAULT_BLUR_KERNEL = np.array([12, 22, 31, 41, 44, 41, 31, 22, 12], dtype=np.uint16)


class YavoError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: yavo status {status}")


class _BatchView(ctypes.Structure):
    _fields_ = [("max_images", ctypes.c_int), ("max_kp", ctypes.c_int), ("max_pairs", ctypes.c_int),
                ("H", ctypes.c_int), ("W", ctypes.c_int), ("cand_cap", ctypes.c_int64),
                ("cand_count", ctypes.c_void_p), ("det_count", ctypes.c_void_p), ("det_rc", ctypes.c_void_p),
                ("det_resp", ctypes.c_void_p), ("kp_count", ctypes.c_void_p), ("keypoints", ctypes.c_void_p),
                ("blurred", ctypes.c_void_p), ("match_count", ctypes.c_void_p), ("matches", ctypes.c_void_p),
                ("filt_count", ctypes.c_void_p), ("filtered", ctypes.c_void_p),
                ("match_dj", ctypes.c_void_p), ("match_lim", ctypes.c_void_p), ("n_tracks", ctypes.c_int),
                ("edge_count", ctypes.c_void_p), ("edge_X", ctypes.c_void_p), ("edge_uv", ctypes.c_void_p),
                ("edge_query", ctypes.c_void_p), ("edge_outlier", ctypes.c_void_p),
                ("track_inliers", ctypes.c_void_p), ("blur_pitch", ctypes.c_int)]


_lib: Optional[ctypes.CDLL] = None

# symbol -> (restype, argtypes); the same list the C header declares (tests check they all resolve)
_P = ctypes.c_void_p
_I = ctypes.c_int
SIGNATURES = {
    "yv_abi_version": (_I, []),
    "yv_status_string": (ctypes.c_char_p, [_I]),
    "yv_device_count": (_I, []),
    "yv_create": (_I, [_I, ctypes.POINTER(_P)]),
    "yv_destroy": (None, [_P]),
    "yv_stream": (_P, [_P]),
    "yv_side_stream": (_P, [_P]),
    "yv_sync": (_I, [_P]),
    "yv_download": (_I, [_P, _P, _P, ctypes.c_size_t]),
    "yv_upload": (_I, [_P, _P, _P, ctypes.c_size_t]),
    "yv_device_alloc": (_I, [_P, ctypes.c_size_t, ctypes.POINTER(_P)]),
    "yv_device_free": (None, [_P, _P]),
    "yv_host_alloc": (_I, [_P, ctypes.c_size_t, ctypes.POINTER(_P)]),
    "yv_host_free": (None, [_P, _P]),
    "yv_set_fast_params": (_I, [_P, _I, _I]),
    "yv_set_harris_eigen": (_I, [_P, _I]),
    "yv_set_brief_offsets": (_I, [_P, _P]),
    "yv_set_blur_kernel": (_I, [_P, _P]),
    "yv_detect": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_describe": (_I, [_P, _P, _I, _I, _I, _P, _I, _P, ctypes.POINTER(_I)]),
    "yv_match_features": (_I, [_P, _P, _I, _P, _I, _P]),
    "yv_filter_matches": (_I, [_P, _P, _I, _I, _P, ctypes.POINTER(_I)]),
    "yv_batch_create": (_I, [_P, _I, _I, _I, _I, _I, ctypes.POINTER(_P)]),
    "yv_batch_destroy": (None, [_P]),
    "yv_batch_set_pairs": (_I, [_P, _P, _I]),
    "yv_batch_run": (_I, [_P, _P, _I, _I, ctypes.c_int64, _I, _I, _P]),
    "yv_batch_enable_timing": (_I, [_P, _I]),
    "yv_batch_stage_times": (_I, [_P, _P, ctypes.POINTER(_I)]),
    "yv_batch_view_get": (_I, [_P, ctypes.POINTER(_BatchView)]),
    "yv_batch_set_tracks": (_I, [_P, _P, _I, _P, _P]),
    "yv_batch_track": (_I, [_P, _P, _P, _P]),
    "yv_batch_set_track_overlap": (_I, [_P, _I]),
    "yv_batch_track_sync": (_I, [_P]),
    "yv_batch_set_track_lk": (_I, [_P, _I, _I, _I, _I, ctypes.c_double, ctypes.c_double]),
}


_D = ctypes.c_double
GEOM_SIGNATURES = {
    "yv_f_ransac": (_I, [_P, _P, _I, _P, _I, _D, _P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_triangulate": (_I, [_P, _P, _P, _P, _P, _I, _P, _P, ctypes.POINTER(_I)]),
    "yv_world2camera": (_I, [_P, _P, _I, _P, _P, _P]),
    "yv_pose_lm": (_I, [_P, _P, _P, _I, _P, _P, _P, ctypes.POINTER(_I)]),
    "yv_pose_gn": (_I, [_P, _P, _P, _I, _P, _P, ctypes.POINTER(_I)]),
    "yv_pose_lm_batch": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "yv_pose_gn_batch": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "yv_f_ransac_batch": (_I, [_P, _P, ctypes.c_int64, _P, _I, _P, ctypes.c_int64, _I, _D, _P, _P, _P, _P]),
    "yv_lk_create": (_I, [_P, _I, _I, _I, _I, _I, ctypes.POINTER(_P)]),
    "yv_lk_destroy": (None, [_P]),
    "yv_lk_levels": (_I, [_P]),
    "yv_lk_level": (_I, [_P, _I, _I, ctypes.POINTER(_P), ctypes.POINTER(_I), ctypes.POINTER(_P), ctypes.POINTER(_I),
                         ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_lk_build": (_I, [_P, _P, _I, _I, ctypes.c_int64, _P]),
    "yv_lk_track_batch": (_I, [_P, _P, _I, _P, _P, _I, _I, _D, _D, _P, _P, _P, _P]),
    "yv_calc_optical_flow_pyr_lk": (_I, [_P, _P, _P, _I, _I, _I, _P, _I, _I, _I, _I, _D, _D, _P, _P, _P]),
    "yv_essential_create": (_I, [_P, _I, _I, _I, ctypes.POINTER(_P)]),
    "yv_essential_destroy": (None, [_P]),
    "yv_find_essential_batch": (_I, [_P, _P, _P, _P, _I, _I, _D, _D, _D, _D, _D, _P, _P, _P, _P, _P]),
    "yv_recover_pose_batch": (_I, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "yv_find_essential": (_I, [_P, _P, _P, _I, _D, _D, _D, _D, _D, _P, _P, ctypes.POINTER(_I)]),
    "yv_recover_pose": (_I, [_P, _P, _P, _P, _I, _P, _P, _P, ctypes.POINTER(_I)]),
    "yv_ba_create": (_I, [_P, _I, _I, _I, ctypes.POINTER(_P)]),
    "yv_ba_destroy": (None, [_P]),
    "yv_ba_set_problem": (_I, [_P, _I, _I, _I, _P, _P, _P, _I, _P]),
    "yv_ba_solve": (_I, [_P, _P, _P, _I, _P, ctypes.POINTER(_I)]),
    "yv_ba_debug_read": (_I, [_P, _I, _P, ctypes.c_int64]),
    "yv_ba_debug_resumes": (_I, [_P]),
    "yv_ba_debug_ldlt": (_I, [_P, _P, _I, _P, _P, ctypes.POINTER(_I)]),
    "yv_ba_set_stream": (_I, [_P, _P]),
    "yv_ba_set_control": (_I, [_P, _I]),
    "yv_ba_window_create": (_I, [_P, _I, _I, ctypes.POINTER(_P)]),
    "yv_ba_window_destroy": (None, [_P]),
    "yv_ba_window_reserve": (_I, [_P, ctypes.c_int64]),
    "yv_ba_window_add_block": (_I, [_P, _P, ctypes.c_int64, _I, _P, _P, _P, _I, _P]),
    "yv_ba_window_solve": (_I, [_P, ctypes.c_int64, _I, _I, _P, _I, _P, _P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_ba_window_solve_begin": (_I, [_P, ctypes.c_int64, _I, _I, _P, _I, _P]),
    "yv_ba_window_solve_end": (_I, [_P, _P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_ba_window_read": (_I, [_P, ctypes.c_int64, _P, ctypes.POINTER(_I), _P, _P, _P, _P, _I]),
    "yv_ba_window_trajectory": (_I, [_P, ctypes.c_int64, _I, _P]),
    "yv_ba_window_export_block": (_I, [_P, ctypes.c_int64, _I, ctypes.c_int64, ctypes.c_int64, _P, _I, _I, _P]),
    "yv_lm_sum_mode": (_I, []),
    "yv_pose_lm_sum_mode": (_I, [_I]),
    "yv_track_lm_sum_mode": (_I, [_I]),
}

# include/yavo/yavo_map.h (the shared map; ya_vo_amd/map.py wraps the block layout)
MAP_SIGNATURES = {
    "yv_map_block_bytes": (ctypes.c_int64, [_I, _I]),
    "yv_batch_track_map": (_I, [_P, _P, _P, ctypes.c_int64, _I, _P, _I, _P]),
    "yv_batch_map_wait": (_I, [_P, _P]),
    "yv_batch_map_release": (_I, [_P, _P]),
    "yv_map_place": (_I, [_P, _P, _I, ctypes.c_int64, _P, _P, _P]),
}

# include/yavo/yavo_io.h (frame I/O and formats; ya_vo_amd/io.py wraps them)
IO_SIGNATURES = {
    "yv_png_info": (_I, [_P, ctypes.c_size_t, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_png_decode_gray": (_I, [_P, ctypes.c_size_t, _P, _I, _I, _I]),
    "yv_imread_gray": (_I, [ctypes.c_char_p, _P, _I, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_parse_calib_string": (_I, [ctypes.c_char_p, _P]),
    "yv_seq_open": (_I, [ctypes.c_char_p, _I, ctypes.POINTER(_P)]),
    "yv_seq_close": (None, [_P]),
    "yv_seq_frames": (_I, [_P]),
    "yv_seq_path": (_I, [_P, _I, _I, ctypes.c_char_p, _I]),
    "yv_seq_calib": (_I, [_P, _P, _P, _P, _P]),
    "yv_seq_size": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "yv_seq_read": (_I, [_P, _I, _I, _P, ctypes.c_int64, _I]),
    "yv_seq_upload": (_I, [_P, _P, _I, _I, _P, ctypes.c_int64, _I, _P]),
    "yv_png_write_gray": (_I, [ctypes.c_char_p, _P, _I, _I, _I]),
    "yv_pngdec_create": (_I, [_P, _I, _I, _I, ctypes.POINTER(_P)]),
    "yv_pngdec_destroy": (None, [_P]),
    "yv_pngdec_decode": (_I, [_P, _P, _P, _I, _P, ctypes.c_int64, _P]),
    "yv_seq_upload_gpu": (_I, [_P, _P, _I, _I, _P, ctypes.c_int64, _I, _P]),
    "yv_seq_upload_gpu_frames": (_I, [_P, _P, _P, _I, _P, ctypes.c_int64, _I, _P]),
    "yv_pngdec_status": (_I, [_P, _P, ctypes.POINTER(_I)]),
    "yv_pngdec_set_checks": (_I, [_P, _I, _I]),
    "yv_write_kitti_poses": (_I, [ctypes.c_char_p, _P, _I]),
    "yv_read_kitti_poses": (_I, [ctypes.c_char_p, _P, _I, ctypes.POINTER(_I)]),
}


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libyavo.so (built by __graft_entry__.build()).  Raises if it is missing: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process.  torch ships its own libamdhip64 (SONAME libamdhip64.so.7) and links it
    # by the unversioned name; if libyavo.so were loaded first, /opt/rocm's copy would be mapped and torch
    # would then map a second runtime (two HSA instances: "No HIP GPUs are available").  Loading torch first
    # makes libyavo's NEEDED libamdhip64.so.7 resolve to the runtime already in the process.
    if os.environ.get("YAVO_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = ctypes.CDLL(path)
    tables = (SIGNATURES, GEOM_SIGNATURES, IO_SIGNATURES, MAP_SIGNATURES)
    for name, (res, args) in [kv for t in tables for kv in t.items()]:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lm_sum_mode(n_problems=None) -> int:
    """The pose-LM kernel's edge-sum order as the oracle's sum_mode (parity tests use it): the batch's track LM
    (yv_lm_sum_mode) when n_problems is None, else yv_pose_lm / yv_pose_lm_batch over n_problems problems
    (yv_pose_lm_sum_mode)."""
    lib = load_library()
    return int(lib.yv_lm_sum_mode() if n_problems is None else lib.yv_pose_lm_sum_mode(int(n_problems)))


def track_lm_sum_mode(n_tracks) -> int:
    """The batch track LM's edge-sum order (oracle sum_mode) for a batch of n_tracks tracks (yv_track_lm_sum_mode)."""
    return int(load_library().yv_track_lm_sum_mode(int(n_tracks)))


def _check(status: int, what: str) -> None:
    if status != YV_OK:
        raise YavoError(status, what)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _f64(a, shape=None) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a.reshape(shape) if shape is not None else a


class _GeomMixin:
    def map_place(self, d_blocks: int, world: int, block_bytes: int, d_base: int, d_anchors: int,
                  stream: int = 0) -> None:
        """Place gathered map blocks in world coordinates in place (yv_map_place)."""
        _check(self.lib.yv_map_place(self.handle, ctypes.c_void_p(d_blocks), world, block_bytes,
                                     ctypes.c_void_p(d_base), ctypes.c_void_p(d_anchors),
                                     ctypes.c_void_p(stream) if stream else None), "yv_map_place")

    """Geometry rows (include/yavo/yavo_geom.h). Poses: Sophus SE3d::data() = {qx, qy, qz, qw, tx, ty, tz}."""

    def calc_optical_flow_pyr_lk(self, prev, nxt, pts, win=11, max_level=3, max_count=30, eps=0.01, min_eig=0.001):
        """cv::calcOpticalFlowPyrLK (flags 0) -> (next_pts [n, 2] (x = col, y = row), status [n] bool, err [n])."""
        prev = np.ascontiguousarray(prev, np.uint8)
        nxt = np.ascontiguousarray(nxt, np.uint8)
        p = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
        H, W = prev.shape
        out = np.zeros_like(p)
        st = np.zeros(max(len(p), 1), np.uint8)
        err = np.zeros(max(len(p), 1), np.float32)
        _check(self.lib.yv_calc_optical_flow_pyr_lk(self.handle, _ptr(prev), _ptr(nxt), H, W, W, _ptr(p), len(p), win,
                                                    max_level, max_count, eps, min_eig, _ptr(out), _ptr(st),
                                                    _ptr(err)), "yv_calc_optical_flow_pyr_lk")
        return out, st[:len(p)].astype(bool), err[:len(p)]

    def find_essential(self, pts1, pts2, focal=718.8560, pp=(607.1928, 185.2157), prob=0.999, threshold=1.0):
        """cv::findEssentialMat(pts1, pts2, focal, pp, RANSAC, prob, threshold, mask) (src/LoopHandler.cc:239)
        -> (found, E [3, 3], mask [n] bool).  Points: (x, y) pixels as the reference passes them."""
        p1 = np.ascontiguousarray(pts1, np.float32).reshape(-1, 2)
        p2 = np.ascontiguousarray(pts2, np.float32).reshape(-1, 2)
        if len(p1) != len(p2):
            raise ValueError("pts1 and pts2 differ in length")
        E = np.zeros(9, np.float64)
        mask = np.zeros(max(len(p1), 1), np.uint8)
        found = ctypes.c_int(0)
        _check(self.lib.yv_find_essential(self.handle, _ptr(p1), _ptr(p2), len(p1), focal, pp[0], pp[1], prob,
                                          threshold, _ptr(E), _ptr(mask), ctypes.byref(found)), "yv_find_essential")
        return bool(found.value), E.reshape(3, 3), mask[:len(p1)].astype(bool)

    def recover_pose(self, E, pts1, pts2, K):
        """cv::recoverPose(E, pts1, pts2, K, R, t) (src/LoopHandler.cc:256) -> (good, R [3, 3], t [3])."""
        E = np.ascontiguousarray(E, np.float64).reshape(9)
        p1 = np.ascontiguousarray(pts1, np.float32).reshape(-1, 2)
        p2 = np.ascontiguousarray(pts2, np.float32).reshape(-1, 2)
        K = np.ascontiguousarray(K, np.float64).reshape(9)
        R = np.zeros(9, np.float64)
        t = np.zeros(3, np.float64)
        good = ctypes.c_int(0)
        _check(self.lib.yv_recover_pose(self.handle, _ptr(E), _ptr(p1), _ptr(p2), len(p1), _ptr(K), _ptr(R), _ptr(t),
                                        ctypes.byref(good)), "yv_recover_pose")
        return good.value, R.reshape(3, 3), t

    def f_ransac(self, matches: np.ndarray, samples: np.ndarray, thr: float = 0.1):
        """_3DHandler::getFRANSAC -> (found, F [3,3], max_inliers)."""
        m = np.ascontiguousarray(matches, dtype=MATCH_DTYPE)
        smp = np.ascontiguousarray(samples, dtype=np.int32).reshape(-1, 8)
        F = np.zeros(9)
        mi, found = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.yv_f_ransac(self.handle, _ptr(m), len(m), _ptr(smp), len(smp), thr, _ptr(F),
                                    ctypes.byref(mi), ctypes.byref(found)), "yv_f_ransac")
        return bool(found.value), F.reshape(3, 3), mi.value

    def triangulate(self, pose_a, pose_b, K, matches: np.ndarray):
        """triangulate2View per-match part -> (n_ok, Xw [n,3], ok [n] bool)."""
        m = np.ascontiguousarray(matches, dtype=MATCH_DTYPE)
        pa, pb, k = _f64(pose_a, 7), _f64(pose_b, 7), _f64(K, 9)
        X = np.zeros((max(len(m), 1), 3))
        ok = np.zeros(max(len(m), 1), np.uint8)
        n = ctypes.c_int()
        _check(self.lib.yv_triangulate(self.handle, _ptr(pa), _ptr(pb), _ptr(k), _ptr(m), len(m), _ptr(X), _ptr(ok),
                                       ctypes.byref(n)), "yv_triangulate")
        return n.value, X[:len(m)], ok[:len(m)].astype(bool)

    def world2camera(self, X, pose, K):
        X = _f64(X, (-1, 3))
        out = np.zeros_like(X)
        _check(self.lib.yv_world2camera(self.handle, _ptr(X), len(X), _ptr(_f64(pose, 7)), _ptr(_f64(K, 9)),
                                        _ptr(out)), "yv_world2camera")
        return out

    def ba_ldlt(self, S, b):
        """The BA's reduced-system solver alone (yv_ba_debug_ldlt): Eigen LDLT with diagonal pivoting of the symmetric S,
        x = S^-1 b. -> (x, isPositive)."""
        S = np.ascontiguousarray(S, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        n = len(b)
        x = np.zeros(n)
        ok = ctypes.c_int()
        _check(self.lib.yv_ba_debug_ldlt(self.handle, S.ctypes.data, n, b.ctypes.data, x.ctypes.data, ctypes.byref(ok)),
               "yv_ba_debug_ldlt")
        return x, bool(ok.value)

    def pose_lm(self, X, uv, K, pose):
        """LoopHandler::optimizePoseOnly -> (pose [7], outlier [n] bool, inliers)."""
        X, uv = _f64(X, (-1, 3)), _f64(uv, (-1, 2))
        T = _f64(pose, 7).copy()
        out = np.zeros(max(len(X), 1), np.uint8)
        inl = ctypes.c_int()
        _check(self.lib.yv_pose_lm(self.handle, _ptr(X), _ptr(uv), len(X), _ptr(_f64(K, 9)), _ptr(T), _ptr(out),
                                   ctypes.byref(inl)), "yv_pose_lm")
        return T, out[:len(X)].astype(bool), inl.value

    def pose_gn(self, X, uv, K, pose):
        """bundleAdjustmentGaussNewton -> (pose [7], accepted iterations)."""
        X, uv = _f64(X, (-1, 3)), _f64(uv, (-1, 2))
        T = _f64(pose, 7).copy()
        it = ctypes.c_int()
        _check(self.lib.yv_pose_gn(self.handle, _ptr(X), _ptr(uv), len(X), _ptr(_f64(K, 9)), _ptr(T),
                                   ctypes.byref(it)), "yv_pose_gn")
        return T, it.value



_live_contexts: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _close_all() -> None:
    """Release every context (and its batches) before torch / the HIP runtime tear down."""
    for c in list(_live_contexts):
        try:
            c.close()
        except Exception:
            pass


class Context(_GeomMixin):
    """One yv_ctx: a GPU, a HIP stream and the algorithm constants."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        _check(self.lib.yv_create(device, ctypes.byref(h)), f"yv_create(device={device})")
        self.handle = h
        self.device = device
        _live_contexts.add(self)

    def close(self) -> None:
        if self.handle:
            # batches, LK / essential workspaces, bundle adjusters and their windows hold this context (its stream
            # and device state): destroy them first, windows before their adjusters, never one after the context
            owned = list(getattr(self, "_owned", ()))
            for o in sorted(owned, key=lambda o: o._close_rank):
                o.close()
            self.lib.yv_destroy(self.handle)
            self.handle = None

    def _own(self, obj) -> None:
        """Register a workspace that holds this context, so close() destroys it first."""
        if not hasattr(self, "_owned"):
            self._owned = weakref.WeakSet()
        self._owned.add(obj)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return self.lib.yv_stream(self.handle) or 0

    @property
    def side_stream(self) -> int:
        """The context's second stream, on a hardware queue of its own (yv_side_stream)."""
        s = self.lib.yv_side_stream(self.handle)
        if not s:
            raise YavoError("yv_side_stream failed")
        return s

    def sync(self) -> None:
        _check(self.lib.yv_sync(self.handle), "yv_sync")

    def download(self, dev_ptr: int, dtype, count: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        """Copy `count` elements of `dtype` from device memory to a new host array, or into `out` (contiguous,
        e.g. a pinned buffer: a DMA instead of the pageable staging copy)."""
        if out is None:
            out = np.zeros(max(count, 1), dtype=dtype)
        else:
            out = out.reshape(-1).view(dtype)
            if not out.flags["C_CONTIGUOUS"] or out.size < count:
                raise ValueError("download: `out` must be contiguous and hold `count` elements")
        nbytes = out.dtype.itemsize * count
        _check(self.lib.yv_download(self.handle, _ptr(out), ctypes.c_void_p(dev_ptr), nbytes), "yv_download")
        return out[:count]

    def upload(self, dev_ptr: int, host: np.ndarray) -> None:
        h = np.ascontiguousarray(host)
        _check(self.lib.yv_upload(self.handle, ctypes.c_void_p(dev_ptr), _ptr(h), h.nbytes), "yv_upload")

    def set_fast_params(self, intensity_threshold: int = 40, max_corners: int = 2000) -> None:
        _check(self.lib.yv_set_fast_params(self.handle, intensity_threshold, max_corners), "yv_set_fast_params")

    def set_harris_eigen(self, flavour: int = 0) -> None:
        """cv::eigen flavour of the Harris response: 0 = OpenCV JacobiImpl_ (default), 1 = HAVE_EIGEN (Eigen 3.4)."""
        _check(self.lib.yv_set_harris_eigen(self.handle, int(flavour)), "yv_set_harris_eigen")

    def set_brief_offsets(self, offsets: np.ndarray) -> None:
        o = np.ascontiguousarray(offsets, dtype=np.int8).reshape(256, 4)
        _check(self.lib.yv_set_brief_offsets(self.handle, _ptr(o)), "yv_set_brief_offsets")

    def set_blur_kernel(self, k9: np.ndarray) -> None:
        k = np.ascontiguousarray(k9, dtype=np.uint16).reshape(9)
        _check(self.lib.yv_set_blur_kernel(self.handle, _ptr(k)), "yv_set_blur_kernel")

    # ---- host-pointer drop-in calls ----
    def detect(self, img: np.ndarray, max_kp: int = 2000) -> Tuple[np.ndarray, np.ndarray, int]:
        """FastDetector::getFastFeatures -> (rc [n,2] int32 (row, col), resp [n] float32, n_candidates)."""
        img = np.ascontiguousarray(img, dtype=np.uint8)
        H, W = img.shape
        rc = np.zeros((max(max_kp, 1), 2), np.int32)
        resp = np.zeros(max(max_kp, 1), np.float32)
        n, nc = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.yv_detect(self.handle, _ptr(img), H, W, W, max_kp, _ptr(rc), _ptr(resp), ctypes.byref(n),
                                  ctypes.byref(nc)), "yv_detect")
        return rc[:n.value].copy(), resp[:n.value].copy(), nc.value

    def describe(self, img: np.ndarray, rc: np.ndarray) -> np.ndarray:
        """Brief::computeBrief -> KEYPOINT_DTYPE array (points inside checkBoundry)."""
        img = np.ascontiguousarray(img, dtype=np.uint8)
        H, W = img.shape
        rc = np.ascontiguousarray(rc, dtype=np.int32).reshape(-1, 2)
        out = np.zeros(max(len(rc), 1), KEYPOINT_DTYPE)
        m = ctypes.c_int()
        _check(self.lib.yv_describe(self.handle, _ptr(img), H, W, W, _ptr(rc), len(rc), _ptr(out), ctypes.byref(m)),
               "yv_describe")
        return out[:m.value].copy()

    def match_features(self, q: np.ndarray, t: np.ndarray) -> np.ndarray:
        """Brief::matchFeatures -> MATCH_DTYPE array (one per query)."""
        q = np.ascontiguousarray(q, dtype=KEYPOINT_DTYPE)
        t = np.ascontiguousarray(t, dtype=KEYPOINT_DTYPE)
        out = np.zeros(max(len(q), 1), MATCH_DTYPE)
        _check(self.lib.yv_match_features(self.handle, _ptr(q), len(q), _ptr(t), len(t), _ptr(out)),
               "yv_match_features")
        return out[:len(q)].copy()

    def filter_matches(self, matches: np.ndarray, thr: int = 20) -> np.ndarray:
        """Brief::removeOutliers -> MATCH_DTYPE array."""
        m = np.ascontiguousarray(matches, dtype=MATCH_DTYPE)
        out = np.zeros(max(len(m), 1), MATCH_DTYPE)
        n = ctypes.c_int()
        _check(self.lib.yv_filter_matches(self.handle, _ptr(m), len(m), thr, _ptr(out), ctypes.byref(n)),
               "yv_filter_matches")
        return out[:n.value].copy()




class Batch:
    """Device-resident batched pipeline (yv_batch): detect -> describe -> match -> removeOutliers."""

    _close_rank = 2

    def __init__(self, ctx: Context, max_images: int, H: int, W: int, max_kp: int = 2000, max_pairs: int = 0):
        self.ctx = ctx
        self.lib = ctx.lib
        h = ctypes.c_void_p()
        _check(self.lib.yv_batch_create(ctx.handle, max_images, H, W, max_kp, max_pairs, ctypes.byref(h)),
               "yv_batch_create")
        self.handle = h
        self.max_images, self.H, self.W, self.max_kp, self.max_pairs = max_images, H, W, max_kp, max_pairs
        ctx._own(self)

    def close(self) -> None:
        if self.handle:
            self.lib.yv_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_pairs(self, pairs) -> None:
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1, 2))
        _check(self.lib.yv_batch_set_pairs(self.handle, _ptr(p), len(p)), "yv_batch_set_pairs")
        self.n_pairs = len(p)

    def run(self, d_images: int, n_images: int, stride: int, pitch: int, match_thr: int = 20, carry_from: int = -1,
            stream: int = 0) -> None:
        _check(self.lib.yv_batch_run(self.handle, ctypes.c_void_p(d_images), n_images, stride, pitch, match_thr,
                                     carry_from, ctypes.c_void_p(stream) if stream else None), "yv_batch_run")

    def set_tracks(self, tracks, K, T_right) -> None:
        """tracks [n][2] = (stereo pair index, temporal pair index); K 3x3; T_right the right camera pose."""
        t = np.ascontiguousarray(np.asarray(tracks, dtype=np.int32).reshape(-1, 2))
        _check(self.lib.yv_batch_set_tracks(self.handle, _ptr(t), len(t), _ptr(_f64(K, 9)), _ptr(_f64(T_right, 7))),
               "yv_batch_set_tracks")
        self.n_tracks = len(t)

    def track(self, d_priors: int, d_poses: int, stream: int = 0) -> None:
        _check(self.lib.yv_batch_track(self.handle, ctypes.c_void_p(d_priors), ctypes.c_void_p(d_poses),
                                       ctypes.c_void_p(stream) if stream else None), "yv_batch_track")

    def track_map(self, d_priors: int, d_poses: int, first_frame: int, kf_every: int, d_block: int, max_kf: int,
                  stream: int = 0) -> None:
        """yv_batch_track + the chunk's shared-map block (yv_batch_track_map; layout in ya_vo_amd/map.py)."""
        _check(self.lib.yv_batch_track_map(self.handle, ctypes.c_void_p(d_priors), ctypes.c_void_p(d_poses),
                                           first_frame, kf_every, ctypes.c_void_p(d_block), max_kf,
                                           ctypes.c_void_p(stream) if stream else None), "yv_batch_track_map")

    def map_wait(self, stream: int) -> None:
        """`stream` waits for the last map block (yv_batch_map_wait)."""
        _check(self.lib.yv_batch_map_wait(self.handle, ctypes.c_void_p(stream)), "yv_batch_map_wait")

    def map_release(self, stream: int) -> None:
        """The next map block write waits for the work on `stream` so far (yv_batch_map_release)."""
        _check(self.lib.yv_batch_map_release(self.handle, ctypes.c_void_p(stream)), "yv_batch_map_release")

    def set_track_overlap(self, on=True) -> None:
        """Run each track's pose LM on the batch's own stream beside the next run (yv_batch_set_track_overlap):
        True / 1 after the edge build, 2 / 3 / 4 deferred until the next run's detect / describe / top-K stage,
        False / 0 in order."""
        mode = int(on) if not isinstance(on, bool) else (1 if on else 0)
        _check(self.lib.yv_batch_set_track_overlap(self.handle, mode), "yv_batch_set_track_overlap")

    def set_track_lk(self, image_step: int, win: int = 11, max_level: int = 3, max_count: int = 30, eps: float = 0.01,
                     min_eig: float = 0.001) -> None:
        """LK tracking mode (yv_batch_set_track_lk): tracks become {stereo pair of frame k-1, image of frame k}."""
        _check(self.lib.yv_batch_set_track_lk(self.handle, image_step, win, max_level, max_count, eps, min_eig),
               "yv_batch_set_track_lk")

    def track_sync(self) -> None:
        _check(self.lib.yv_batch_track_sync(self.handle), "yv_batch_track_sync")

    def enable_timing(self, on=True) -> None:
        """on: False/0 off, True/1 every stage, 2 the detect kernel only (yavo.h)."""
        mode = 2 if (not isinstance(on, bool) and on == 2) else (1 if on else 0)
        _check(self.lib.yv_batch_enable_timing(self.handle, mode), "yv_batch_enable_timing")

    def stage_times(self) -> Tuple[np.ndarray, int]:
        ms = np.zeros(8, np.float32)
        n = ctypes.c_int()
        _check(self.lib.yv_batch_stage_times(self.handle, _ptr(ms), ctypes.byref(n)), "yv_batch_stage_times")
        return ms[:YV_NUM_STAGES].copy(), n.value

    def view(self) -> _BatchView:
        v = _BatchView()
        _check(self.lib.yv_batch_view_get(self.handle, ctypes.byref(v)), "yv_batch_view_get")
        return v


class Lk:
    """Batched pyramidal LK workspace (yv_lk): build pyramids of device images, track point lists per pair."""

    _close_rank = 2

    def __init__(self, ctx: "Context", max_images: int, H: int, W: int, win: int = 11, max_level: int = 3):
        self.ctx, self.lib = ctx, ctx.lib
        h = ctypes.c_void_p()
        _check(self.lib.yv_lk_create(ctx.handle, max_images, H, W, win, max_level, ctypes.byref(h)), "yv_lk_create")
        self.handle = h
        ctx._own(self)
        self.levels = self.lib.yv_lk_levels(h)

    def close(self) -> None:
        if self.handle:
            self.lib.yv_lk_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def build(self, d_images: int, n_images: int, stride: int, pitch: int, stream: int = 0) -> None:
        _check(self.lib.yv_lk_build(self.handle, ctypes.c_void_p(d_images), n_images, stride, pitch,
                                    ctypes.c_void_p(stream) if stream else None), "yv_lk_build")

    def level(self, image: int, level: int):
        """(d_img, img_stride, d_deriv, deriv_stride, H, W) of one pyramid level of the last build (yv_lk_level)."""
        img, st, der, dst = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_void_p(), ctypes.c_int()
        H, W = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.yv_lk_level(self.handle, image, level, ctypes.byref(img), ctypes.byref(st), ctypes.byref(der),
                                    ctypes.byref(dst), ctypes.byref(H), ctypes.byref(W)), "yv_lk_level")
        return img.value, st.value, der.value, dst.value, H.value, W.value

    def track(self, d_pairs: int, n_pairs: int, d_pts: int, d_counts: int, pts_stride: int, d_next: int,
              d_status: int, d_err: int, max_count: int = 30, eps: float = 0.01, min_eig: float = 0.001,
              stream: int = 0) -> None:
        _check(self.lib.yv_lk_track_batch(self.handle, ctypes.c_void_p(d_pairs), n_pairs, ctypes.c_void_p(d_pts),
                                          ctypes.c_void_p(d_counts), pts_stride, max_count, eps, min_eig,
                                          ctypes.c_void_p(d_next), ctypes.c_void_p(d_status), ctypes.c_void_p(d_err),
                                          ctypes.c_void_p(stream) if stream else None), "yv_lk_track_batch")


class Essential:
    """Batched cv::findEssentialMat (RANSAC) + cv::recoverPose workspace (yv_essential)."""

    _close_rank = 2

    def __init__(self, ctx: "Context", max_pairs: int, max_points: int, max_iters: int = 1000):
        self.ctx, self.lib = ctx, ctx.lib
        h = ctypes.c_void_p()
        _check(self.lib.yv_essential_create(ctx.handle, max_pairs, max_points, max_iters, ctypes.byref(h)),
               "yv_essential_create")
        self.handle = h
        ctx._own(self)

    def close(self) -> None:
        if self.handle:
            self.lib.yv_essential_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def find(self, d_pts1: int, d_pts2: int, d_counts: int, n_pairs: int, pts_stride: int, d_E: int, d_found: int,
             d_mask: int = 0, d_stats: int = 0, focal: float = 718.8560, pp=(607.1928, 185.2157), prob: float = 0.999,
             threshold: float = 1.0, stream: int = 0) -> None:
        _check(self.lib.yv_find_essential_batch(self.handle, ctypes.c_void_p(d_pts1), ctypes.c_void_p(d_pts2),
                                                ctypes.c_void_p(d_counts), n_pairs, pts_stride, focal, pp[0], pp[1],
                                                prob, threshold, ctypes.c_void_p(d_E),
                                                ctypes.c_void_p(d_mask) if d_mask else None, ctypes.c_void_p(d_found),
                                                ctypes.c_void_p(d_stats) if d_stats else None,
                                                ctypes.c_void_p(stream) if stream else None), "yv_find_essential_batch")

    def recover(self, d_E: int, d_pts1: int, d_pts2: int, d_counts: int, n_pairs: int, pts_stride: int, K,
                d_R: int, d_t: int, d_good: int = 0, stream: int = 0) -> None:
        K = np.ascontiguousarray(K, np.float64).reshape(9)
        _check(self.lib.yv_recover_pose_batch(self.handle, ctypes.c_void_p(d_E), ctypes.c_void_p(d_pts1),
                                              ctypes.c_void_p(d_pts2), ctypes.c_void_p(d_counts), n_pairs, pts_stride,
                                              _ptr(K), ctypes.c_void_p(d_R), ctypes.c_void_p(d_t),
                                              ctypes.c_void_p(d_good) if d_good else None,
                                              ctypes.c_void_p(stream) if stream else None), "yv_recover_pose_batch")


class BundleAdjuster:
    """Sliding-window bundle adjustment (yv_ba): g2o Levenberg-Marquardt over BlockSolver_6_3 with the reference's
    projection edge (include/Optimizer.hpp:64-126) between keyframe poses and landmarks; poses SE3d::data() of T_cw,
    the first n_fixed held fixed."""

    _close_rank = 1

    def __init__(self, ctx: "Context", max_poses: int, max_landmarks: int, max_edges: int):
        self.ctx, self.lib = ctx, ctx.lib
        h = ctypes.c_void_p()
        _check(self.lib.yv_ba_create(ctx.handle, max_poses, max_landmarks, max_edges, ctypes.byref(h)), "yv_ba_create")
        self.handle = h
        ctx._own(self)  # Context.close destroys it (and its windows) before the context: no leaked workspace

    def close(self) -> None:
        if self.handle:
            for w in list(getattr(self, "_windows", ())):  # a window holds its adjuster
                w.close()
            self.lib.yv_ba_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream: int = 0) -> None:
        """Run on a caller stream (yv_ba_set_stream; 0 = the context's stream)."""
        _check(self.lib.yv_ba_set_stream(self.handle, ctypes.c_void_p(stream) if stream else None),
               "yv_ba_set_stream")

    def set_control(self, on_device: bool = True) -> None:
        """LM control on the device (default: no read-back per trial) or on the host (yv_ba_set_control)."""
        _check(self.lib.yv_ba_set_control(self.handle, 1 if on_device else 0), "yv_ba_set_control")

    def resumes(self) -> int:
        """Suspended trial loops the device LM resumed from the host so far (yv_ba_debug_resumes)."""
        return int(self.lib.yv_ba_debug_resumes(self.handle))

    def set_problem(self, n_poses: int, n_fixed: int, n_landmarks: int, edge_pose, edge_landmark, meas, K) -> None:
        self._ep = np.ascontiguousarray(edge_pose, np.int32).reshape(-1)
        self._el = np.ascontiguousarray(edge_landmark, np.int32).reshape(-1)
        self._meas = _f64(meas, (-1, 2))
        if not (len(self._ep) == len(self._el) == len(self._meas)):
            raise ValueError("edge arrays differ in length")
        K = _f64(K, (9,))
        _check(self.lib.yv_ba_set_problem(self.handle, n_poses, n_fixed, n_landmarks, _ptr(self._ep), _ptr(self._el),
                                          _ptr(self._meas), len(self._ep), _ptr(K)), "yv_ba_set_problem")
        self.n_poses, self.n_landmarks = n_poses, n_landmarks

    def solve(self, poses, landmarks, max_iters: int = 10):
        """-> (poses [P, 7], landmarks [L, 3], chi2 log [iters + 1], iterations run)."""
        poses = _f64(poses, (-1, 7)).copy()
        X = _f64(landmarks, (-1, 3)).copy()
        if len(poses) != self.n_poses or len(X) != self.n_landmarks:
            raise ValueError("estimate does not match the problem")
        log = np.zeros(max_iters + 1)
        it = ctypes.c_int(0)
        _check(self.lib.yv_ba_solve(self.handle, _ptr(poses), _ptr(X), max_iters, _ptr(log), ctypes.byref(it)),
               "yv_ba_solve")
        return poses, X, log[: it.value + 1], it.value


class BaWindow:
    """The chained front end's sliding BA window on the device (yv_ba_window_*; include/yavo/yavo_geom.h): frame
    records from placed map blocks, the window graph built and solved by `ba` and written back in HBM."""

    _close_rank = 0

    def __init__(self, ba: "BundleAdjuster", max_lm: int, max_kf: int):
        self.ba, self.lib = ba, ba.lib
        h = ctypes.c_void_p()
        _check(self.lib.yv_ba_window_create(ba.handle, max_lm, max_kf, ctypes.byref(h)), "yv_ba_window_create")
        self.handle, self.max_lm = h, max_lm
        if not hasattr(ba, "_windows"):
            ba._windows = weakref.WeakSet()
        ba._windows.add(self)
        ba.ctx._own(self)

    def close(self) -> None:
        if self.handle:
            self.lib.yv_ba_window_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, n_frames: int) -> None:
        """Size the record store for n_frames frames up front (yv_ba_window_reserve: no growth inside the loop)."""
        _check(self.lib.yv_ba_window_reserve(self.handle, int(n_frames)), "yv_ba_window_reserve")

    def add_block(self, d_block: int, first_frame: int, n_frames: int, d_edge_uv: int, d_edge_query: int,
                  d_matches: int, max_kp: int, stream: int = 0) -> None:
        _check(self.lib.yv_ba_window_add_block(self.handle, ctypes.c_void_p(d_block), first_frame, n_frames,
                                               ctypes.c_void_p(d_edge_uv), ctypes.c_void_p(d_edge_query),
                                               ctypes.c_void_p(d_matches), max_kp,
                                               ctypes.c_void_p(stream) if stream else None), "yv_ba_window_add_block")

    def solve(self, first: int, n: int, n_fixed: int, K, max_iters: int, d_anchor: int = 0):
        """-> (solved, chi2 log [iters + 1], iterations run)"""
        K = _f64(K, (9,))
        log = np.zeros(max_iters + 1)
        it, ok = ctypes.c_int(0), ctypes.c_int(0)
        _check(self.lib.yv_ba_window_solve(self.handle, first, n, n_fixed, _ptr(K), max_iters,
                                           ctypes.c_void_p(d_anchor) if d_anchor else None, _ptr(log),
                                           ctypes.byref(it), ctypes.byref(ok)), "yv_ba_window_solve")
        return bool(ok.value), log[: it.value + 1], it.value

    def solve_begin(self, first: int, n: int, n_fixed: int, K, max_iters: int, d_anchor: int = 0) -> None:
        """Enqueue the solve (yv_ba_window_solve_begin) and return; solve_end collects it."""
        self._iters = max_iters
        _check(self.lib.yv_ba_window_solve_begin(self.handle, first, n, n_fixed, _ptr(_f64(K, (9,))), max_iters,
                                                 ctypes.c_void_p(d_anchor) if d_anchor else None),
               "yv_ba_window_solve_begin")

    def solve_end(self):
        """-> (solved, chi2 log [iters + 1], iterations run) of the solve solve_begin enqueued"""
        log = np.zeros(self._iters + 1)
        it, ok = ctypes.c_int(0), ctypes.c_int(0)
        _check(self.lib.yv_ba_window_solve_end(self.handle, _ptr(log), ctypes.byref(it), ctypes.byref(ok)),
               "yv_ba_window_solve_end")
        return bool(ok.value), log[: it.value + 1], it.value

    def read(self, frame: int):
        """-> (T_wc [7], edge ids [n], X [n, 3], uv_own [n, 2], uv_prev [n, 2])"""
        T = np.zeros(7)
        e = np.zeros(self.max_lm, np.int32)
        X = np.zeros((self.max_lm, 3))
        uo = np.zeros((self.max_lm, 2))
        up = np.zeros((self.max_lm, 2))
        n = ctypes.c_int(0)
        _check(self.lib.yv_ba_window_read(self.handle, frame, _ptr(T), ctypes.byref(n), _ptr(e), _ptr(X), _ptr(uo),
                                          _ptr(up), self.max_lm), "yv_ba_window_read")
        k = n.value
        return T, e[:k].copy(), X[:k].copy(), uo[:k].copy(), up[:k].copy()

    def trajectory(self, first: int, n: int) -> np.ndarray:
        T = np.zeros((n, 7))
        _check(self.lib.yv_ba_window_trajectory(self.handle, first, n, _ptr(T)), "yv_ba_window_trajectory")
        return T

    def export_block(self, first: int, n: int, chunk_frame: int, frame_id_offset: int, d_block: int, max_kf: int,
                     lm_stride: int, stream: int = 0) -> None:
        """Recorded frames [first, first + n) as a sequence shard's map block (yv_ba_window_export_block)."""
        _check(self.lib.yv_ba_window_export_block(self.handle, first, n, chunk_frame, frame_id_offset,
                                                  ctypes.c_void_p(d_block), max_kf, lm_stride,
                                                  ctypes.c_void_p(stream) if stream else None),
               "yv_ba_window_export_block")
