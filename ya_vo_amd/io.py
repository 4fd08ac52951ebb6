"""Frame I/O and formats (include/yavo/yavo_io.h): PNG decode as cv::imread(path, 0), the sorted
KITTI sequence listing (getFilesInFolder / generatePathTrain), calib.txt (getCalibParams / parseCalibString), a
threaded decoder feeding HBM through pinned staging, and the KITTI odometry pose format.  All native (libyavo.so)."""
import ctypes

import numpy as np

from . import YV_OK, YavoError, _check, load_library


def _lib():
    return load_library()


def png_decode_gray(data: bytes) -> np.ndarray:
    """PNG bytes -> uint8 [H, W] (cv::imread(..., IMREAD_GRAYSCALE) semantics, see yavo_io.h)."""
    lib = _lib()
    buf = np.frombuffer(data, np.uint8)
    H, W = ctypes.c_int(0), ctypes.c_int(0)
    _check(lib.yv_png_info(buf.ctypes.data, len(buf), ctypes.byref(H), ctypes.byref(W)), "yv_png_info")
    out = np.zeros((H.value, W.value), np.uint8)
    _check(lib.yv_png_decode_gray(buf.ctypes.data, len(buf), out.ctypes.data, W.value, H.value, W.value),
           "yv_png_decode_gray")
    return out


def imread_gray(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        return png_decode_gray(f.read())


def png_write_gray(path: str, img) -> None:
    """8-bit grey image -> PNG file (Sub rows, deflate level 1 + Z_RLE as cv::imwrite writes; yv_png_write_gray).  Releases the GIL (ctypes)."""
    a = np.ascontiguousarray(img, np.uint8)
    _check(_lib().yv_png_write_gray(path.encode(), a.ctypes.data, a.shape[0], a.shape[1], a.shape[1]),
           "yv_png_write_gray")


def parse_calib_string(line: str) -> np.ndarray:
    """parseCalibString (src/Utils.cc:4-28) -> 4x4 float64 (missing values 0)."""
    out = np.zeros(16, np.float64)
    n = _lib().yv_parse_calib_string(line.encode(), out.ctypes.data)
    if n < 0:
        raise YavoError(n, "yv_parse_calib_string")
    return out.reshape(4, 4)


class Sequence:
    """A KITTI odometry sequence directory (<dir>/image_0/, image_1/, calib.txt)."""

    def __init__(self, sequence_dir: str, stereo: bool = False):
        self.lib = _lib()
        h = ctypes.c_void_p()
        _check(self.lib.yv_seq_open(sequence_dir.encode(), int(stereo), ctypes.byref(h)), "yv_seq_open")
        self.handle = h
        self.stereo = stereo
        H, W = ctypes.c_int(0), ctypes.c_int(0)
        _check(self.lib.yv_seq_size(h, ctypes.byref(H), ctypes.byref(W)), "yv_seq_size")
        self.H, self.W = H.value, W.value

    def close(self) -> None:
        if self.handle:
            self.lib.yv_seq_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return self.lib.yv_seq_frames(self.handle)

    def path(self, frame: int, side: int = 0) -> str:
        buf = ctypes.create_string_buffer(4096)
        n = self.lib.yv_seq_path(self.handle, frame, side, buf, len(buf))
        if n < 0:
            raise YavoError(n, "yv_seq_path")
        return buf.value.decode()

    def calib(self):
        """getCalibParams -> (P0 [4, 4], P1 [4, 4], K0 [3, 3], K1 [3, 3])."""
        P0, P1 = np.zeros(16), np.zeros(16)
        K0, K1 = np.zeros(9), np.zeros(9)
        _check(self.lib.yv_seq_calib(self.handle, P0.ctypes.data, P1.ctypes.data, K0.ctypes.data, K1.ctypes.data),
               "yv_seq_calib")
        return P0.reshape(4, 4), P1.reshape(4, 4), K0.reshape(3, 3), K1.reshape(3, 3)

    def read(self, first: int, n: int, threads: int = 0) -> np.ndarray:
        """frames [first, first + n) -> uint8 [n (x2 stereo: left, right per frame), H, W]."""
        per = 2 if self.stereo else 1
        out = np.zeros((n * per, self.H, self.W), np.uint8)
        _check(self.lib.yv_seq_read(self.handle, first, n, out.ctypes.data, self.H * self.W, threads), "yv_seq_read")
        return out

    def upload(self, ctx, first: int, n: int, d_dst: int, pitch: int = 0, threads: int = 0, stream: int = 0) -> None:
        """decode into pinned staging, then an async copy to the device buffer d_dst on stream."""
        pitch = pitch or self.H * self.W
        _check(self.lib.yv_seq_upload(self.handle, ctx.handle, first, n, ctypes.c_void_p(d_dst), pitch, threads,
                                      ctypes.c_void_p(stream) if stream else None), "yv_seq_upload")


def write_kitti_poses(path: str, poses) -> None:
    """poses [n, 7] (SE3d::data() of T_cw) -> KITTI lines of T_wc [R | t] (12 numbers)."""
    p = np.ascontiguousarray(poses, np.float64).reshape(-1, 7)
    _check(_lib().yv_write_kitti_poses(path.encode(), p.ctypes.data, len(p)), "yv_write_kitti_poses")


def read_kitti_poses(path: str, cap: int = 1 << 20) -> np.ndarray:
    """KITTI pose file -> [n, 3, 4]."""
    with open(path) as f:
        lines = sum(1 for ln in f if ln.strip())
    out = np.zeros((max(min(lines, cap), 1), 12), np.float64)
    n = ctypes.c_int(0)
    _check(_lib().yv_read_kitti_poses(path.encode(), out.ctypes.data, len(out), ctypes.byref(n)),
           "yv_read_kitti_poses")
    return out[:n.value].reshape(-1, 3, 4)


class PngDecoder:
    """PNG decoding on the GPU (yv_pngdec_*): inflate + scanline filters as kernels, one wave per image, for 8-bit
    grey non-interlaced H x W files (KITTI frames).  Calls are asynchronous on `stream` (0: the context stream)."""

    def __init__(self, ctx, max_images: int, H: int, W: int):
        self.lib = _lib()
        h = ctypes.c_void_p()
        _check(self.lib.yv_pngdec_create(ctx.handle, max_images, H, W, ctypes.byref(h)), "yv_pngdec_create")
        self.handle, self.H, self.W = h, H, W

    def decode(self, files, d_dst: int, pitch: int = 0, stream: int = 0) -> None:
        """files: list of PNG bytes objects -> device images at d_dst + i * pitch"""
        n = len(files)
        bufs = [np.frombuffer(f, np.uint8) for f in files]
        ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
        sizes = (ctypes.c_size_t * n)(*[len(b) for b in bufs])
        _check(self.lib.yv_pngdec_decode(self.handle, ptrs, sizes, n, ctypes.c_void_p(d_dst), pitch or self.H * self.W,
                                         ctypes.c_void_p(stream) if stream else None), "yv_pngdec_decode")
        self._n = n

    def upload_sequence(self, seq, first: int, n: int, d_dst: int, pitch: int = 0, threads: int = 0,
                        stream: int = 0) -> None:
        _check(self.lib.yv_seq_upload_gpu(seq.handle, self.handle, first, n, ctypes.c_void_p(d_dst),
                                          pitch or self.H * self.W, threads, ctypes.c_void_p(stream) if stream else None),
               "yv_seq_upload_gpu")
        self._n = n * (2 if seq.stereo else 1)

    def upload_frames(self, seq, frames, d_dst: int, pitch: int = 0, threads: int = 0, stream: int = 0) -> None:
        """the listed frames in one decode: frame frames[i] -> images (2 i, 2 i + 1) (stereo) or i at d_dst"""
        fr = np.ascontiguousarray(frames, dtype=np.int32)
        _check(self.lib.yv_seq_upload_gpu_frames(seq.handle, self.handle, fr.ctypes.data, len(fr), ctypes.c_void_p(d_dst),
                                                 pitch or self.H * self.W, threads,
                                                 ctypes.c_void_p(stream) if stream else None),
               "yv_seq_upload_gpu_frames")
        self._n = len(fr) * (2 if seq.stereo else 1)

    def set_checks(self, crc: int = 1, adler: int = 1) -> None:
        """integrity checks of the following decodes: IDAT chunk CRC-32, zlib Adler-32 (both on by default)"""
        _check(self.lib.yv_pngdec_set_checks(self.handle, int(crc), int(adler)), "yv_pngdec_set_checks")

    def status(self):
        """(codes of the last call's images, images failed in every call since the previous status); waits for the
        last call.  Codes: 7 = an IDAT chunk's CRC-32, 8 = the zlib Adler-32 trailer (yavo_io.h); failed images are
        zero-filled on the device."""
        bad = ctypes.c_int()
        codes = np.zeros(max(getattr(self, "_n", 0), 1), np.int32)
        _check(self.lib.yv_pngdec_status(self.handle, codes.ctypes.data, ctypes.byref(bad)), "yv_pngdec_status")
        return codes, bad.value

    def close(self) -> None:
        if self.handle:
            self.lib.yv_pngdec_destroy(self.handle)
            self.handle = None
