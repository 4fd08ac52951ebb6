/*
 * yavo_io.h -- frame I/O and formats on either side of the hot path, behind the same C ABI as
 * yavo.h (status codes, caller-owned buffers).  Replaces the reference's:
 *   getFilesInFolder          src/Utils.cc:31-36       directory entries sorted as boost::filesystem::path
 *   generatePathTrain         src/LoopHandler.cc:37-57  <seq>/image_0/ (and image_1/ for stereo)
 *   getCalibParams            src/Utils.cc:39-62       first two lines of <seq>/calib.txt -> Camera Left / Right
 *   parseCalibString          src/Utils.cc:4-28        ' '-separated std::stod, unparsable tokens skipped
 *   cv::imread(path, 0)       src/LoopHandler.cc:919   PNG -> 8-bit grey
 * and adds the KITTI odometry pose writer / reader the reference lacks (needed for trajectory RMSE).
 */
#ifndef YAVO_IO_H
#define YAVO_IO_H

#include <stddef.h>
#include <stdint.h>

#include "yavo.h"

#ifdef __cplusplus
extern "C" {
#endif

/* PNG -> 8-bit grey as cv::imread(..., IMREAD_GRAYSCALE) does through libpng: grey 1/2/4-bit expanded to 8
 * (v * 255 / (2^d - 1)), 16-bit stripped to the high byte, alpha dropped, RGB / palette converted with libpng's
 * rgb_to_gray(0.299, 0.587) integer path (9797 R + 19234 G + 3737 B) >> 15 (R when R == G == B; no gAMA
 * linearisation).  Interlaced and 16-bit colour PNGs return YV_ERR_INVALID. */
int yv_png_info(const uint8_t* data, size_t len, int* H, int* W);
int yv_png_decode_gray(const uint8_t* data, size_t len, uint8_t* dst, int stride, int H, int W);
/* file variant: *H / *W receive the size; the image must fit cap_h x cap_w (row stride = stride) */
int yv_imread_gray(const char* path, uint8_t* dst, int stride, int cap_h, int cap_w, int* H, int* W);

/* parseCalibString: numbers of a "Pn: v0 v1 ..." line into a row-major 4x4 (missing values 0; the reference reads
 * past a 12-value vector).  Returns the count parsed. */
int yv_parse_calib_string(const char* line, double out[16]);

/* A KITTI odometry sequence directory (basePath + sequence, src/LoopHandler.cc:12-24). */
typedef struct yv_seq yv_seq;
/* stereo != 0 also lists image_1/.  Fails (YV_ERR_INVALID) when image_0/ is missing or empty. */
int yv_seq_open(const char* sequence_dir, int stereo, yv_seq** out);
void yv_seq_close(yv_seq* seq);
int yv_seq_frames(const yv_seq* seq);
/* the path of frame i (side 0 = image_0, 1 = image_1); returns its length, or an error when cap is too small */
int yv_seq_path(const yv_seq* seq, int frame, int side, char* buf, int cap);
/* getCalibParams: P0 / P1 (4x4, row-major) and their top-left 3x3 K (Camera::K); YV_ERR_INVALID without calib.txt */
int yv_seq_calib(const yv_seq* seq, double P0[16], double P1[16], double K0[9], double K1[9]);
/* size of frame 0 of image_0 */
int yv_seq_size(const yv_seq* seq, int* H, int* W);
/* decode frames [first, first + n) into host memory, images of pitch bytes, rows of W bytes; stereo sequences
 * store left, right per frame (2n images).  threads <= 0 picks the host's hardware concurrency (at most 64). */
int yv_seq_read(yv_seq* seq, int first, int n, uint8_t* dst, int64_t pitch, int threads);
/* the same decode into the sequence's pinned staging (two slots, reused once their copy completed) followed by an
 * async copy to d_dst on stream (NULL: the context stream of ctx) -- PCIe overlapped with the caller's kernels */
int yv_seq_upload(yv_seq* seq, struct yv_ctx* ctx, int first, int n, uint8_t* d_dst, int64_t pitch, int threads,
                  void* stream);

/* PNG decoding on the GPU (yavo_inflate.hip): the inflate (RFC 1950/1951) and the scanline filters run as kernels,
 * one wave per image; the host only reads the files and gathers each image's IDAT stream into pinned staging.
 * Formats: 8-bit grey, non-interlaced, H x W (every KITTI frame). A file in any other format (yv_png_decode_gray /
 * yv_seq_upload decode every format on the host), or missing, unreadable or truncated, fails alone with code 9: its
 * output is zero-filled and the call's other images decode, as cv::imread fails per file.  Calls of one decoder are ordered on
 * the stream they are given (use one stream per decoder); the staging of a call is reused two calls later, after its
 * copy completed. */
typedef struct yv_pngdec yv_pngdec;
int yv_pngdec_create(struct yv_ctx* ctx, int max_images, int H, int W, yv_pngdec** out);
void yv_pngdec_destroy(yv_pngdec* d);
/* n PNG files in host memory (files[i], sizes[i] bytes) -> device images at d_dst + i * pitch, rows of W bytes;
 * asynchronous on stream (NULL: the context stream) */
int yv_pngdec_decode(yv_pngdec* d, const uint8_t* const* files, const size_t* sizes, int n, uint8_t* d_dst,
                     int64_t pitch, void* stream);
/* the frames [first, first + n) of a sequence (left, right per frame for stereo), read by `threads` host threads
 * straight into the pinned staging, then decoded as yv_pngdec_decode does */
int yv_seq_upload_gpu(yv_seq* seq, yv_pngdec* d, int first, int n, uint8_t* d_dst, int64_t pitch, int threads,
                      void* stream);
/* the same for the listed frames: frame frames[i] -> images per * i (+ 1 for its right image) at d_dst, in one decode
 * (e.g. a shard's frames then its halo frame) */
int yv_seq_upload_gpu_frames(yv_seq* seq, yv_pngdec* d, const int* frames, int n, uint8_t* d_dst, int64_t pitch,
                             int threads, void* stream);
/* waits for the last decode; codes[i] (optional, host, n of the last call) = 0 or the image's decode error
 * (1 zlib header, 2 block, 3 Huffman code, 4 output overrun, 5 stream short, 6 filter type, 7 an IDAT chunk's CRC-32,
 * 8 the zlib Adler-32 trailer: missing or wrong, 9 the file: missing, unreadable, truncated or not an 8-bit grey
 * non-interlaced H x W PNG); *n_bad = images that failed in EVERY decode since the previous
 * yv_pngdec_status call.  A failed image's device output is zero-filled (cv::imread returns an empty Mat). */
int yv_pngdec_status(yv_pngdec* d, int32_t* codes, int* n_bad);
/* the integrity checks of the following decodes (default both on, as libpng / zlib do): crc = every IDAT chunk's
 * CRC-32 (libpng png_set_crc_action), adler = the zlib Adler-32 trailer (libpng PNG_IGNORE_ADLER32 turns it off) */
int yv_pngdec_set_checks(yv_pngdec* d, int crc, int adler);

/* The writer side, for test sequences (the reference only reads PNGs): an 8-bit grey image to a PNG file, every row
 * Sub-filtered and deflated at level 1 with Z_RLE, as cv::imwrite writes PNGs (the reference's tests/epilines.png:
 * filter 1 on every row, zlib header 0x7801); rows of W bytes, stride bytes apart. */
int yv_png_write_gray(const char* path, const uint8_t* img, int H, int W, int stride);

/* KITTI odometry poses: one line per frame, the 12 row-major numbers of the 3x4 [R | t] of T_wc = T_cw^-1, for
 * poses given as Sophus SE3d::data() of T_cw ({qx, qy, qz, qw, tx, ty, tz}, yavo_geom.h). */
int yv_write_kitti_poses(const char* path, const double* poses, int n);
/* reads up to cap lines of 12 numbers (the same 3x4 layout) into out [cap][12] */
int yv_read_kitti_poses(const char* path, double* out, int cap, int* n);

#ifdef __cplusplus
}
#endif
#endif /* YAVO_IO_H */
