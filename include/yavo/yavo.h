/*
 * yavo.h -- C ABI of the MI355X-native YA_VO front end (libyavo.so, gfx950).
 *
 * Drop-in boundary for the reference's per-frame hot path.  Each host-pointer entry point replaces one
 * reference member function (cited below) with the same argument meaning; results are bit-identical
 * to the reference's integer arithmetic (FAST indices, BRIEF bits, Hamming matches) and follow the
 * reference's float arithmetic operation-for-operation where it has one.
 *
 * Conventions:
 *   - plain C, no exceptions cross the boundary; every call returns YV_OK (0) or a negative status;
 *   - caller-allocated output buffers, capacities passed in, counts returned through out-pointers;
 *   - one yv_ctx per thread and per GPU (not thread-shared); all work is issued on the ctx's HIP stream
 *     unless a stream is passed explicitly;
 *   - coordinates follow the reference: x / rc[2i] = ROW, y / rc[2i+1] = COLUMN.
 *
 * There is no CPU fallback: without a usable gfx950 device every compute entry point returns
 * YV_ERR_NODEVICE.
 */
#ifndef YAVO_H
#define YAVO_H

#include <stddef.h>
#include <stdint.h>

#include "yavo_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define YV_OK 0
#define YV_ERR_INVALID (-1)   /* bad argument (null pointer, bad size, capacity too small) */
#define YV_ERR_HIP (-2)       /* HIP runtime error */
#define YV_ERR_NODEVICE (-3)  /* no usable GPU */
#define YV_ERR_CAPACITY (-4)  /* request exceeds the batch / context capacity */

#define YV_ABI_VERSION 2

typedef struct yv_ctx yv_ctx;
typedef struct yv_batch yv_batch;

/* ---- library / context ------------------------------------------------------------------------ */
int yv_abi_version(void);
const char* yv_status_string(int status);
/* Number of visible HIP devices (0 when none); never fails. */
int yv_device_count(void);
/* Create a context on `device`: a HIP stream, default parameters (FAST threshold 40, 2000 corners,
 * the 9x9/sigma 2.5 fixed-point blur kernel, an all-zero BRIEF offset table until set). */
int yv_create(int device, yv_ctx** out);
void yv_destroy(yv_ctx* ctx);
/* The stream all yv_* calls on this context use (hipStream_t as void*). */
void* yv_stream(yv_ctx* ctx);
/* Block until all work queued on the context stream has finished. */
/* A second stream of the context on a hardware queue of its own (never the context stream's), made on first use and
 * kept until yv_destroy: work issued on it overlaps the context stream's (the sequence's BA windows). */
void* yv_side_stream(yv_ctx* ctx);
int yv_sync(yv_ctx* ctx);
/* Synchronous copies between host memory and device memory (e.g. a yv_batch_view array) on the
 * context stream. */
int yv_download(yv_ctx* ctx, void* host_dst, const void* dev_src, size_t bytes);
int yv_upload(yv_ctx* ctx, void* dev_dst, const void* host_src, size_t bytes);
/* Device memory on the context's GPU and pinned host memory, for callers without a HIP toolchain of their own (the C++
 * LoopHandler's GPU-decode look-ahead): the batch / decoder entry points take device pointers. */
int yv_device_alloc(yv_ctx* ctx, size_t bytes, void** out);
void yv_device_free(yv_ctx* ctx, void* p);
int yv_host_alloc(yv_ctx* ctx, size_t bytes, void** out);
void yv_host_free(yv_ctx* ctx, void* p);

/* FastDetector constructor constants (include/FastDetector.hpp:32-38): intensityThreshold (40) and
 * fastCornerNumThreshold (2000). */
int yv_set_fast_params(yv_ctx* ctx, int intensity_threshold, int max_corners);
/* Which cv::eigen the Harris response (src/FastDetector.cc:265) restates -- the reference's OpenCV build decides:
 * 0 (default) = OpenCV's JacobiImpl_<float> (built without Eigen), 1 = HAVE_EIGEN's
 * Eigen::SelfAdjointEigenSolver<MatrixXf> (Eigen 3.4).  Both are bit-exact against the oracle's restatements; they
 * differ from each other in the last bits of most responses. */
#define YV_HARRIS_EIGEN_JACOBI 0
#define YV_HARRIS_EIGEN_EIGEN3 1
int yv_set_harris_eigen(yv_ctx* ctx, int flavour);
/* Brief offsets table (src/BriefDescriptor.cc:4-20): 256 rows of {drow1, dcol1, drow2, dcol2},
 * each in [-8, 8]. */
int yv_set_brief_offsets(yv_ctx* ctx, const int8_t* offsets /* [256*4] */);
/* 9-tap fixed-point Gaussian (8 fractional bits, sum 256) used in place of cv::GaussianBlur
 * (src/BriefDescriptor.cc:90).  Default = OpenCV's bit-exact 9 / 2.5 kernel {12,22,31,41,44,...}.
 * Each tap must be <= 255 (YV_ERR_INVALID otherwise). */
int yv_set_blur_kernel(yv_ctx* ctx, const uint16_t* k9);

/* ---- host-pointer drop-in entry points (synchronous) --------------------------------------------- */
/* FastDetector::getFastFeatures (src/FastDetector.cc:277-369; include/FastDetector.hpp:48).
 * img: H x W u8, row stride `stride` bytes.  Writes up to max_kp (row, col) pairs into rc[2*max_kp] in
 * response-descending order (ties: row-major index ascending) and their Harris responses into resp
 * (may be NULL).  *n = number written, *n_candidates (may be NULL) = corners before the top-K cut. */
int yv_detect(yv_ctx* ctx, const uint8_t* img, int H, int W, int stride, int max_kp, int32_t* rc,
              float* resp, int* n, int* n_candidates);
/* Brief::computeBrief (src/BriefDescriptor.cc:86-124; include/BriefDescriptor.hpp:61): blur, keep the
 * points inside checkBoundry (:128-136), emit KeyPoint records (id = input index).  out capacity n. */
int yv_describe(yv_ctx* ctx, const uint8_t* img, int H, int W, int stride, const int32_t* rc, int n,
                yv_keypoint* out, int* n_out);
/* Brief::matchFeatures (src/BriefDescriptor.cc:163-183; include/BriefDescriptor.hpp:62): for every
 * query the first train point at minimum Hamming distance.  out capacity nq. */
int yv_match_features(yv_ctx* ctx, const yv_keypoint* q, int nq, const yv_keypoint* t, int nt, yv_match* out);
/* Brief::removeOutliers (src/BriefDescriptor.cc:213-231; include/BriefDescriptor.hpp:64). */
int yv_filter_matches(yv_ctx* ctx, const yv_match* in, int n, int thr, yv_match* out, int* n_out);

/* ---- batched device pipeline (inputs resident in HBM) ---------------------------------------------- */
/* A batch owns device workspace for up to max_images images of H x W and max_pairs match pairs.  Slot
 * index max_images is the "carry" slot: it holds the keypoints / descriptors of one image of the
 * previous run (see yv_batch_run's carry_from), so consecutive runs chain frame k-1 -> k.  YV_ERR_CAPACITY for
 * W > 2048 (BRIEF stages 49 image rows in LDS) or H > 8192 (top-K's per-band keypoint lists). */
int yv_batch_create(yv_ctx* ctx, int max_images, int H, int W, int max_kp, int max_pairs,
                    yv_batch** out);
void yv_batch_destroy(yv_batch* b);
/* Match pairs (query image, train image) for subsequent runs; indices in [0, max_images] (max_images =
 * carry slot).  Copied to the device once. */
int yv_batch_set_pairs(yv_batch* b, const int32_t* pairs /* [2*n_pairs] */, int n_pairs);
/* Run detect -> describe -> match -> removeOutliers for n_images device images
 *   image i at d_images + i*image_pitch, rows `stride` bytes apart,
 * then copy image carry_from's keypoints into the carry slot (carry_from < 0: no copy).  Asynchronous
 * on `stream` (NULL = the context stream).  match_thr is removeOutliers' threshold (20 in
 * src/LoopHandler.cc:192,537). */
int yv_batch_run(yv_batch* b, const uint8_t* d_images, int n_images, int stride, int64_t image_pitch,
                 int match_thr, int carry_from, void* stream);
/* Tracking (PnP) over the last run's matches: track t = {stereo_pair, temporal_pair} (pair indices of
 * yv_batch_set_pairs) where the stereo pair's query image (frame k left) is the temporal pair's train
 * image.  Each frame-(k-1) keypoint kept by removeOutliers in the temporal pair whose frame-k keypoint is
 * itself kept in the stereo pair becomes one pose edge: X = LoopHandler::triangulation of the stereo match
 * (src/LoopHandler.cc:867-885, left camera = world, right camera pose T_right; accepted iff success and
 * Z > 0 as in triangulate2View :658-726), measurement = the frame-(k-1) keypoint (x, y).  The pose of
 * frame k-1 in frame k's camera is then LoopHandler::optimizePoseOnly (:730-861) from the prior.  K and
 * T_right are copied once; tracks are validated against the pairs (YV_ERR_INVALID otherwise). */
int yv_batch_set_tracks(yv_batch* b, const int32_t* tracks /* [2*n_tracks] */, int n_tracks, const double K[9],
                        const double T_right[7]);
/* Build the track edges and solve every track's pose in one launch each (asynchronous on `stream`, NULL =
 * context stream).  d_priors [n_tracks][7] in, d_poses [n_tracks][7] out (may alias d_priors). */
int yv_batch_track(yv_batch* b, const double* d_priors, double* d_poses, void* stream);
/* Overlap mode: the pose LM of each yv_batch_track runs on a stream of the batch, ordered after that call's
 * edge build only, so it executes beside the next yv_batch_run's kernels (edge buffers rotate over three
 * copies; the build of track i + 3 waits for the LM of track i).  With the match tracker the edge build itself
 * also runs on a stream of the batch, after the run's matches, beside the next run's detect; the next run's
 * top-K waits for it (environment YAVO_BUILD_ASYNC=0 keeps it on the call's stream).  d_priors / d_poses / the
 * track views are then complete only after yv_batch_track_sync (or a device-wide synchronization).  on = 2 / 3 / 4 defer each
 * LM further: it is launched by the next yv_batch_run once that run's detect (2) / describe (3) / top-K (4) stage is issued
 * (so it runs beside the later, less occupancy-sensitive stages), or by yv_batch_track_sync /
 * yv_batch_map_wait / the next yv_batch_track, whichever comes first. */
int yv_batch_set_track_overlap(yv_batch* b, int on);
int yv_batch_track_sync(yv_batch* b);
/* LK tracking mode, the reference's trackLastFrame (src/LoopHandler.cc:298-454): with image_step > 0 a track
 * is {stereo pair of frame k-1, image index of frame k}.  Frame k-1's map points are its left keypoints whose
 * stereo match survives removeOutliers and triangulates; they are tracked into frame k by
 * calcOpticalFlowPyrLK(win, max_level, TermCriteria(COUNT+EPS, max_count, eps), flags 0, min_eig) on the last
 * run's images 0, image_step, 2 image_step, ... (both images of a track must be among them), and every point
 * with status 1 becomes an edge at cv::Point2i(next.y, next.x) (truncation).  image_step = 0: match mode.
 * Clears the tracks (set them again).  Declared in yavo_geom.h: the LK workspace API it uses. */
int yv_batch_set_track_lk(yv_batch* b, int image_step, int win, int max_level, int max_count, double eps,
                          double min_eig);
/* Per-stage device time of the runs since the last reset, when timing is enabled (HIP events recorded
 * on the run stream around every stage).  Stages: 0 detect (FAST + Harris + blur, one fused kernel),
 * 1 top-K + checkBoundry, 2 BRIEF, 3 match, 4 Matches records + removeOutliers (+ carry copies),
 * 5 track edges (stereo triangulation), 6 track poses (LM).  ms[i] = summed milliseconds, *n_runs = runs
 * accumulated (stages 5-6 summed over the runs followed by yv_batch_track).  on = 2: events around the
 * detect kernel only (ms[0]; the other stages read 0) -- two events per run instead of nine. */
int yv_batch_enable_timing(yv_batch* b, int on);
int yv_batch_stage_times(yv_batch* b, float* ms /* [8] */, int* n_runs);
#define YV_NUM_STAGES 7

/* Device views of the batch results (valid until the next run / destroy).  All arrays are indexed
 * [slot][...] with the per-slot strides given. */
typedef struct yv_batch_view {
    int max_images, max_kp, max_pairs, H, W;
    int64_t cand_cap;                 /* candidate capacity per image = (H-8)*(W-8) */
    const uint32_t* cand_count;       /* [max_images+1]: FAST corners before the cut */
    const int32_t* det_count;         /* [max_images+1]: min(corners, max_kp) */
    const int32_t* det_rc;            /* [max_images+1][max_kp][2] (row, col), response order */
    const float* det_resp;            /* [max_images+1][max_kp] */
    const int32_t* kp_count;          /* [max_images+1]: keypoints that passed checkBoundry */
    const yv_keypoint* keypoints;     /* [max_images+1][max_kp] */
    const uint8_t* blurred;           /* [max_images][H][blur_pitch] (row pitch: the last field) */
    const int32_t* match_count;       /* [max_pairs]: = kp_count of the query image */
    const yv_match* matches;          /* [max_pairs][max_kp] */
    const int32_t* filt_count;        /* [max_pairs] */
    const yv_match* filtered;         /* [max_pairs][max_kp] */
    /* per-query {distance, train keypoint index (-1: empty train)} and the removeOutliers limit
     * (kept iff distance < limit) of every pair */
    const int32_t* match_dj;          /* [max_pairs][max_kp][2] */
    const int32_t* match_lim;         /* [max_pairs] */
    /* tracks (yv_batch_set_tracks / yv_batch_track): the buffers of the last yv_batch_track call */
    int n_tracks;
    const int32_t* edge_count;        /* [n_tracks] */
    const double* edge_X;             /* [n_tracks][max_kp][3] */
    const double* edge_uv;            /* [n_tracks][max_kp][2] */
    const int32_t* edge_query;        /* [n_tracks][max_kp]: temporal query keypoint index */
    const uint8_t* edge_outlier;      /* [n_tracks][max_kp] */
    const int32_t* track_inliers;     /* [n_tracks] */
    int blur_pitch;                   /* row pitch of `blurred` in bytes (128-B aligned, >= W + 1) */
} yv_batch_view;
int yv_batch_view_get(yv_batch* b, yv_batch_view* view);

#ifdef __cplusplus
}
#endif

#include "yavo_geom.h"

#endif /* YAVO_H */
