// yavo_internal.h -- launchers shared between the kernel translation unit and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/yavo/yavo_types.h"

struct yv_ctx;

namespace yavo {

// pow(t, 3) of g2o's LM step scaling (alpha = 1 - pow(2 rho - 1, 3)), correctly rounded: t^2 = p + e1 and p t = q + e2
// exactly (fma), t^3 = q + (e2 + e1 t) rounded once (oracle/yavo_oracle.h or_cube, the same operations).
__host__ __device__ inline double cube_cr(double t) {
    const double p = t * t, e1 = fma(t, t, -p);
    const double q = p * t, e2 = fma(p, t, -q);
    return q + (e2 + e1 * t);
}

constexpr int kMaxKp = 4096;
constexpr int kMaxWidth = 2048;  // image width limit (BRIEF keeps 49 rows of the blurred image in LDS)       // per-image keypoint capacity supported by the top-K / scan kernels
// BRIEF's row bands: 32 image rows per workgroup.  top-K buckets each image's kept keypoints by band
// (kp_band[image][max_kp] int4 {row, col, id, slot}, band b at [band_off[image][b], band_off[image][b + 1])), so a
// BRIEF workgroup reads its band's keypoints only; H <= kBandRows * kMaxBands.
constexpr int kBandRows = 32;
constexpr int kMaxBands = 256;
constexpr int kBandCounters = 1024;  // top-K's (band, bank class) counters: 32 classes up to 32 bands, else 1
constexpr int kFastTileW = 64;     // FAST / blur output tile: one wave per tile row
constexpr int kFastTileH = 56;
// The blurred image (detect's second output, BRIEF's input) is stored with a 128-B aligned row pitch, so the
// detect tiles write whole 64-B row segments with dword stores (a row stride of W = 1241 put every segment across
// two cache lines, stored byte by byte).  Columns [W, pitch) are padding no reader uses; pitch >= W + 1
// (brief_lds_stride(W) <= pitch: BRIEF stages whole 16-B words of a row).
__host__ __device__ constexpr int blur_pitch(int W) { return (W + 1 + 127) & ~127; }
// BRIEF's LDS band row stride: >= W + 1 (column W holds the next row's first pixel, see brief_kernel), 16-B rows
__host__ __device__ constexpr int brief_lds_stride(int W) { return (W + 1 + 15) & ~15; }
// Blurred images are laid out [image][H][blur_pitch(W)].
__host__ __device__ constexpr int64_t blur_image_bytes(int H, int W) { return (int64_t)H * blur_pitch(W); }
// XCD-aware block order (MI355X: 8 XCDs, each with its own L2; blocks are observed to round-robin over them by
// linear id): the bijective remap turns linear block b into a logical index so that every XCD runs one contiguous
// range of logical blocks -- neighbouring tiles (and their shared halo rows) stay in one L2.  Pure speed.
__device__ __forceinline__ int xcd_swizzle(int b, int nblocks) {
    const int q = nblocks >> 3, r = nblocks & 7, xcd = b & 7, slot = b >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

struct Desc {                      // 256-bit BRIEF descriptor, test j -> bit j (LSB-first bytes)
    uint32_t w[8];
};

// FAST-12 candidate test + Harris response, appends (response, index) keys per image.  eig: the cv::eigen
// flavour (0 = JacobiImpl_, 1 = HAVE_EIGEN's SelfAdjointEigenSolver).
void launch_fast_harris(const uint8_t* imgs, int n_images, int H, int W, int stride, int64_t pitch,
                        int thr, int eig, uint64_t* cand_keys, int64_t cap, uint32_t* cand_count,
                        hipStream_t s);
// Fused FAST + Harris + 9x9 blur over the same LDS tile (the image is read once).
void launch_detect_blur(const uint8_t* imgs, int n_images, int H, int W, int stride, int64_t pitch, int thr,
                        int eig, uint64_t* cand_keys, int64_t cap, uint32_t* cand_count, const uint16_t* k9_host,
                        uint8_t* blur, hipStream_t s);
// 9-tap separable fixed-point Gaussian, BORDER_REFLECT_101; output [image][H][blur_pitch(W)].
void launch_blur9(const uint8_t* imgs, int n_images, int H, int W, int stride, int64_t pitch,
                  const uint16_t* k9_host, uint8_t* blur, hipStream_t s);
// Per-image top-K (response desc, index asc) + checkBoundry compaction.
// cand_count is copied to cand_seen and reset to 0 after it is read (ready for the next detection).
void launch_topk(const uint64_t* cand_keys, int64_t cap, uint32_t* cand_count, uint32_t* cand_seen, int n_images,
                 int H, int W, int max_kp, int keep, int32_t* det_rc, float* det_resp, int32_t* det_count,
                 int32_t* kp_src, int32_t* kp_count, int32_t* kp_band, int32_t* band_off, hipStream_t s);
// checkBoundry compaction of externally supplied points (det_rc / det_count already on the device).
void launch_kp_boundary(const int32_t* det_rc, const int32_t* det_count, int n_images, int H, int W,
                        int max_kp, int32_t* kp_src, int32_t* kp_count, int32_t* kp_band, int32_t* band_off,
                        hipStream_t s);
// BRIEF: writes KeyPoint records + packed descriptors.  loff: a 2 KB device scratch of the caller holding the tests'
// LDS offsets for this W, formed on stream s first when new_loff (the offsets table or W changed since it was formed).
void launch_brief(const uint8_t* blur, int n_images, int H, int W, const int8_t* offsets,
                  const int32_t* kp_src, const int32_t* kp_band, const int32_t* band_off, int max_kp,
                  yv_keypoint* keypoints, Desc* desc, int32_t* loff, bool new_loff, hipStream_t s);
// Pack KeyPoint records -> descriptors (host-supplied keypoints).
void launch_pack_desc(const yv_keypoint* keypoints, const int32_t* kp_count, int n_slots, int max_kp,
                      Desc* desc, hipStream_t s);
// Brute-force Hamming NN: match_key[pair][q] = min over t of (dist << 16 | t).  max_train bounds every train
// list's length (<= 2048: the FP4 matcher, otherwise the int8 +-1 form); max_kp is the slot stride.
void launch_match(const Desc* desc, const int32_t* kp_count, const int32_t* pairs, int n_pairs,
                  int max_kp, int max_train, uint32_t* match_key, hipStream_t s);
// Matches records (matchFeatures) + removeOutliers per pair.  match_key entries are reset to
// 0xFFFFFFFF after they are read (ready for the next match).
void launch_match_finalize(uint32_t* match_key, const yv_keypoint* keypoints,
                           const int32_t* kp_count, const int32_t* pairs, int n_pairs, int max_kp,
                           int thr, yv_match* matches, int32_t* match_count, yv_match* filtered,
                           int32_t* filt_count, int2* match_dj, int32_t* match_lim, hipStream_t s,
                           int32_t* kp_count_copy = nullptr, int n_slots = 0);  // + kp_count[0, n_slots) -> copy
// removeOutliers on externally supplied Matches records (one list).
void launch_filter_records(const yv_match* in, int n, int thr, yv_match* out, int32_t* out_count,
                           hipStream_t s);

// ---- geometry (yavo_geom.hip) ----
// device workspace of launch_f_ransac: [n_lists][iters] hypotheses' F and inlier counts
size_t f_ransac_ws_bytes(int n_lists, int iters);
void launch_f_ransac(const yv_match* matches, int64_t list_stride, const int32_t* counts, int n_lists,
                     const int32_t* samples, int64_t sample_stride, int iters, double thr, double* F_out,
                     int32_t* max_inliers, int32_t* found, void* ws, hipStream_t s);
void launch_triangulate(const yv_match* m, int n, const double* poses2, const double* K, double* Xw, uint8_t* ok,
                        int32_t* n_ok, hipStream_t s);
void launch_world2camera(const double* X, int n, const double* T, const double* K, double* out, hipStream_t s);
void launch_pose_lm(const int32_t* offsets, int n_problems, const double* X, const double* uv, const double* K,
                    double* poses, uint8_t* outlier, int32_t* inliers, hipStream_t s);
void launch_pose_gn(const int32_t* offsets, int n_problems, const double* X, const double* uv, const double* K,
                    double* poses, int32_t* iters, hipStream_t s);
// cv::calcOpticalFlowPyrLK workspace view (yavo_lk.hip).  Level 0 is the caller's image; levels >= 1 live in
// `pyr` ([image][pyr_pitch], level l at off[l], row stride ps[l] = w[l] rounded up to 64 bytes: every pyrDown store
// is a whole aligned dword of full cache lines).  The tracker computes Scharr derivatives inside its windows; `der`
// is one level's (dx, dy) int16 image for yv_lk_level only (ds[l] pixels per row = w[l] rounded up to 16).
constexpr int kLkMaxLevels = 8;
struct LkParams {
    int levels = 0, win = 11, max_count = 30;
    double eps2 = 1e-4, min_eig = 1e-3;
    int h[kLkMaxLevels] = {}, w[kLkMaxLevels] = {};
    int ps[kLkMaxLevels] = {}, ds[kLkMaxLevels] = {};
    int64_t off[kLkMaxLevels] = {};
    const uint8_t* img0 = nullptr;
    int stride0 = 0;
    int64_t pitch0 = 0;
    uint8_t* pyr = nullptr;
    int64_t pyr_pitch = 0;
    int16_t* der = nullptr;
    int64_t der_pitch = 0;  // int16 elements of `der`
};
void launch_lk_pyramid(const LkParams& P, int n_images, hipStream_t s);
void launch_lk_derivs(const LkParams& P, int image, int level, int16_t* der, hipStream_t s);
void launch_lk_track(const LkParams& P, const int32_t* pairs, int n_pairs, const float* pts, const int32_t* counts,
                     int pts_stride, int max_pts, float* next_pts, uint8_t* status, float* err, hipStream_t s);
void launch_track_build(const int32_t* tracks, int n_tracks, const int32_t* pairs, const yv_keypoint* keypoints,
                        const int32_t* kp_count, const int2* match_dj, const int32_t* match_lim, int max_kp,
                        const double* K, const double* T_right, double* edge_X, double* edge_uv, int32_t* edge_query,
                        int32_t* edge_count, hipStream_t s);
void launch_stereo_points(const int32_t* stereo_pairs, int n_tracks, const int32_t* pairs,
                          const yv_keypoint* keypoints, const int32_t* kp_count, const int2* match_dj,
                          const int32_t* match_lim, int max_kp, const double* K, const double* T_right, double* pX,
                          float* pts, int32_t* pq, int32_t* pcount, hipStream_t s);
void launch_lk_edges(int n_tracks, const double* pX, const float* next, const uint8_t* status, const int32_t* pq,
                     const int32_t* pcount, int max_kp, double* edge_X, double* edge_uv, int32_t* edge_query,
                     int32_t* edge_count, hipStream_t s);

// cv::findEssentialMat (RANSAC) + cv::recoverPose (yavo_essential.hip).  Workspace of a yv_essential.
// RANSAC iterations evaluated per round: 64, or 1024 (>= findEssentialMat's 1000) for workspaces of at most kEssWidePairs
// lists, where the chip is otherwise idle: a list that needs all its iterations (the LoopHandler's re-initialisation
// lists, one image translation apart, never reach the 0.999 confidence early) then takes one round instead of four
// dependent ones, and a list that converges early costs the same one round (the sequential selection ignores the
// iterations past niters, so the result is the same)
constexpr int kEssChunk = 64;
constexpr int kEssChunkWide = 1024;
constexpr int kEssWidePairs = 8;
inline int ess_chunk_for(int max_pairs) { return max_pairs <= kEssWidePairs ? kEssChunkWide : kEssChunk; }
struct EssParams {
    int max_pairs = 0, max_points = 0, max_iters = 0;
    int chunk = kEssChunk;     // iterations per round (ess_chunk_for)
    double* m1 = nullptr;      // [max_pairs][max_points][2] normalised points1
    double* m2 = nullptr;      // [max_pairs][max_points][2] normalised points2
    int32_t* idx = nullptr;    // [max_pairs][max_iters][5] getSubset draws
    double* models = nullptr;  // [max_pairs][chunk][10][9]
    int32_t* nmod = nullptr;   // [max_pairs][chunk]
    int32_t* good = nullptr;   // [max_pairs][chunk][10]
    int32_t* state = nullptr;  // [max_pairs][8]: niters, max_good, iterations run, models, found, n, -, -
    double* best = nullptr;    // [max_pairs][9]
    double* cand = nullptr;    // [max_pairs][4][12] recoverPose candidates P1..P4
    int32_t* cgood = nullptr;  // [max_pairs][4]
    // cv::RNG((uint64)-1)'s states after 1 .. rng_len draws (list-independent: every list's round 0 starts there), for
    // the parallel subset draws of wide rounds (ess_subsets_par_kernel); null for narrow rounds
    uint64_t* rng_tab = nullptr;
    int rng_len = 0;
};
struct EssRun {
    double focal, ppx, ppy, prob, threshold;
    int max_iters;
};
void launch_find_essential(const EssParams& P, const EssRun& r, const float* pts1, const float* pts2,
                           const int32_t* counts, int n_pairs, int pts_stride, double* E, uint8_t* mask,
                           int32_t* found, int32_t* stats, hipStream_t s);
struct Mat3 {
    double v[9];
};
// the context's device / stream for the host-side modules (yavo_io.hip); defined in yavo_api.hip
int ctx_device(struct ::yv_ctx* ctx);
hipStream_t ctx_stream(struct ::yv_ctx* ctx);
void launch_recover_pose(const EssParams& P, const double* E, const float* pts1, const float* pts2,
                         const int32_t* counts, int n_pairs, int pts_stride, const Mat3& K, double* R, double* t,
                         int32_t* good, hipStream_t s);
// sliding-window BA (yavo_ba.hip): the device graph, workspace and estimate of a yv_ba
struct BaParams {
    int P = 0, nf = 0, np = 0, ns = 0, L = 0, E = 0;
    const int32_t* ep = nullptr;      // [E]
    const int32_t* el = nullptr;      // [E]
    const double* meas = nullptr;     // [E][2]
    const int32_t* pe_off = nullptr;  // [P + 1] edges per pose (edge order)
    const int32_t* pe = nullptr;      // [E]
    const int32_t* le_off = nullptr;  // [L + 1] edges per landmark (edge order)
    const int32_t* le = nullptr;      // [E]
    const int32_t* cv_off = nullptr;  // [P * P + 1] per pose pair (p1 <= p2): shared landmarks ascending
    const int32_t* cv_e1 = nullptr;   // the p1 edge of each
    const int32_t* cv_e2 = nullptr;   // the p2 edge of each
    double* poses = nullptr;          // [P][7]
    double* X = nullptr;              // [L][3]
    double* err = nullptr;            // [E][2]
    double* Jp = nullptr;             // [E][12]
    double* Jl = nullptr;             // [E][6]
    double* Hpp = nullptr;            // [P][36]
    double* bp = nullptr;             // [P][6]
    double* Hll = nullptr;            // [L][9]
    double* bl = nullptr;             // [L][3]
    double* S = nullptr;              // [ns][ns]
    double* bs = nullptr;             // [ns]
    double* xp = nullptr;             // [ns]
    double* xl = nullptr;             // [L][3]
    int32_t* tr = nullptr;            // [ns] LDLT transpositions
    double* scal = nullptr;           // [4]: chi2, scale, LDLT ok
    // device-driven LM (yv_ba_solve): a kernel returns at once when *gate != 0 (its phase is skipped), and the trial
    // kernels read lambda from *lam; both nullptr under host control
    const int* gate = nullptr;
    const double* lam = nullptr;
    // the trial state: ba_step_kernel writes the trial estimate into the other buffer (poses2 / X2 when *cur == 0),
    // an accepted trial flips *cur; ba_finish_kernel leaves the result in poses / X
    double* poses2 = nullptr;          // [P][7]
    double* X2 = nullptr;              // [L][3]
    int* cur = nullptr;
    struct BaCtl* ctl = nullptr;        // device control block (nullptr: host control)
    double* log = nullptr;             // [max_iters + 1] chi2 per iteration (device control)
    unsigned long long* maxdiag = nullptr;
    unsigned* ticket = nullptr;        // [kBaTickets] last-workgroup counters (0 between launches)
    double* part = nullptr;            // [1 + 2 blocks]: the free poses' scale part, then per block of 256
                                       // landmarks its chi2 and scale totals (ba_step_kernel)
    double* spart = nullptr;           // [Schur task][kWG][36] tree4096 class totals of the Schur workgroups
    unsigned* sticket = nullptr;       // [Schur task] last-workgroup counters (0 between launches)
    double* rpart = nullptr;           // [free pose][kWG][27] class totals of the H_pp / b_p reduce
    unsigned* rticket = nullptr;       // [free pose] last-workgroup counters
};
// The device-side Levenberg-Marquardt control of one solve (g2o OptimizationAlgorithmLevenberg::solve, the
// host loop's arithmetic): written by the last workgroups of ba_reduce_kernel / ba_chi2_kernel, read by the gates.
struct BaCtl {
    double currentChi, lambda, ni, rho;
    int q, it, stop, iters;
    int skip_iter, skip_trial, suspended, iter_done;
};
struct BaMat3 {
    double v[9];
};
// linearise + the H / b blocks (first: the largest diagonal into *P.maxdiag; device control: the iteration begins)
void launch_ba_linearize(const BaParams& P, const BaMat3& K, int first, hipStream_t s);
// one damping trial: Dinv / W, Schur, LDLT, step into the trial state, chi2 + scale (device control: the decision)
void launch_ba_trial(const BaParams& P, const BaMat3& K, double lambda, hipStream_t s);
// the solve's first chi2 (device control: the control block's initialisation)
void launch_ba_chi2(const BaParams& P, const BaMat3& K, hipStream_t s);
void launch_ba_finish(const BaParams& P, hipStream_t s);
void launch_ba_ctl_resume(BaCtl* c, hipStream_t s);

// the shared map (yavo_map.hip): one chunk's block after its pose LM
void launch_map_chunk(const double* rel, int n, int64_t first_frame, int kf_every, const int32_t* edge_count,
                      const double* edge_X, const uint8_t* edge_outlier, int max_kp, int max_kf, void* block,
                      hipStream_t s);

// PNG decoding on the GPU (yavo_inflate.hip): per-image status codes and the two kernels
enum : int32_t {
    kPngOk = 0, kPngErrHeader = 1, kPngErrBlock = 2, kPngErrCode = 3, kPngErrOverrun = 4, kPngErrShort = 5,
    kPngErrFilter = 6, kPngErrCrc = 7, kPngErrAdler = 8,
    kPngErrFile = 9  // missing, unreadable, truncated or not an 8-bit grey PNG of the decoder's size (host side)
};
// one IDAT payload of a PNG file staged on the device: len bytes from src to dst (byte offsets in the staging buffers);
// the chunk's type is the 4 bytes before src, its CRC the 4 after src + len; img = the payload's image in the call
struct PngPiece {
    int64_t src, dst;
    int32_t len, img;
};
// gather + chunk CRCs: crc_bad[img] = 1 when a payload's CRC-32 (type + data) differs from the stored one
void launch_png_gather(const uint8_t* src, uint8_t* dst, const PngPiece* pieces, int n, int32_t* crc_bad, hipStream_t s);
// inflate: reads and clears crc_bad; adler[i] = the zlib trailer of image i
void launch_png_inflate(const uint8_t* src, const int64_t* off, const int32_t* len, int n, uint8_t* out,
                        int64_t out_pitch, uint32_t out_len, int32_t* status, int32_t* crc_bad, uint32_t* adler,
                        hipStream_t s);
// unfilter + the Adler-32 of the inflated bytes against adler[i]; failed images are zero-filled and counted in
// *bad_total
void launch_png_unfilter(const uint8_t* raw, int64_t raw_pitch, int n, int H, int W, uint8_t* dst, int64_t dst_pitch,
                         int dst_stride, int32_t* status, const uint32_t* adler, uint32_t* bad_total, hipStream_t s);

void launch_track_pose(int n_tracks, const int32_t* edge_count, int stride, const double* edge_X,
                       const double* edge_uv, const double* K, const double* priors, double* poses,
                       uint8_t* edge_outlier, int32_t* inliers, hipStream_t s);

}  // namespace yavo
