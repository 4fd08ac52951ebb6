// yavo_api.hip -- the C ABI of libyavo.so (include/yavo/yavo.h): contexts, batches, the host-pointer
// drop-in entry points and the batched device pipeline.  Host code only; kernels live in
// yavo_kernels.hip.  No CPU fallback exists: every compute path runs the gfx950 kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/yavo/yavo.h"
#include "../../include/yavo/yavo_map.h"
#include "yavo_internal.h"

using yavo::Desc;

struct yv_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int fast_thr = 40;         // include/FastDetector.hpp:35
    int harris_eigen = 0;      // cv::eigen flavour of the Harris response (yv_set_harris_eigen)
    int max_corners = 2000;    // include/FastDetector.hpp:36
    uint16_t k9[9] = {12, 22, 31, 41, 44, 41, 31, 22, 12};  // cv::GaussianBlur 9x9, sigma 2.5, 8U
    int8_t* d_offsets = nullptr;                              // [256*4]
    int offsets_version = 0;                                  // bumped by yv_set_brief_offsets
    yv_batch* single = nullptr;                               // workspace of the host-pointer API
    int32_t* h_pinned = nullptr;                              // small pinned scratch for counts
    void* scratch = nullptr;                                  // device arena of the geometry host calls
    size_t scratch_cap = 0;
    uint8_t* scratch_h = nullptr;                             // its pinned host mirror (same offsets)
    uint8_t* scratch_hd = nullptr;                            // the mirror's address for kernels (zero-copy regions)
    void* fr_ws = nullptr;                                    // yv_f_ransac_batch's hypothesis workspace
    size_t fr_ws_cap = 0;
    // yv_calc_optical_flow_pyr_lk's pyramid workspace, kept between calls (creating and destroying it per call
    // costs two hipMalloc / hipFree pairs and a device-wide synchronisation per tracked frame)
    yv_lk* lk_cache = nullptr;
    // its two image slots (device, with a pinned host copy of what each holds): a call whose prev image is the previous
    // call's next image (the tracking loop's consecutive frames) finds it and its pyramid already there
    uint8_t* lk_img_d = nullptr;
    uint8_t* lk_img_h = nullptr;
    int lk_last = -1;  // the slot holding the previous call's next image (-1: none)
    // the host findEssentialMat / recoverPose calls' workspace (yv_essential_create is ~10 hipMallocs, its destroy a
    // device synchronisation: per call they cost more than the solve), grown on demand
    yv_essential* ess_cache = nullptr;
    int lk_key[4] = {0, 0, 0, 0};  // H, W, win, max_level
    // Pinned staging of the host-pointer entry points.  The caller's buffers are pageable: a hipMemcpyAsync from or to
    // pageable memory is synchronous and goes through the runtime's own staging (~250 us per call, even for a
    // 4-byte count, and serialised across threads).  Uploads are copied into this buffer and DMA'd from it;
    // downloads land in it and are copied out after the call's stream synchronisation (stage_sync).
    uint8_t* h_stage = nullptr;
    size_t h_stage_cap = 0, h_stage_off = 0;
    struct PendingD2H {
        void* dst;
        const void* src;
        size_t bytes;
    };
    std::vector<PendingD2H> pending;
    hipStream_t side = nullptr;  // yv_side_stream: a stream on a hardware queue of its own, made on first use
};

namespace yavo {
int ctx_device(yv_ctx* ctx) { return ctx->device; }
hipStream_t ctx_stream(yv_ctx* ctx) { return ctx->stream; }
}  // namespace yavo

// Track edge buffers in flight: the build of track i + kEdgeBufs waits for the pose LM of track i (side stream), so
// an LM deferred into the next run (overlap modes 2-4) does not hold up the next build.
constexpr int kEdgeBufs = 3;

struct yv_batch {
    yv_ctx* ctx = nullptr;
    int max_images = 0, H = 0, W = 0, max_kp = 0, max_pairs = 0, n_pairs = 0;
    int64_t cap = 0;
    int nslots = 0;
    uint64_t* cand_keys = nullptr;
    uint32_t* cand_count = nullptr;
    uint32_t* cand_seen = nullptr;
    int32_t* det_rc = nullptr;
    float* det_resp = nullptr;
    int32_t* det_count = nullptr;
    int32_t* kp_src = nullptr;
    int32_t* kp_count = nullptr;
    int32_t* kp_count_build = nullptr;  // the asynchronous edge build's copy of the run's counts (top-K rewrites them)
    int32_t* kp_band = nullptr;     // [slot][max_kp] int4 {row, col, id, slot}: the kept keypoints by BRIEF band
    int32_t* band_off = nullptr;    // [slot][kMaxBands + 1]
    int32_t* brief_loff = nullptr;  // [256][2] BRIEF test offsets in the band's LDS layout (launch_brief)
    int loff_version = -1;          // the ctx offsets_version brief_loff was formed from (-1: never)
    bool counts_copied = false;     // this run's finalize wrote kp_count_build (the asynchronous build's copy)
    yv_keypoint* keypoints = nullptr;
    Desc* desc = nullptr;
    uint8_t* blur = nullptr;
    int32_t* pairs = nullptr;
    uint32_t* match_key = nullptr;
    yv_match* matches = nullptr;
    int32_t* match_count = nullptr;
    yv_match* filtered = nullptr;
    int32_t* filt_count = nullptr;
    int2* match_dj = nullptr;       // [max_pairs][max_kp] {distance, train index}
    int32_t* match_lim = nullptr;   // [max_pairs] removeOutliers limit
    uint8_t* staging = nullptr;  // one H x W input image (host-pointer API)
    std::vector<int32_t> h_pairs;   // host copy of the pairs (track validation)
    // tracks (PnP over the matches)
    int n_tracks = 0, max_tracks = 0;
    int32_t* tracks = nullptr;      // [max_tracks][2] {stereo pair, temporal pair}
    double* track_K = nullptr;      // [max_tracks][9]
    double* T_right = nullptr;      // [7]
    // edge / LM buffers, double-buffered ([2][...]): with the LM on the side stream, track i's LM reads
    // buffer i % 2 while track i + 1 builds into the other one
    double* edge_X = nullptr;       // [2][max_tracks][max_kp][3]
    double* edge_uv = nullptr;      // [2][max_tracks][max_kp][2]
    int32_t* edge_query = nullptr;  // [2][max_tracks][max_kp]
    int32_t* edge_count = nullptr;  // [2][max_tracks]
    uint8_t* edge_outlier = nullptr;
    int32_t* track_inliers = nullptr;
    // LK tracking mode (yv_batch_set_track_lk): tracks are {stereo pair of frame k-1, image index of frame k}
    int lk_step = 0;                // > 0: LK mode, LK images are the run's images 0, lk_step, 2 lk_step, ...
    yv_lk* lk = nullptr;
    int lk_max_count = 30;
    double lk_eps = 0.01, lk_min_eig = 1e-3;
    int32_t* lk_sp = nullptr;       // [max_tracks] stereo pair per track
    int32_t* lk_pairs = nullptr;    // [max_tracks][2] LK slots (prev, next)
    double* lk_X = nullptr;         // [max_tracks][max_kp][3]
    float* lk_pts = nullptr;        // [max_tracks][max_kp][2]
    float* lk_next = nullptr;
    float* lk_err = nullptr;
    uint8_t* lk_status = nullptr;
    int32_t* lk_q = nullptr;
    int32_t* lk_count = nullptr;
    // lk_X / lk_pts / lk_q / lk_count come in two sets: with the asynchronous build (overlap mode) the LK stage of
    // track i reads set i & 1 on bstream while track i + 1's stereo points fill the other one on the run's stream
    int lk_set = 0;
    hipEvent_t ev_lk[2] = {};
    bool lk_ev_pending[2] = {false, false};
    const uint8_t* run_images = nullptr;  // the last yv_batch_run's images (LK reads them)
    int run_n = 0, run_stride = 0;
    int64_t run_pitch = 0;
    int tbuf = 0;                   // buffer of the last yv_batch_track
    int track_calls = 0;
    bool overlap = false;           // LM on the side stream
    int overlap_mode = 0;           // 1: LM after the edge build; 2 / 3 / 4: after the next run's detect / describe / top-K
    struct DeferredLM {              // overlap modes 2 / 3: an LM launch waiting for the next yv_batch_run
        bool active = false;
        int k = 0, run = -1;
        const double* priors = nullptr;
        double* poses = nullptr;
        hipEvent_t* ev = nullptr;   // stage timing events of the run the track belongs to
        bool has_map = false;
        int64_t first_frame = 0;
        int kf_every = 1, max_kf = 1;
        void* block = nullptr;
    } deferred;
    hipEvent_t ev_defer = nullptr;
    hipStream_t side = nullptr;
    // edge build beside the next run (YAVO_BUILD_ASYNC, default on with the overlap, match tracker only): the
    // build runs on `bstream` after the run's finalize (ev_fin); the next run's top-K, which rewrites the keypoint
    // counts the build reads, waits for ev_built
    hipStream_t bstream = nullptr;
    bool build_async = false, build_pending = false;
    hipEvent_t ev_fin = nullptr, ev_built = nullptr;
    hipEvent_t ev_edges[kEdgeBufs] = {}, ev_lm[kEdgeBufs] = {};
    bool lm_pending[kEdgeBufs] = {};
    hipEvent_t ev_map = nullptr;    // after the last yv_batch_track_map's block (yv_batch_map_wait)
    bool map_written = false;
    hipEvent_t ev_map_release = nullptr;  // the block's readers (yv_batch_map_release): the next block write waits
    bool map_release_pending = false;
    // stage timing: events 0..5 bracket the run's stages, 6..8 the track's
    int timing = 0;  // 0 off, 1 every stage, 2 detect only
    std::vector<hipEvent_t> events;  // kEvPerRun per recorded run
    std::vector<uint8_t> tracked;    // run r was followed by a timed yv_batch_track
    int runs_recorded = 0;
    int last_run = -1;
    int pending_carry = -1;  // image whose keypoints enter the carry slot at the start of the next run
};

namespace {

constexpr int kEvPerRun = 9;
constexpr int kMaxTimedRuns = 4096;

#define YV_HIP(call)                                                                           \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "yavo: %s failed: %s (%s:%d)\n", #call, hipGetErrorString(e_), \
                         __FILE__, __LINE__);                                                  \
            return YV_ERR_HIP;                                                                 \
        }                                                                                      \
    } while (0)

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::fprintf(stderr, "yavo: kernel launch failed: %s\n", hipGetErrorString(e));
        return YV_ERR_HIP;
    }
    return YV_OK;
}

// the next writer of what an asynchronous edge build reads (keypoint counts, keypoints, match lists, pairs,
// tracks) is ordered after it on stream s
int join_build(yv_batch* b, hipStream_t s) {
    if (!b->build_pending) return YV_OK;
    YV_HIP(hipStreamWaitEvent(s, b->ev_built, 0));
    b->build_pending = false;
    return YV_OK;
}

bool finite_pose(const double* p) {
    for (int i = 0; i < 7; ++i)
        if (!(p[i] == p[i])) return false;
    return true;
}

template <class T>
int dalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
    if (e != hipSuccess) {
        std::fprintf(stderr, "yavo: hipMalloc(%zu B) failed: %s\n", count * sizeof(T), hipGetErrorString(e));
        return YV_ERR_HIP;
    }
    return YV_OK;
}

void batch_free(yv_batch* b) {
    if (!b) return;
    void* ptrs[] = {b->cand_keys, b->cand_count, b->cand_seen, b->det_rc,   b->det_resp,    b->det_count, b->kp_src, b->kp_band, b->band_off,
                    b->brief_loff, b->kp_count,  b->kp_count_build, b->keypoints,  b->desc, b->blur,   b->pairs,     b->match_key,
                    b->matches,   b->match_count, b->filtered, b->filt_count, b->staging,  b->match_dj,
                    b->match_lim, b->tracks,     b->track_K,  b->T_right,    b->edge_X,    b->edge_uv,
                    b->edge_query, b->edge_count, b->edge_outlier, b->track_inliers};
    if (b->bstream) (void)hipStreamSynchronize(b->bstream);
    if (b->side) (void)hipStreamSynchronize(b->side);
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    void* lk_ptrs[] = {b->lk_sp, b->lk_pairs, b->lk_X, b->lk_pts, b->lk_next, b->lk_err, b->lk_status, b->lk_q,
                       b->lk_count};
    for (void* p : lk_ptrs)
        if (p) (void)hipFree(p);
    if (b->lk) yv_lk_destroy(b->lk);
    for (hipEvent_t e : b->events) (void)hipEventDestroy(e);
    for (int k = 0; k < kEdgeBufs; ++k) {
        if (b->ev_edges[k]) (void)hipEventDestroy(b->ev_edges[k]);
        if (b->ev_lm[k]) (void)hipEventDestroy(b->ev_lm[k]);
    }
    if (b->ev_map) (void)hipEventDestroy(b->ev_map);
    if (b->ev_defer) (void)hipEventDestroy(b->ev_defer);
    if (b->ev_map_release) (void)hipEventDestroy(b->ev_map_release);
    if (b->ev_fin) (void)hipEventDestroy(b->ev_fin);
    if (b->ev_built) (void)hipEventDestroy(b->ev_built);
    for (hipEvent_t e : b->ev_lk)
        if (e) (void)hipEventDestroy(e);
    if (b->bstream) (void)hipStreamDestroy(b->bstream);
    if (b->side) (void)hipStreamDestroy(b->side);
    delete b;
}

int set_device(yv_ctx* ctx) {
    YV_HIP(hipSetDevice(ctx->device));
    return YV_OK;
}

// ---- pinned staging of the host-pointer entry points (yv_ctx::h_stage) ----
bool in_pinned_scratch(const yv_ctx* ctx, const void* p) {
    const char* c = static_cast<const char*>(p);
    const char* b = reinterpret_cast<const char*>(ctx->h_pinned);
    return ctx->h_pinned && c >= b && c < b + 64 * sizeof(int32_t);
}

// the downloads of the call land in the caller's buffers once the stream has drained
hipError_t stage_sync(yv_ctx* ctx, hipStream_t s) {
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        ctx->pending.clear();
        return e;
    }
    for (const auto& d : ctx->pending) std::memcpy(d.dst, d.src, d.bytes);
    ctx->pending.clear();
    ctx->h_stage_off = 0;
    return hipSuccess;
}

// `bytes` of the staging buffer for this call (64-B aligned); grows it after draining the stream when full
uint8_t* stage_alloc(yv_ctx* ctx, size_t bytes, hipStream_t s) {
    const size_t need = (bytes + 63) & ~(size_t)63;
    if (ctx->h_stage_off + need > ctx->h_stage_cap) {
        if (ctx->h_stage_off > 0 && stage_sync(ctx, s) != hipSuccess) return nullptr;
        if (need > ctx->h_stage_cap) {
            if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
            ctx->h_stage = nullptr;
            ctx->h_stage_cap = 0;
            const size_t cap = std::max(need, (size_t)4 << 20);
            if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_stage), cap) != hipSuccess) {
                ctx->h_stage = nullptr;
                return nullptr;
            }
            ctx->h_stage_cap = cap;
        }
    }
    uint8_t* p = ctx->h_stage + ctx->h_stage_off;
    ctx->h_stage_off += need;
    return p;
}

hipError_t stage_h2d(yv_ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (in_pinned_scratch(ctx, src)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
    uint8_t* p = stage_alloc(ctx, bytes, s);
    if (!p) return hipErrorOutOfMemory;
    std::memcpy(p, src, bytes);
    return hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, s);
}

// a pitched host image (rows of `width` bytes, `spitch` apart) into a pitched device image
hipError_t stage_h2d_2d(yv_ctx* ctx, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                        size_t height, hipStream_t s) {
    if (width == 0 || height == 0) return hipSuccess;
    uint8_t* p = stage_alloc(ctx, width * height, s);
    if (!p) return hipErrorOutOfMemory;
    const uint8_t* q = static_cast<const uint8_t*>(src);
    if (spitch == width) std::memcpy(p, q, width * height);
    else
        for (size_t r = 0; r < height; ++r) std::memcpy(p + r * width, q + r * spitch, width);
    // a packed destination takes one linear DMA: hipMemcpy2DAsync moves a 376-row image as row-sized transfers at
    // ~0.2 GB/s (2.6 ms per KITTI frame in the r03 LoopHandler trace)
    if (dpitch == width) return hipMemcpyAsync(dst, p, width * height, hipMemcpyHostToDevice, s);
    return hipMemcpy2DAsync(dst, dpitch, p, width, width, height, hipMemcpyHostToDevice, s);
}

hipError_t stage_d2h(yv_ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (in_pinned_scratch(ctx, dst)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
    uint8_t* p = stage_alloc(ctx, bytes, s);
    if (!p) return hipErrorOutOfMemory;
    ctx->pending.push_back({dst, p, bytes});
    return hipMemcpyAsync(p, src, bytes, hipMemcpyDeviceToHost, s);
}

// Drops the downloads of a call that returns before its stage_sync (an error path): they must not be copied into
// buffers the caller no longer expects to be written.  The staging offset is kept, so nothing still in flight is
// overwritten before the next stage_sync.
struct StageScope {
    yv_ctx* ctx;
    explicit StageScope(yv_ctx* c) : ctx(c) {}
    ~StageScope() { ctx->pending.clear(); }
};

// The host-pointer entry points share one single-image workspace per context.
int ensure_single(yv_ctx* ctx, int H, int W) {
    if (ctx->single && ctx->single->H == H && ctx->single->W == W) return YV_OK;
    if (ctx->single) {
        batch_free(ctx->single);
        ctx->single = nullptr;
    }
    yv_batch* b = nullptr;
    int rc = yv_batch_create(ctx, 1, H, W, yavo::kMaxKp, 1, &b);
    if (rc != YV_OK) return rc;
    const int32_t pair[2] = {0, 1};  // query = slot 0, train = slot 1 (the carry slot)
    rc = yv_batch_set_pairs(b, pair, 1);
    if (rc != YV_OK) {
        batch_free(b);
        return rc;
    }
    ctx->single = b;
    return YV_OK;
}

int record_stage(yv_batch* b, hipStream_t s, int run, int stage) {
    if (!b->timing || run < 0) return YV_OK;
    if (b->timing == 2 && stage > 1) return YV_OK;  // detect-only: the two events around the detect kernel
    YV_HIP(hipEventRecord(b->events[(size_t)run * kEvPerRun + stage], s));
    return YV_OK;
}

}  // namespace

extern "C" {

int yv_abi_version(void) { return YV_ABI_VERSION; }

const char* yv_status_string(int status) {
    switch (status) {
        case YV_OK: return "ok";
        case YV_ERR_INVALID: return "invalid argument";
        case YV_ERR_HIP: return "HIP runtime error";
        case YV_ERR_NODEVICE: return "no usable GPU";
        case YV_ERR_CAPACITY: return "capacity exceeded";
        default: return "unknown status";
    }
}

int yv_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int yv_create(int device, yv_ctx** out) {
    if (!out) return YV_ERR_INVALID;
    *out = nullptr;
    int n = yv_device_count();
    if (n <= 0) return YV_ERR_NODEVICE;
    if (device < 0 || device >= n) return YV_ERR_INVALID;
    yv_ctx* ctx = new (std::nothrow) yv_ctx();
    if (!ctx) return YV_ERR_INVALID;
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return YV_ERR_HIP;
    }
    if (dalloc(&ctx->d_offsets, 1024) != YV_OK || hipMemset(ctx->d_offsets, 0, 1024) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&ctx->h_pinned), 64 * sizeof(int32_t)) != hipSuccess) {
        yv_destroy(ctx);
        return YV_ERR_HIP;
    }
    *out = ctx;
    return YV_OK;
}

void yv_destroy(yv_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->lk_cache) yv_lk_destroy(ctx->lk_cache);
    if (ctx->lk_img_d) (void)hipFree(ctx->lk_img_d);
    if (ctx->lk_img_h) (void)hipHostFree(ctx->lk_img_h);
    if (ctx->ess_cache) yv_essential_destroy(ctx->ess_cache);
    batch_free(ctx->single);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->scratch_h) (void)hipHostFree(ctx->scratch_h);
    if (ctx->fr_ws) (void)hipFree(ctx->fr_ws);
    if (ctx->d_offsets) (void)hipFree(ctx->d_offsets);
    if (ctx->h_pinned) (void)hipHostFree(ctx->h_pinned);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->side) {
        (void)hipStreamSynchronize(ctx->side);
        (void)hipStreamDestroy(ctx->side);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

void* yv_stream(yv_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

// HIP binds each new stream to one of a few hardware queues (GPU_MAX_HW_QUEUES, 4 by default), reusing the least
// used one once they are all taken, so two streams can end up on one queue and run in order: work meant to overlap
// then serialises (the sequence's BA stream against the context stream measured 0.067 vs 0.097 s for 1000 frames, one
// fresh stream in four, profiles/r06/c5, c6).  A stream with an explicit CU mask gets a queue of its own (the mask is
// a property of the queue); with every CU enabled it is an ordinary stream that never shares the context's queue.
void* yv_side_stream(yv_ctx* ctx) {
    if (!ctx) return nullptr;
    if (ctx->side) return reinterpret_cast<void*>(ctx->side);
    if (set_device(ctx) != YV_OK) return nullptr;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus <= 0)
        cus = 256;
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
    if (hipExtStreamCreateWithCUMask(&ctx->side, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        ctx->side = nullptr;
        (void)hipGetLastError();
        if (hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess) ctx->side = nullptr;
    }
    return reinterpret_cast<void*>(ctx->side);
}

int yv_sync(yv_ctx* ctx) {
    if (!ctx) return YV_ERR_INVALID;
    YV_HIP(hipStreamSynchronize(ctx->stream));
    return YV_OK;
}

int yv_download(yv_ctx* ctx, void* host_dst, const void* dev_src, size_t bytes) {
    if (!ctx || (bytes > 0 && (!host_dst || !dev_src))) return YV_ERR_INVALID;
    if (bytes == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    YV_HIP(hipMemcpyAsync(host_dst, dev_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    YV_HIP(hipStreamSynchronize(ctx->stream));
    return YV_OK;
}

int yv_upload(yv_ctx* ctx, void* dev_dst, const void* host_src, size_t bytes) {
    if (!ctx || (bytes > 0 && (!host_src || !dev_dst))) return YV_ERR_INVALID;
    if (bytes == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    YV_HIP(hipMemcpyAsync(dev_dst, host_src, bytes, hipMemcpyHostToDevice, ctx->stream));
    YV_HIP(hipStreamSynchronize(ctx->stream));
    return YV_OK;
}

int yv_device_alloc(yv_ctx* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return YV_ERR_INVALID;
    *out = nullptr;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    YV_HIP(hipMalloc(out, bytes ? bytes : 1));
    return YV_OK;
}

void yv_device_free(yv_ctx* ctx, void* p) {
    if (!ctx || !p) return;
    (void)set_device(ctx);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(p);
}

int yv_host_alloc(yv_ctx* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return YV_ERR_INVALID;
    *out = nullptr;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    YV_HIP(hipHostMalloc(out, bytes ? bytes : 1));
    return YV_OK;
}

void yv_host_free(yv_ctx* ctx, void* p) {
    if (!ctx || !p) return;
    (void)set_device(ctx);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipHostFree(p);
}

int yv_set_fast_params(yv_ctx* ctx, int intensity_threshold, int max_corners) {
    if (!ctx || intensity_threshold < 0 || intensity_threshold > 255 || max_corners < 0 ||
        max_corners > yavo::kMaxKp)
        return YV_ERR_INVALID;
    ctx->fast_thr = intensity_threshold;
    ctx->max_corners = max_corners;
    return YV_OK;
}

int yv_set_harris_eigen(yv_ctx* ctx, int flavour) {
    if (!ctx || flavour < 0 || flavour > 1) return YV_ERR_INVALID;
    ctx->harris_eigen = flavour;
    return YV_OK;
}

int yv_set_brief_offsets(yv_ctx* ctx, const int8_t* offsets) {
    if (!ctx || !offsets) return YV_ERR_INVALID;
    for (int i = 0; i < 1024; ++i)
        if (offsets[i] < -8 || offsets[i] > 8) return YV_ERR_INVALID;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    YV_HIP(hipMemcpyAsync(ctx->d_offsets, offsets, 1024, hipMemcpyHostToDevice, ctx->stream));
    YV_HIP(hipStreamSynchronize(ctx->stream));
    ++ctx->offsets_version;
    return YV_OK;
}

int yv_set_blur_kernel(yv_ctx* ctx, const uint16_t* k9) {
    if (!ctx || !k9) return YV_ERR_INVALID;
    uint32_t sum = 0;
    for (int i = 0; i < 9; ++i) {
        if (k9[i] > 255u) return YV_ERR_INVALID;  // taps are packed as u8 for v_dot4_u32_u8
        sum += k9[i];
    }
    if (sum != 256u) return YV_ERR_INVALID;  // 8 fractional bits: the kernel must sum to 1.0
    std::memcpy(ctx->k9, k9, sizeof(ctx->k9));
    return YV_OK;
}

// ------------------------------------------------------------------------------------------------
// batches
// ------------------------------------------------------------------------------------------------
int yv_batch_create(yv_ctx* ctx, int max_images, int H, int W, int max_kp, int max_pairs, yv_batch** out) {
    if (!ctx || !out || max_images <= 0 || H < 9 || W < 9 || max_kp <= 0 || max_kp > yavo::kMaxKp ||
        max_pairs < 0 || (int64_t)H * W >= (1ll << 31))
        return YV_ERR_INVALID;
    if (W > yavo::kMaxWidth) return YV_ERR_CAPACITY;  // BRIEF stages 49 image rows in LDS
    if (H > yavo::kBandRows * yavo::kMaxBands) return YV_ERR_CAPACITY;  // top-K's band lists
    *out = nullptr;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    yv_batch* b = new (std::nothrow) yv_batch();
    if (!b) return YV_ERR_INVALID;
    b->ctx = ctx;
    b->max_images = max_images;
    b->H = H;
    b->W = W;
    b->max_kp = max_kp;
    b->max_pairs = max_pairs;
    b->nslots = max_images + 1;
    b->cap = (int64_t)(H - 8) * (W - 8);  // every pixel FAST can test: no candidate is ever dropped
    const size_t ns = (size_t)b->nslots, nk = (size_t)max_kp, np = (size_t)std::max(max_pairs, 1);
    int rc = YV_OK;
    rc |= dalloc(&b->cand_keys, (size_t)max_images * (size_t)b->cap);
    rc |= dalloc(&b->cand_count, ns);
    rc |= dalloc(&b->cand_seen, ns);
    rc |= dalloc(&b->det_rc, ns * nk * 2);
    rc |= dalloc(&b->det_resp, ns * nk);
    rc |= dalloc(&b->det_count, ns);
    rc |= dalloc(&b->kp_src, ns * nk * 4);
    rc |= dalloc(&b->kp_count, ns);
    rc |= dalloc(&b->kp_count_build, ns);
    rc |= dalloc(&b->kp_band, ns * nk * 4);
    rc |= dalloc(&b->band_off, ns * (size_t)(yavo::kMaxBands + 1));
    rc |= dalloc(&b->brief_loff, 512);
    rc |= dalloc(&b->keypoints, ns * nk);
    rc |= dalloc(&b->desc, ns * nk);
    rc |= dalloc(&b->blur, (size_t)max_images * (size_t)yavo::blur_image_bytes(H, W));
    rc |= dalloc(&b->pairs, np * 2);
    rc |= dalloc(&b->match_key, np * nk);
    rc |= dalloc(&b->matches, np * nk);
    rc |= dalloc(&b->match_count, np);
    rc |= dalloc(&b->filtered, np * nk);
    rc |= dalloc(&b->filt_count, np);
    rc |= dalloc(&b->match_dj, np * nk);
    rc |= dalloc(&b->match_lim, np);
    rc |= dalloc(&b->staging, (size_t)H * W);
    if (rc != YV_OK) {
        batch_free(b);
        return YV_ERR_HIP;
    }
    hipStream_t s = ctx->stream;
    bool ok = hipMemsetAsync(b->cand_count, 0, ns * sizeof(uint32_t), s) == hipSuccess &&
              hipMemsetAsync(b->cand_seen, 0, ns * sizeof(uint32_t), s) == hipSuccess &&
              hipMemsetAsync(b->kp_count, 0, ns * sizeof(int32_t), s) == hipSuccess &&
              hipMemsetAsync(b->det_count, 0, ns * sizeof(int32_t), s) == hipSuccess &&
              hipMemsetAsync(b->match_key, 0xFF, np * nk * sizeof(uint32_t), s) == hipSuccess &&
              hipMemsetAsync(b->keypoints, 0, ns * nk * sizeof(yv_keypoint), s) == hipSuccess &&
              hipMemsetAsync(b->match_count, 0, np * sizeof(int32_t), s) == hipSuccess &&
              hipMemsetAsync(b->filt_count, 0, np * sizeof(int32_t), s) == hipSuccess &&
              hipMemsetAsync(b->match_lim, 0, np * sizeof(int32_t), s) == hipSuccess &&
              hipStreamSynchronize(s) == hipSuccess;
    if (!ok) {
        batch_free(b);
        return YV_ERR_HIP;
    }
    *out = b;
    return YV_OK;
}

void yv_batch_destroy(yv_batch* b) {
    if (!b) return;
    (void)hipSetDevice(b->ctx->device);
    (void)hipStreamSynchronize(b->ctx->stream);
    batch_free(b);
}

int yv_batch_set_pairs(yv_batch* b, const int32_t* pairs, int n_pairs) {
    if (!b || n_pairs < 0 || n_pairs > b->max_pairs || (n_pairs > 0 && !pairs)) return YV_ERR_INVALID;
    for (int i = 0; i < 2 * n_pairs; ++i)
        if (pairs[i] < 0 || pairs[i] > b->max_images) return YV_ERR_INVALID;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    if (b->bstream) YV_HIP(hipStreamSynchronize(b->bstream));  // an edge build in flight reads pairs
    b->build_pending = false;
    if (n_pairs > 0) {
        YV_HIP(hipMemcpyAsync(b->pairs, pairs, sizeof(int32_t) * 2 * (size_t)n_pairs, hipMemcpyHostToDevice,
                              b->ctx->stream));
        YV_HIP(hipStreamSynchronize(b->ctx->stream));
    }
    b->h_pairs.assign(pairs, pairs + 2 * (size_t)n_pairs);
    b->n_pairs = n_pairs;
    b->n_tracks = 0;  // tracks refer to pair indices: set them again
    return YV_OK;
}

int yv_batch_enable_timing(yv_batch* b, int on) {
    if (!b) return YV_ERR_INVALID;
    if (on && b->events.empty()) {
        if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
        b->events.resize((size_t)kMaxTimedRuns * kEvPerRun);
        for (auto& e : b->events) YV_HIP(hipEventCreate(&e));
        b->tracked.assign(kMaxTimedRuns, 0);
    }
    b->timing = on == 2 ? 2 : (on != 0 ? 1 : 0);
    b->runs_recorded = 0;
    b->last_run = -1;
    std::fill(b->tracked.begin(), b->tracked.end(), 0);
    return YV_OK;
}

int yv_batch_stage_times(yv_batch* b, float* ms, int* n_runs) {
    if (!b || !ms) return YV_ERR_INVALID;
    for (int i = 0; i < 8; ++i) ms[i] = 0.f;
    const int runs = std::min(b->runs_recorded, kMaxTimedRuns);
    if (n_runs) *n_runs = runs;
    if (runs == 0) return YV_OK;
    for (int r = 0; r < runs; ++r) {
        const hipEvent_t* ev = &b->events[(size_t)r * kEvPerRun];
        if (b->timing == 2) {
            float t = 0.f;
            YV_HIP(hipEventSynchronize(ev[1]));
            YV_HIP(hipEventElapsedTime(&t, ev[0], ev[1]));
            ms[0] += t;
            continue;
        }
        YV_HIP(hipEventSynchronize(ev[b->tracked[r] ? 8 : 5]));
        for (int st = 0; st < 5; ++st) {
            float t = 0.f;
            YV_HIP(hipEventElapsedTime(&t, ev[st], ev[st + 1]));
            ms[st] += t;
        }
        if (b->tracked[r])
            for (int st = 5; st < 7; ++st) {
                float t = 0.f;
                YV_HIP(hipEventElapsedTime(&t, ev[st + 1], ev[st + 2]));
                ms[st] += t;
            }
    }
    return YV_OK;
}

namespace {
int launch_deferred_after(yv_batch* b, hipStream_t s);
int flush_deferred(yv_batch* b);
}  // namespace

int yv_batch_run(yv_batch* b, const uint8_t* d_images, int n_images, int stride, int64_t image_pitch, int match_thr,
                 int carry_from, void* stream) {
    if (!b || !d_images || n_images <= 0 || n_images > b->max_images || stride < b->W ||
        image_pitch < (int64_t)stride * (b->H - 1) + b->W || carry_from >= n_images)
        return YV_ERR_INVALID;
    yv_ctx* ctx = b->ctx;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
    const int H = b->H, W = b->W, K = b->max_kp;
    const int keep = std::min(ctx->max_corners, K);
    if (b->pending_carry >= 0 && join_build(b, s) != YV_OK) return YV_ERR_HIP;
    if (b->pending_carry >= 0) {
        const size_t c = (size_t)b->pending_carry, dst = (size_t)b->max_images, nk = (size_t)K;
        YV_HIP(hipMemcpyAsync(b->keypoints + dst * nk, b->keypoints + c * nk, nk * sizeof(yv_keypoint),
                              hipMemcpyDeviceToDevice, s));
        YV_HIP(hipMemcpyAsync(b->desc + dst * nk, b->desc + c * nk, nk * sizeof(Desc), hipMemcpyDeviceToDevice, s));
        YV_HIP(hipMemcpyAsync(b->kp_count + dst, b->kp_count + c, sizeof(int32_t), hipMemcpyDeviceToDevice, s));
        b->pending_carry = -1;
    }
    int run = -1;
    if (b->timing && b->runs_recorded < kMaxTimedRuns) run = b->runs_recorded++;
    b->last_run = run;
    int rc = YV_OK;
    rc |= record_stage(b, s, run, 0);
    yavo::launch_detect_blur(d_images, n_images, H, W, stride, image_pitch, ctx->fast_thr, ctx->harris_eigen, b->cand_keys, b->cap,
                             b->cand_count, ctx->k9, b->blur, s);
    rc |= record_stage(b, s, run, 1);
    if (b->overlap_mode == 2) rc |= launch_deferred_after(b, s);
    yavo::launch_topk(b->cand_keys, b->cap, b->cand_count, b->cand_seen, n_images, H, W, K, keep, b->det_rc,
                      b->det_resp, b->det_count, b->kp_src, b->kp_count, b->kp_band, b->band_off, s);
    rc |= record_stage(b, s, run, 2);
    if (b->overlap_mode == 4) rc |= launch_deferred_after(b, s);  // after top-K
    // the previous track's build (beside detect and top-K) reads keypoints / matches: BRIEF and finalize rewrite them
    // (its keypoint counts are a copy, kp_count_build, so top-K need not wait)
    rc |= join_build(b, s);
    // the tests' LDS offsets depend on the offsets table and W only: formed again only when the table changed (a
    // 256-thread launch in the step waited ~15-50 us for a CU behind the side stream's LM, profiles/r06/c17)
    const bool new_loff = b->loff_version != ctx->offsets_version;
    b->loff_version = ctx->offsets_version;
    yavo::launch_brief(b->blur, n_images, H, W, ctx->d_offsets, b->kp_src, b->kp_band, b->band_off, K, b->keypoints,
                       b->desc, b->brief_loff, new_loff, s);
    rc |= record_stage(b, s, run, 3);
    if (b->overlap_mode == 3) rc |= launch_deferred_after(b, s);  // after describe
    if (b->n_pairs > 0) {
        yavo::launch_match(b->desc, b->kp_count, b->pairs, b->n_pairs, K, K, b->match_key, s);
        rc |= record_stage(b, s, run, 4);
        // the asynchronous edge build reads a copy of the keypoint counts (the next run's top-K rewrites them):
        // the finalize kernel writes it, where a separate device copy waited ~50 us for a CU at the end of the step
        const bool copy_counts = b->overlap && b->build_async && b->lk_step == 0;
        yavo::launch_match_finalize(b->match_key, b->keypoints, b->kp_count, b->pairs, b->n_pairs, K, match_thr,
                                    b->matches, b->match_count, b->filtered, b->filt_count, b->match_dj,
                                    b->match_lim, s, copy_counts ? b->kp_count_build : nullptr, b->nslots);
        b->counts_copied = copy_counts;
    } else {
        rc |= record_stage(b, s, run, 4);
        b->counts_copied = false;
    }
    rc |= record_stage(b, s, run, 5);
    if (rc != YV_OK) return YV_ERR_HIP;
    // The carry slot keeps this run's frame k-1 (the query of its first temporal pair) until the next run
    // starts, so yv_batch_track and the view still see it; the copy of image carry_from is deferred.
    b->pending_carry = carry_from;
    b->run_images = d_images;
    b->run_n = n_images;
    b->run_stride = stride;
    b->run_pitch = image_pitch;
    return check_launch();
}

int yv_batch_view_get(yv_batch* b, yv_batch_view* v) {
    if (!b || !v) return YV_ERR_INVALID;
    v->max_images = b->max_images;
    v->max_kp = b->max_kp;
    v->max_pairs = b->max_pairs;
    v->H = b->H;
    v->W = b->W;
    v->cand_cap = b->cap;
    v->cand_count = b->cand_seen;
    v->det_count = b->det_count;
    v->det_rc = b->det_rc;
    v->det_resp = b->det_resp;
    v->kp_count = b->kp_count;
    v->keypoints = b->keypoints;
    v->blurred = b->blur;
    v->blur_pitch = yavo::blur_pitch(b->W);
    v->match_count = b->match_count;
    v->matches = b->matches;
    v->filt_count = b->filt_count;
    v->filtered = b->filtered;
    v->match_dj = reinterpret_cast<const int32_t*>(b->match_dj);
    v->match_lim = b->match_lim;
    v->n_tracks = b->n_tracks;
    const size_t nt = (size_t)b->max_tracks, nk = (size_t)b->max_kp, k = (size_t)b->tbuf;
    v->edge_count = b->edge_count ? b->edge_count + k * nt : nullptr;
    v->edge_X = b->edge_X ? b->edge_X + k * nt * nk * 3 : nullptr;
    v->edge_uv = b->edge_uv ? b->edge_uv + k * nt * nk * 2 : nullptr;
    v->edge_query = b->edge_query ? b->edge_query + k * nt * nk : nullptr;
    v->edge_outlier = b->edge_outlier ? b->edge_outlier + k * nt * nk : nullptr;
    v->track_inliers = b->track_inliers ? b->track_inliers + k * nt : nullptr;
    return YV_OK;
}

int yv_batch_set_tracks(yv_batch* b, const int32_t* tracks, int n_tracks, const double K[9], const double T_right[7]) {
    if (!b || n_tracks < 0 || (n_tracks > 0 && (!tracks || !K || !T_right))) return YV_ERR_INVALID;
    for (int t = 0; t < n_tracks; ++t) {
        const int sp = tracks[2 * t], tp = tracks[2 * t + 1];
        if (sp < 0 || sp >= b->n_pairs) return YV_ERR_INVALID;
        if (b->lk_step > 0) {
            // LK mode: {stereo pair of frame k-1, image of frame k}, both LK images (multiples of the step)
            const int prev = b->h_pairs[2 * sp];
            if (prev % b->lk_step || prev >= b->max_images || tp < 0 || tp >= b->max_images || tp % b->lk_step)
                return YV_ERR_INVALID;
        } else {
            if (tp < 0 || tp >= b->n_pairs) return YV_ERR_INVALID;
            if (b->h_pairs[2 * sp] != b->h_pairs[2 * tp + 1]) return YV_ERR_INVALID;  // stereo query = temporal train
        }
    }
    for (int i = 0; i < 9 && n_tracks > 0; ++i)
        if (!std::isfinite(K[i])) return YV_ERR_INVALID;
    if (n_tracks > 0 && !finite_pose(T_right)) return YV_ERR_INVALID;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    hipStream_t s = b->ctx->stream;
    if (b->bstream) YV_HIP(hipStreamSynchronize(b->bstream));  // a build in flight reads tracks / K
    b->build_pending = false;
    if (b->side) YV_HIP(hipStreamSynchronize(b->side));  // an LM in flight reads tracks / K
    if (n_tracks > b->max_tracks) {
        void* old[] = {b->tracks, b->track_K, b->T_right, b->edge_X, b->edge_uv, b->edge_query, b->edge_count,
                       b->edge_outlier, b->track_inliers};
        YV_HIP(hipStreamSynchronize(s));
        if (b->side) YV_HIP(hipStreamSynchronize(b->side));
        for (void* p : old)
            if (p) (void)hipFree(p);
        b->tracks = nullptr; b->track_K = nullptr; b->T_right = nullptr; b->edge_X = nullptr; b->edge_uv = nullptr;
        b->edge_query = nullptr; b->edge_count = nullptr; b->edge_outlier = nullptr; b->track_inliers = nullptr;
        b->max_tracks = 0;
        b->n_tracks = 0;
        const size_t nt = (size_t)n_tracks, nk = (size_t)b->max_kp;
        int rc = YV_OK;
        rc |= dalloc(&b->tracks, 2 * nt);
        rc |= dalloc(&b->track_K, 9 * nt);
        rc |= dalloc(&b->T_right, 7);
        rc |= dalloc(&b->edge_X, kEdgeBufs * 3 * nt * nk);
        rc |= dalloc(&b->edge_uv, kEdgeBufs * 2 * nt * nk);
        rc |= dalloc(&b->edge_query, kEdgeBufs * nt * nk);
        rc |= dalloc(&b->edge_count, kEdgeBufs * nt);
        rc |= dalloc(&b->edge_outlier, kEdgeBufs * nt * nk);
        rc |= dalloc(&b->track_inliers, kEdgeBufs * nt);
        void* lk_old[] = {b->lk_sp, b->lk_pairs, b->lk_X, b->lk_pts, b->lk_next, b->lk_err, b->lk_status, b->lk_q,
                          b->lk_count};
        for (void* p : lk_old)
            if (p) (void)hipFree(p);
        b->lk_sp = b->lk_pairs = b->lk_q = b->lk_count = nullptr;
        b->lk_X = nullptr;
        b->lk_pts = b->lk_next = b->lk_err = nullptr;
        b->lk_status = nullptr;
        rc |= dalloc(&b->lk_sp, nt);
        rc |= dalloc(&b->lk_pairs, 2 * nt);
        rc |= dalloc(&b->lk_X, 2 * 3 * nt * nk);
        rc |= dalloc(&b->lk_pts, 2 * 2 * nt * nk);
        rc |= dalloc(&b->lk_next, 2 * nt * nk);
        rc |= dalloc(&b->lk_err, nt * nk);
        rc |= dalloc(&b->lk_status, nt * nk);
        rc |= dalloc(&b->lk_q, 2 * nt * nk);
        rc |= dalloc(&b->lk_count, 2 * nt);
        b->lk_ev_pending[0] = b->lk_ev_pending[1] = false;
        if (rc != YV_OK) return YV_ERR_HIP;
        b->max_tracks = n_tracks;
    }
    if (n_tracks > 0) {
        std::vector<double> Ks(9 * (size_t)n_tracks);
        for (int t = 0; t < n_tracks; ++t) std::memcpy(&Ks[9 * (size_t)t], K, 9 * sizeof(double));
        YV_HIP(hipMemcpyAsync(b->tracks, tracks, 2 * sizeof(int32_t) * (size_t)n_tracks, hipMemcpyHostToDevice, s));
        YV_HIP(hipMemcpyAsync(b->track_K, Ks.data(), Ks.size() * sizeof(double), hipMemcpyHostToDevice, s));
        YV_HIP(hipMemcpyAsync(b->T_right, T_right, 7 * sizeof(double), hipMemcpyHostToDevice, s));
        YV_HIP(hipMemsetAsync(b->edge_count, 0, kEdgeBufs * sizeof(int32_t) * (size_t)b->max_tracks, s));
        if (b->lk_step > 0) {
            std::vector<int32_t> sp(n_tracks), lp(2 * (size_t)n_tracks);
            for (int t = 0; t < n_tracks; ++t) {
                sp[t] = tracks[2 * t];
                lp[2 * t] = b->h_pairs[2 * sp[t]] / b->lk_step;
                lp[2 * t + 1] = tracks[2 * t + 1] / b->lk_step;
            }
            YV_HIP(hipMemcpyAsync(b->lk_sp, sp.data(), sizeof(int32_t) * sp.size(), hipMemcpyHostToDevice, s));
            YV_HIP(hipMemcpyAsync(b->lk_pairs, lp.data(), sizeof(int32_t) * lp.size(), hipMemcpyHostToDevice, s));
        }
        YV_HIP(hipStreamSynchronize(s));
    }
    b->n_tracks = n_tracks;
    return YV_OK;
}

namespace {

struct MapArgs {
    int64_t first_frame;
    int kf_every, max_kf;
    void* block;
};

int batch_track(yv_batch* b, const double* d_priors, double* d_poses, void* stream, const MapArgs* map);

// The pose LM (and the map block) of one track. Overlap: on the side stream after the edge build (ev_edges[k]);
// otherwise on `s`, in order.
int launch_lm(yv_batch* b, const yv_batch::DeferredLM& L, hipStream_t s) {
    const int k = L.k;
    const size_t nt = (size_t)b->max_tracks, nk = (size_t)b->max_kp;
    double* eX = b->edge_X + k * nt * nk * 3;
    double* euv = b->edge_uv + k * nt * nk * 2;
    int32_t* ec = b->edge_count + k * nt;
    uint8_t* eo = b->edge_outlier + k * nt * nk;
    int32_t* inl = b->track_inliers + k * nt;
    hipStream_t ls = s;
    if (b->overlap) {
        // the LM reads only this track's edge buffer, priors and poses: it runs on the side stream beside the
        // next batch's image kernels (which overwrite keypoints / matches, already consumed by the build)
        YV_HIP(hipStreamWaitEvent(b->side, b->ev_edges[k], 0));
        ls = b->side;
    }
    if (L.ev) YV_HIP(hipEventRecord(L.ev[7], ls));
    yavo::launch_track_pose(b->n_tracks, ec, b->max_kp, eX, euv, b->track_K, L.priors, L.poses, eo, inl, ls);
    if (L.ev) {
        YV_HIP(hipEventRecord(L.ev[8], ls));
        b->tracked[L.run] = 1;
    }
    if (L.has_map) {
        // the chunk's map block, after the LM on its stream: the build that next rewrites this edge buffer waits
        // for ev_lm[k], recorded below, so it also waits for these reads. The block itself is rewritten only
        // after its last reader released it (the all-gather of the previous chunk, yv_batch_map_release).
        if (b->map_release_pending) {
            YV_HIP(hipStreamWaitEvent(ls, b->ev_map_release, 0));
            b->map_release_pending = false;
        }
        yavo::launch_map_chunk(L.poses, b->n_tracks, L.first_frame, L.kf_every, ec, eX, eo, b->max_kp, L.max_kf,
                               L.block, ls);
        if (!b->ev_map) YV_HIP(hipEventCreateWithFlags(&b->ev_map, hipEventDisableTiming));
        YV_HIP(hipEventRecord(b->ev_map, ls));
        b->map_written = true;
    }
    if (b->overlap) {
        YV_HIP(hipEventRecord(b->ev_lm[k], ls));
        b->lm_pending[k] = true;
    }
    return YV_OK;
}

// The deferred LM of the previous track, ordered after the work issued on s so far (the stage it waits for).
int launch_deferred_after(yv_batch* b, hipStream_t s) {
    if (!b->deferred.active) return YV_OK;
    if (!b->ev_defer) YV_HIP(hipEventCreateWithFlags(&b->ev_defer, hipEventDisableTiming));
    YV_HIP(hipEventRecord(b->ev_defer, s));
    YV_HIP(hipStreamWaitEvent(b->side, b->ev_defer, 0));
    b->deferred.active = false;
    return launch_lm(b, b->deferred, s) == YV_OK ? YV_OK : YV_ERR_HIP;
}

// Launch a deferred LM now (its inputs are complete once ev_edges was recorded).
int flush_deferred(yv_batch* b) {
    if (!b->deferred.active) return YV_OK;
    b->deferred.active = false;
    return launch_lm(b, b->deferred, b->ctx->stream);
}

}  // namespace

int yv_batch_track(yv_batch* b, const double* d_priors, double* d_poses, void* stream) {
    return batch_track(b, d_priors, d_poses, stream, nullptr);
}

int yv_batch_track_map(yv_batch* b, const double* d_priors, double* d_poses, int64_t first_frame, int kf_every,
                       void* d_block, int max_kf, void* stream) {
    if (!b || !d_block || kf_every < 1 || max_kf < 1 || first_frame < 0) return YV_ERR_INVALID;
    const MapArgs m{first_frame, kf_every, max_kf, d_block};
    return batch_track(b, d_priors, d_poses, stream, &m);
}

int yv_batch_map_wait(yv_batch* b, void* stream) {
    if (!b || !stream) return YV_ERR_INVALID;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    if (flush_deferred(b) != YV_OK) return YV_ERR_HIP;  // the block is written after the LM
    if (!b->map_written) return YV_OK;
    YV_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), b->ev_map, 0));
    return YV_OK;
}

int yv_batch_map_release(yv_batch* b, void* stream) {
    if (!b || !stream) return YV_ERR_INVALID;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    if (!b->ev_map_release) YV_HIP(hipEventCreateWithFlags(&b->ev_map_release, hipEventDisableTiming));
    YV_HIP(hipEventRecord(b->ev_map_release, reinterpret_cast<hipStream_t>(stream)));
    b->map_release_pending = true;
    return YV_OK;
}

namespace {

int batch_track(yv_batch* b, const double* d_priors, double* d_poses, void* stream, const MapArgs* map) {
    if (!b || (b->n_tracks > 0 && (!d_priors || !d_poses))) return YV_ERR_INVALID;
    if (b->n_tracks == 0) return YV_OK;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : b->ctx->stream;
    if (flush_deferred(b) != YV_OK) return YV_ERR_HIP;  // two tracks without a run between them
    const int k = b->track_calls++ % kEdgeBufs;
    const size_t nt = (size_t)b->max_tracks, nk = (size_t)b->max_kp;
    double* eX = b->edge_X + k * nt * nk * 3;
    double* euv = b->edge_uv + k * nt * nk * 2;
    int32_t* eq = b->edge_query + k * nt * nk;
    int32_t* ec = b->edge_count + k * nt;
    const int run = b->last_run;
    const bool timed = b->timing == 1 && run >= 0 && !b->tracked[run];
    hipEvent_t* ev = timed ? &b->events[(size_t)run * kEvPerRun] : nullptr;
    const hipStream_t s_run = s;
    double* lkX = nullptr;
    float* lkP = nullptr;
    int32_t *lkQ = nullptr, *lkC = nullptr;
    int lk_j = 0;
    if (b->lk_step > 0) {
        // LK: frame k-1's stereo map points from this run's keypoints / matches, on the run's stream (the next run
        // rewrites them), into the point set the LK stage two tracks ago has finished reading
        if (!b->run_images || b->run_n < b->lk_step) return YV_ERR_INVALID;
        lk_j = b->lk_set;
        b->lk_set ^= 1;
        lkX = b->lk_X + (size_t)lk_j * nt * nk * 3;
        lkP = b->lk_pts + (size_t)lk_j * nt * nk * 2;
        lkQ = b->lk_q + (size_t)lk_j * nt * nk;
        lkC = b->lk_count + (size_t)lk_j * nt;
        if (b->lk_ev_pending[lk_j]) YV_HIP(hipStreamWaitEvent(s_run, b->ev_lk[lk_j], 0));
        b->lk_ev_pending[lk_j] = false;
        yavo::launch_stereo_points(b->lk_sp, b->n_tracks, b->pairs, b->keypoints, b->kp_count, b->match_dj,
                                   b->match_lim, b->max_kp, b->track_K, b->T_right, lkX, lkP, lkQ, lkC, s_run);
    }
    const int32_t* build_counts = b->kp_count;
    if (b->overlap && b->build_async) {
        // the build (match: edges from the run's matches; LK: pyramids, flow, edges) waits for the run on s and
        // leaves s free for the next run's detect; the match build reads a copy of the keypoint counts
        if (b->lk_step == 0) {
            if (!b->counts_copied)
                YV_HIP(hipMemcpyAsync(b->kp_count_build, b->kp_count, sizeof(int32_t) * (size_t)b->nslots,
                                      hipMemcpyDeviceToDevice, s_run));
            build_counts = b->kp_count_build;
        }
        YV_HIP(hipEventRecord(b->ev_fin, s_run));
        YV_HIP(hipStreamWaitEvent(b->bstream, b->ev_fin, 0));
        s = b->bstream;
    }
    // buffer k was last read by the LM kEdgeBufs tracks ago (side stream): the build must not overwrite it early
    if (b->lm_pending[k]) YV_HIP(hipStreamWaitEvent(s, b->ev_lm[k], 0));
    if (timed) YV_HIP(hipEventRecord(ev[6], s));
    if (b->lk_step > 0) {
        // trackLastFrame: frame k-1's stereo map points -> calcOpticalFlowPyrLK into frame k -> edges
        const int n_lk = (b->run_n + b->lk_step - 1) / b->lk_step;
        int rc = yv_lk_build(b->lk, b->run_images, n_lk, b->run_stride, b->run_pitch * b->lk_step, s);
        if (rc != YV_OK) return rc;
        rc = yv_lk_track_batch(b->lk, b->lk_pairs, b->n_tracks, lkP, lkC, b->max_kp, b->lk_max_count, b->lk_eps,
                               b->lk_min_eig, b->lk_next, b->lk_status, b->lk_err, s);
        if (rc != YV_OK) return rc;
        yavo::launch_lk_edges(b->n_tracks, lkX, b->lk_next, b->lk_status, lkQ, lkC, b->max_kp, eX, euv, eq, ec, s);
        if (s != s_run) {
            if (!b->ev_lk[lk_j]) YV_HIP(hipEventCreateWithFlags(&b->ev_lk[lk_j], hipEventDisableTiming));
            YV_HIP(hipEventRecord(b->ev_lk[lk_j], s));
            b->lk_ev_pending[lk_j] = true;
        }
    } else {
        yavo::launch_track_build(b->tracks, b->n_tracks, b->pairs, b->keypoints, build_counts, b->match_dj,
                                 b->match_lim, b->max_kp, b->track_K, b->T_right, eX, euv, eq, ec, s);
    }
    if (b->overlap) YV_HIP(hipEventRecord(b->ev_edges[k], s));
    if (s != s_run && b->lk_step == 0) {  // (the LK stage reads nothing the next run writes: no join)
        YV_HIP(hipEventRecord(b->ev_built, s));
        b->build_pending = true;
    }
    yv_batch::DeferredLM L;
    L.active = true;
    L.k = k;
    L.run = timed ? run : -1;
    L.priors = d_priors;
    L.poses = d_poses;
    L.ev = ev;
    if (map) {
        L.has_map = true;
        L.first_frame = map->first_frame;
        L.kf_every = map->kf_every;
        L.max_kf = map->max_kf;
        L.block = map->block;
    }
    b->tbuf = k;
    if (b->overlap_mode >= 2) {
        // launched by the next yv_batch_run after its detect (2) / describe (3) stage, or by a flush
        b->deferred = L;
        return check_launch();
    }
    const int rc = launch_lm(b, L, s);
    if (rc != YV_OK) return rc;
    return check_launch();
}

}  // namespace

int yv_batch_set_track_overlap(yv_batch* b, int on) {
    if (!b || on < 0 || on > 4) return YV_ERR_INVALID;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    if (flush_deferred(b) != YV_OK) return YV_ERR_HIP;
    if (on && !b->side) {
        // lowest priority: the LM fills the CUs the next batch's detect / describe / match leave idle
        int least = 0, greatest = 0;
        YV_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        YV_HIP(hipStreamCreateWithPriority(&b->side, hipStreamNonBlocking, least));
        for (int k = 0; k < kEdgeBufs; ++k) {
            YV_HIP(hipEventCreateWithFlags(&b->ev_edges[k], hipEventDisableTiming));
            YV_HIP(hipEventCreateWithFlags(&b->ev_lm[k], hipEventDisableTiming));
        }
        // the build stream at the default priority (the highest and the lowest measured the same)
        YV_HIP(hipStreamCreateWithFlags(&b->bstream, hipStreamNonBlocking));
        YV_HIP(hipEventCreateWithFlags(&b->ev_fin, hipEventDisableTiming));
        YV_HIP(hipEventCreateWithFlags(&b->ev_built, hipEventDisableTiming));
    }
    if (!on && b->bstream) YV_HIP(hipStreamSynchronize(b->bstream));
    if (!on) b->build_pending = false;
    {
        const char* e = std::getenv("YAVO_BUILD_ASYNC");
        b->build_async = on != 0 && !(e && e[0] == '0');
    }
    if (!on && b->side) YV_HIP(hipStreamSynchronize(b->side));
    b->overlap = on != 0;
    b->overlap_mode = on;
    return YV_OK;
}

int yv_batch_track_sync(yv_batch* b) {
    if (!b) return YV_ERR_INVALID;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    if (flush_deferred(b) != YV_OK) return YV_ERR_HIP;
    if (b->bstream) YV_HIP(hipStreamSynchronize(b->bstream));
    if (b->side) YV_HIP(hipStreamSynchronize(b->side));
    return YV_OK;
}

int yv_batch_set_track_lk(yv_batch* b, int image_step, int win, int max_level, int max_count, double eps,
                          double min_eig) {
    if (!b || image_step < 0 || (image_step > 0 && (win < 3 || win > 22 || max_level < 0))) return YV_ERR_INVALID;
    if (set_device(b->ctx) != YV_OK) return YV_ERR_HIP;
    if (flush_deferred(b) != YV_OK) return YV_ERR_HIP;
    if (b->side) YV_HIP(hipStreamSynchronize(b->side));
    if (b->bstream) YV_HIP(hipStreamSynchronize(b->bstream));  // an edge build in flight (as its siblings drain)
    b->build_pending = false;
    YV_HIP(hipStreamSynchronize(b->ctx->stream));
    if (b->lk) {
        yv_lk_destroy(b->lk);
        b->lk = nullptr;
    }
    b->lk_step = image_step;
    b->n_tracks = 0;  // tracks change meaning with the mode: set them again
    if (image_step == 0) return YV_OK;
    const int slots = (b->max_images + image_step - 1) / image_step;
    const int rc = yv_lk_create(b->ctx, slots, b->H, b->W, win, max_level, &b->lk);
    if (rc != YV_OK) {
        b->lk_step = 0;
        return rc;
    }
    b->lk_max_count = max_count;
    b->lk_eps = eps;
    b->lk_min_eig = min_eig;
    return YV_OK;
}

// ------------------------------------------------------------------------------------------------
// host-pointer drop-in entry points
// ------------------------------------------------------------------------------------------------
static int upload_image(yv_batch* b, const uint8_t* img, int stride, hipStream_t s) {
    YV_HIP(stage_h2d_2d(b->ctx, b->staging, (size_t)b->W, img, (size_t)stride, (size_t)b->W, (size_t)b->H, s));
    return YV_OK;
}

int yv_detect(yv_ctx* ctx, const uint8_t* img, int H, int W, int stride, int max_kp, int32_t* rc, float* resp,
              int* n, int* n_candidates) {
    if (!ctx || !img || !rc || !n || H < 9 || W < 9 || stride < W || max_kp < 0) return YV_ERR_INVALID;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    int st = ensure_single(ctx, H, W);
    if (st != YV_OK) return st;
    yv_batch* b = ctx->single;
    hipStream_t s = ctx->stream;
    const int keep = std::min(std::min(ctx->max_corners, max_kp), b->max_kp);
    if (upload_image(b, img, stride, s) != YV_OK) return YV_ERR_HIP;
    yavo::launch_fast_harris(b->staging, 1, H, W, W, (int64_t)H * W, ctx->fast_thr, ctx->harris_eigen, b->cand_keys, b->cap,
                             b->cand_count, s);
    yavo::launch_topk(b->cand_keys, b->cap, b->cand_count, b->cand_seen, 1, H, W, b->max_kp, keep, b->det_rc, b->det_resp,
                      b->det_count, b->kp_src, b->kp_count, b->kp_band, b->band_off, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    YV_HIP(stage_d2h(ctx, ctx->h_pinned, b->det_count, sizeof(int32_t), s));
    YV_HIP(stage_d2h(ctx, ctx->h_pinned + 1, b->cand_seen, sizeof(uint32_t), s));
    YV_HIP(stage_sync(ctx, s));
    const int k = ctx->h_pinned[0];
    if (k > 0) {
        YV_HIP(stage_d2h(ctx, rc, b->det_rc, sizeof(int32_t) * 2 * (size_t)k, s));
        if (resp) YV_HIP(stage_d2h(ctx, resp, b->det_resp, sizeof(float) * (size_t)k, s));
        YV_HIP(stage_sync(ctx, s));
    }
    *n = k;
    if (n_candidates) *n_candidates = ctx->h_pinned[1];
    return YV_OK;
}

int yv_describe(yv_ctx* ctx, const uint8_t* img, int H, int W, int stride, const int32_t* rc, int n, yv_keypoint* out,
                int* n_out) {
    if (!ctx || !img || !out || !n_out || H < 9 || W < 9 || stride < W || n < 0 || (n > 0 && !rc)) return YV_ERR_INVALID;
    if (n > yavo::kMaxKp) return YV_ERR_CAPACITY;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    int st = ensure_single(ctx, H, W);
    if (st != YV_OK) return st;
    yv_batch* b = ctx->single;
    hipStream_t s = ctx->stream;
    if (upload_image(b, img, stride, s) != YV_OK) return YV_ERR_HIP;
    ctx->h_pinned[0] = n;
    if (n > 0) YV_HIP(stage_h2d(ctx, b->det_rc, rc, sizeof(int32_t) * 2 * (size_t)n, s));
    YV_HIP(stage_h2d(ctx, b->det_count, ctx->h_pinned, sizeof(int32_t), s));
    yavo::launch_blur9(b->staging, 1, H, W, W, (int64_t)H * W, ctx->k9, b->blur, s);
    yavo::launch_kp_boundary(b->det_rc, b->det_count, 1, H, W, b->max_kp, b->kp_src, b->kp_count, b->kp_band,
                             b->band_off, s);
    const bool new_loff = b->loff_version != ctx->offsets_version;
    b->loff_version = ctx->offsets_version;
    yavo::launch_brief(b->blur, 1, H, W, ctx->d_offsets, b->kp_src, b->kp_band, b->band_off, b->max_kp, b->keypoints,
                       b->desc, b->brief_loff, new_loff, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    YV_HIP(stage_d2h(ctx, ctx->h_pinned + 2, b->kp_count, sizeof(int32_t), s));
    YV_HIP(stage_sync(ctx, s));
    const int m = ctx->h_pinned[2];
    if (m > 0) {
        YV_HIP(stage_d2h(ctx, out, b->keypoints, sizeof(yv_keypoint) * (size_t)m, s));
        YV_HIP(stage_sync(ctx, s));
    }
    *n_out = m;
    return YV_OK;
}

int yv_match_features(yv_ctx* ctx, const yv_keypoint* q, int nq, const yv_keypoint* t, int nt, yv_match* out) {
    if (!ctx || nq < 0 || nt < 0 || (nq > 0 && (!q || !out)) || (nt > 0 && !t)) return YV_ERR_INVALID;
    if (nq > yavo::kMaxKp || nt > yavo::kMaxKp) return YV_ERR_CAPACITY;
    if (nq == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    // the matcher does not look at the image size: reuse whatever workspace exists (or a minimal one)
    int st = ctx->single ? YV_OK : ensure_single(ctx, 16, 16);
    if (st != YV_OK) return st;
    yv_batch* b = ctx->single;
    hipStream_t s = ctx->stream;
    const size_t nk = (size_t)b->max_kp;
    YV_HIP(stage_h2d(ctx, b->keypoints, q, sizeof(yv_keypoint) * (size_t)nq, s));
    if (nt > 0) YV_HIP(stage_h2d(ctx, b->keypoints + nk, t, sizeof(yv_keypoint) * (size_t)nt, s));
    ctx->h_pinned[0] = nq;
    ctx->h_pinned[1] = nt;
    YV_HIP(stage_h2d(ctx, b->kp_count, ctx->h_pinned, 2 * sizeof(int32_t), s));
    yavo::launch_pack_desc(b->keypoints, b->kp_count, 2, b->max_kp, b->desc, s);
    yavo::launch_match(b->desc, b->kp_count, b->pairs, 1, b->max_kp, nt, b->match_key, s);
    yavo::launch_match_finalize(b->match_key, b->keypoints, b->kp_count, b->pairs, 1, b->max_kp, 0, b->matches,
                                b->match_count, b->filtered, b->filt_count, b->match_dj, b->match_lim, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    YV_HIP(stage_d2h(ctx, out, b->matches, sizeof(yv_match) * (size_t)nq, s));
    YV_HIP(stage_sync(ctx, s));
    return YV_OK;
}

int yv_filter_matches(yv_ctx* ctx, const yv_match* in, int n, int thr, yv_match* out, int* n_out) {
    if (!ctx || !n_out || n < 0 || (n > 0 && (!in || !out))) return YV_ERR_INVALID;
    if (n > yavo::kMaxKp) return YV_ERR_CAPACITY;
    *n_out = 0;
    if (n == 0) return YV_OK;  // reference: minmax_element on an empty list is dereferenced (UB)
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    int st = ctx->single ? YV_OK : ensure_single(ctx, 16, 16);
    if (st != YV_OK) return st;
    yv_batch* b = ctx->single;
    hipStream_t s = ctx->stream;
    YV_HIP(stage_h2d(ctx, b->matches, in, sizeof(yv_match) * (size_t)n, s));
    yavo::launch_filter_records(b->matches, n, thr, b->filtered, b->filt_count, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    YV_HIP(stage_d2h(ctx, ctx->h_pinned, b->filt_count, sizeof(int32_t), s));
    YV_HIP(stage_sync(ctx, s));
    const int m = ctx->h_pinned[0];
    if (m > 0) {
        YV_HIP(stage_d2h(ctx, out, b->filtered, sizeof(yv_match) * (size_t)m, s));
        YV_HIP(stage_sync(ctx, s));
    }
    *n_out = m;
    return YV_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// geometry (include/yavo/yavo_geom.h)
// ------------------------------------------------------------------------------------------------
namespace {

// Carves 256-B aligned sub-buffers out of the context's device arena (grown on demand, outside any
// timed loop: the host-pointer calls are synchronous anyway).  The arena has a pinned host mirror with the same
// offsets: a call's inputs are copied into the mirror (`in`), one DMA moves the range they span (`upload`), and its
// outputs come back in one DMA of the range they span (`download`, then `finish` after the stream drained).  A
// host-pointer call is then two copies however many buffers it has (round 3: one staged copy per buffer, ~10 per
// LoopHandler frame).
//
// Regions added with add_host live in the pinned mirror itself and kernels address them there (zero-copy over PCIe):
// read-once inputs and the small outputs, which then need no DMA at all (a host call's outputs are a few hundred
// bytes to a few tens of KB; a DMA costs a copy-engine round trip each way).  Inputs the kernels read many times stay
// device regions.
struct Arena {
    yv_ctx* ctx;
    size_t need = 0;
    struct Req {
        void** p;
        size_t bytes;
        bool host;
    };
    std::vector<Req> reqs;
    size_t in_lo = SIZE_MAX, in_hi = 0, out_lo = SIZE_MAX, out_hi = 0;
    struct Out {
        void* dst;
        size_t off, bytes;
    };
    std::vector<Out> outs;
    std::vector<std::pair<size_t, size_t>> host_spans;  // [off, off + bytes) of every add_host region
    template <class T>
    void add(T** p, size_t count) {
        reqs.push_back({reinterpret_cast<void**>(p), count * sizeof(T), false});
        need += (count * sizeof(T) + 255) & ~(size_t)255;
    }
    template <class T>
    void add_host(T** p, size_t count) {
        reqs.push_back({reinterpret_cast<void**>(p), count * sizeof(T), true});
        need += (count * sizeof(T) + 255) & ~(size_t)255;
    }
    int commit() {
        if (need > ctx->scratch_cap) {
            if (ctx->scratch) (void)hipFree(ctx->scratch);
            if (ctx->scratch_h) (void)hipHostFree(ctx->scratch_h);
            ctx->scratch = nullptr;
            ctx->scratch_h = nullptr;
            ctx->scratch_cap = 0;
            size_t cap = std::max(need, (size_t)1 << 20);
            if (hipMalloc(&ctx->scratch, cap) != hipSuccess) return YV_ERR_HIP;
            void* hd = nullptr;
            // coherent (fine-grained) host memory: kernels read and write the host regions uncached, so nothing of a
            // previous call can be stale in the GPU's caches
            if (hipHostMalloc(reinterpret_cast<void**>(&ctx->scratch_h), cap,
                              hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
                hipHostGetDevicePointer(&hd, ctx->scratch_h, 0) != hipSuccess) {
                if (ctx->scratch_h) (void)hipHostFree(ctx->scratch_h);
                ctx->scratch_h = nullptr;
                return YV_ERR_HIP;
            }
            ctx->scratch_hd = static_cast<uint8_t*>(hd);
            ctx->scratch_cap = cap;
        }
        char* base = reinterpret_cast<char*>(ctx->scratch);
        size_t off = 0;
        host_spans.clear();
        for (auto& r : reqs) {
            *r.p = r.host ? static_cast<void*>(ctx->scratch_hd + off) : static_cast<void*>(base + off);
            if (r.host) host_spans.push_back({off, off + r.bytes});
            off += (r.bytes + 255) & ~(size_t)255;
        }
        return YV_OK;
    }
    bool is_host(const void* p) const {
        const uint8_t* q = static_cast<const uint8_t*>(p);
        return q >= ctx->scratch_hd && q < ctx->scratch_hd + ctx->scratch_cap;
    }
    size_t off_of(const void* p) const {
        return is_host(p) ? (size_t)(static_cast<const uint8_t*>(p) - ctx->scratch_hd)
                          : (size_t)(static_cast<const char*>(p) - static_cast<const char*>(ctx->scratch));
    }
    void in(const void* dev, const void* src, size_t bytes) {
        if (!bytes) return;
        const size_t o = off_of(dev);
        std::memcpy(ctx->scratch_h + o, src, bytes);
        if (is_host(dev)) return;  // read by the kernel where it is
        in_lo = std::min(in_lo, o);
        in_hi = std::max(in_hi, o + bytes);
    }
    // a pitched host image into a packed device image
    void in_2d(const void* dev, const uint8_t* src, size_t spitch, size_t width, size_t height) {
        if (!width || !height) return;
        const size_t o = off_of(dev);
        uint8_t* p = ctx->scratch_h + o;
        if (spitch == width) std::memcpy(p, src, width * height);
        else
            for (size_t r = 0; r < height; ++r) std::memcpy(p + r * width, src + r * spitch, width);
        in_lo = std::min(in_lo, o);
        in_hi = std::max(in_hi, o + width * height);
    }
    void out(void* dst, const void* dev, size_t bytes) {
        if (!bytes) return;
        const size_t o = off_of(dev);
        outs.push_back({dst, o, bytes});
        if (is_host(dev)) return;  // written by the kernel where it is
        out_lo = std::min(out_lo, o);
        out_hi = std::max(out_hi, o + bytes);
    }
    hipError_t upload(hipStream_t s) {
        if (in_hi <= in_lo) return hipSuccess;
        return hipMemcpyAsync(static_cast<char*>(ctx->scratch) + in_lo, ctx->scratch_h + in_lo, in_hi - in_lo,
                              hipMemcpyHostToDevice, s);
    }
    // one DMA over the span of the device outputs, unless a host region (written in place by the kernel) lies inside
    // it: then one DMA per device output, so the span's stale device bytes never land on those host results
    hipError_t download(hipStream_t s) {
        if (out_hi <= out_lo) return hipSuccess;
        bool split = false;
        for (const auto& h : host_spans) split |= h.first < out_hi && h.second > out_lo;
        if (!split)
            return hipMemcpyAsync(ctx->scratch_h + out_lo, static_cast<char*>(ctx->scratch) + out_lo,
                                  out_hi - out_lo, hipMemcpyDeviceToHost, s);
        for (const auto& o : outs) {
            bool host = false;
            for (const auto& h : host_spans) host |= o.off >= h.first && o.off < h.second;
            if (host) continue;
            hipError_t e = hipMemcpyAsync(ctx->scratch_h + o.off, static_cast<char*>(ctx->scratch) + o.off, o.bytes,
                                          hipMemcpyDeviceToHost, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // after the stream drained: the outputs into the caller's buffers
    void finish() {
        for (const auto& o : outs) std::memcpy(o.dst, ctx->scratch_h + o.off, o.bytes);
    }
    // download, wait, finish
    hipError_t fetch(hipStream_t s) {
        hipError_t e = download(s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess) finish();
        return e;
    }
};


}  // namespace

extern "C" {

int yv_f_ransac(yv_ctx* ctx, const yv_match* m, int n, const int32_t* samples, int iters, double thr, double F[9],
                int* max_inliers, int* found) {
    if (!ctx || !F || !max_inliers || !found || n < 0 || iters < 0 || (n > 0 && !m) || (iters > 0 && !samples))
        return YV_ERR_INVALID;
    if (n > yavo::kMaxKp) return YV_ERR_CAPACITY;
    *found = 0;
    if (n < 8) return YV_OK;  // "Not enough matches": false, F untouched (src/3DHandler.cc:154-156)
    for (int i = 0; i < 8 * iters; ++i)
        if (samples[i] < 0 || samples[i] >= n) return YV_ERR_INVALID;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    hipStream_t s = ctx->stream;
    Arena a{ctx};
    yv_match* dm;
    int32_t *dcnt, *dsmp, *dmax, *dfound;
    double* dF;
    uint8_t* dws;
    a.add(&dm, (size_t)n);  // every hypothesis' count reads the whole list: on the device
    a.add(&dws, yavo::f_ransac_ws_bytes(1, iters));
    a.add_host(&dcnt, 1);
    a.add_host(&dsmp, (size_t)std::max(8 * iters, 1));
    a.add_host(&dF, 9);
    a.add_host(&dmax, 1);
    a.add_host(&dfound, 1);
    if (a.commit() != YV_OK) return YV_ERR_HIP;
    a.in(dm, m, sizeof(yv_match) * (size_t)n);
    a.in(dcnt, &n, sizeof(int32_t));
    if (iters > 0) a.in(dsmp, samples, sizeof(int32_t) * 8 * (size_t)iters);
    a.in(dF, F, sizeof(double) * 9);  // untouched if iters == 0
    YV_HIP(a.upload(s));
    yavo::launch_f_ransac(dm, n, dcnt, 1, dsmp, 8 * (int64_t)iters, iters, thr, dF, dmax, dfound, dws, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    a.out(F, dF, sizeof(double) * 9);
    a.out(max_inliers, dmax, sizeof(int32_t));
    a.out(found, dfound, sizeof(int32_t));
    YV_HIP(a.fetch(s));
    return YV_OK;
}

int yv_triangulate(yv_ctx* ctx, const double pose_a[7], const double pose_b[7], const double K[9], const yv_match* m,
                   int n, double* Xw, uint8_t* ok, int* n_ok) {
    if (!ctx || !pose_a || !pose_b || !K || !n_ok || n < 0 || (n > 0 && (!m || !Xw || !ok))) return YV_ERR_INVALID;
    *n_ok = 0;
    if (n == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    hipStream_t s = ctx->stream;
    Arena a{ctx};
    yv_match* dm;
    double *dposes, *dK, *dX;
    uint8_t* dok;
    // every record, pose and output is read or written once: all in the pinned mirror, no DMA
    a.add_host(&dm, (size_t)n);
    a.add_host(&dposes, 14);
    a.add_host(&dK, 9);
    a.add_host(&dX, 3 * (size_t)n);
    a.add_host(&dok, (size_t)n);
    if (a.commit() != YV_OK) return YV_ERR_HIP;
    a.in(dm, m, sizeof(yv_match) * (size_t)n);
    a.in(dposes, pose_a, sizeof(double) * 7);
    a.in(dposes + 7, pose_b, sizeof(double) * 7);
    a.in(dK, K, sizeof(double) * 9);
    yavo::launch_triangulate(dm, n, dposes, dK, dX, dok, nullptr, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    a.out(Xw, dX, sizeof(double) * 3 * (size_t)n);
    a.out(ok, dok, (size_t)n);
    YV_HIP(a.fetch(s));
    int cnt = 0;
    for (int i = 0; i < n; ++i) cnt += ok[i] ? 1 : 0;
    *n_ok = cnt;
    return YV_OK;
}

int yv_world2camera(yv_ctx* ctx, const double* X, int n, const double pose[7], const double K[9], double* out) {
    if (!ctx || !pose || !K || n < 0 || (n > 0 && (!X || !out))) return YV_ERR_INVALID;
    if (n == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    hipStream_t s = ctx->stream;
    Arena a{ctx};
    double *dX, *dT, *dK, *dO;
    // one read and one write per point: all in the pinned mirror, no DMA
    a.add_host(&dX, 3 * (size_t)n);
    a.add_host(&dT, 7);
    a.add_host(&dK, 9);
    a.add_host(&dO, 3 * (size_t)n);
    if (a.commit() != YV_OK) return YV_ERR_HIP;
    a.in(dX, X, sizeof(double) * 3 * (size_t)n);
    a.in(dT, pose, sizeof(double) * 7);
    a.in(dK, K, sizeof(double) * 9);
    yavo::launch_world2camera(dX, n, dT, dK, dO, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    a.out(out, dO, sizeof(double) * 3 * (size_t)n);
    YV_HIP(a.fetch(s));
    return YV_OK;
}

static int pose_single(yv_ctx* ctx, const double* X, const double* uv, int n, const double* K, double* pose,
                       uint8_t* outlier, int* result, bool lm) {
    if (!ctx || !K || !pose || !result || n < 0 || (n > 0 && (!X || !uv)) || (lm && n > 0 && !outlier))
        return YV_ERR_INVALID;
    if (n > 4096) return YV_ERR_CAPACITY;
    if (!finite_pose(pose)) return YV_ERR_INVALID;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    hipStream_t s = ctx->stream;
    Arena a{ctx};
    int32_t *doff, *dres;
    double *dX, *duv, *dK, *dP;
    uint8_t* dout;
    a.add(&dX, 3 * (size_t)std::max(n, 1));  // read by every pass: on the device
    a.add(&duv, 2 * (size_t)std::max(n, 1));
    a.add_host(&doff, 2);                      // read once, or written once: in the pinned mirror
    a.add_host(&dK, 9);
    a.add_host(&dP, 7);
    a.add_host(&dout, (size_t)std::max(n, 1));
    a.add_host(&dres, 1);
    if (a.commit() != YV_OK) return YV_ERR_HIP;
    const int32_t off2[2] = {0, n};
    a.in(doff, off2, 2 * sizeof(int32_t));
    if (n > 0) {
        a.in(dX, X, sizeof(double) * 3 * (size_t)n);
        a.in(duv, uv, sizeof(double) * 2 * (size_t)n);
    }
    a.in(dK, K, sizeof(double) * 9);
    a.in(dP, pose, sizeof(double) * 7);
    YV_HIP(a.upload(s));
    if (lm) yavo::launch_pose_lm(doff, 1, dX, duv, dK, dP, dout, dres, s);
    else yavo::launch_pose_gn(doff, 1, dX, duv, dK, dP, dres, s);
    if (check_launch() != YV_OK) return YV_ERR_HIP;
    a.out(pose, dP, sizeof(double) * 7);
    if (lm && n > 0) a.out(outlier, dout, (size_t)n);
    a.out(result, dres, sizeof(int32_t));
    YV_HIP(a.fetch(s));
    return YV_OK;
}

int yv_pose_lm(yv_ctx* ctx, const double* X, const double* uv, int n, const double K[9], double pose[7],
               uint8_t* outlier, int* inliers) {
    return pose_single(ctx, X, uv, n, K, pose, outlier, inliers, true);
}

int yv_pose_gn(yv_ctx* ctx, const double* X, const double* uv, int n, const double K[9], double pose[7],
               int* iterations) {
    return pose_single(ctx, X, uv, n, K, pose, nullptr, iterations, false);
}

int yv_pose_lm_batch(yv_ctx* ctx, int n_problems, const int32_t* d_offsets, const double* d_X, const double* d_uv,
                     const double* d_K, double* d_poses, uint8_t* d_outlier, int32_t* d_inliers, void* stream) {
    if (!ctx || n_problems < 0 || (n_problems > 0 && (!d_offsets || !d_X || !d_uv || !d_K || !d_poses || !d_outlier ||
                                                      !d_inliers)))
        return YV_ERR_INVALID;
    if (n_problems == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
    yavo::launch_pose_lm(d_offsets, n_problems, d_X, d_uv, d_K, d_poses, d_outlier, d_inliers, s);
    return check_launch();
}

int yv_pose_gn_batch(yv_ctx* ctx, int n_problems, const int32_t* d_offsets, const double* d_X, const double* d_uv,
                     const double* d_K, double* d_poses, int32_t* d_iterations, void* stream) {
    if (!ctx || n_problems < 0 ||
        (n_problems > 0 && (!d_offsets || !d_X || !d_uv || !d_K || !d_poses || !d_iterations)))
        return YV_ERR_INVALID;
    if (n_problems == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
    yavo::launch_pose_gn(d_offsets, n_problems, d_X, d_uv, d_K, d_poses, d_iterations, s);
    return check_launch();
}

int yv_f_ransac_batch(yv_ctx* ctx, const yv_match* d_matches, int64_t list_stride, const int32_t* d_counts, int n_lists,
                      const int32_t* d_samples, int64_t sample_stride, int iters, double thr, double* d_F,
                      int32_t* d_max_inliers, int32_t* d_found, void* stream) {
    if (!ctx || n_lists < 0 || iters < 0 ||
        (n_lists > 0 && (!d_matches || !d_counts || !d_samples || !d_F || !d_max_inliers || !d_found)))
        return YV_ERR_INVALID;
    if (n_lists == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
    const size_t need = yavo::f_ransac_ws_bytes(n_lists, iters);
    if (need > ctx->fr_ws_cap) {  // grown outside any timed loop; earlier launches that use it have finished
        YV_HIP(hipDeviceSynchronize());
        if (ctx->fr_ws) (void)hipFree(ctx->fr_ws);
        ctx->fr_ws = nullptr;
        ctx->fr_ws_cap = 0;
        YV_HIP(hipMalloc(&ctx->fr_ws, need));
        ctx->fr_ws_cap = need;
    }
    yavo::launch_f_ransac(d_matches, list_stride, d_counts, n_lists, d_samples, sample_stride, iters, thr, d_F,
                          d_max_inliers, d_found, ctx->fr_ws, s);
    return check_launch();
}

// ------------------------------------------------------------------------------------------------
// cv::calcOpticalFlowPyrLK
// ------------------------------------------------------------------------------------------------
}  // extern "C"

struct yv_lk {
    yv_ctx* ctx = nullptr;
    int max_images = 0, H = 0, W = 0;
    int built_images = 0;  // n_images of the last yv_lk_build
    hipEvent_t built = nullptr;  // recorded after the last yv_lk_build's pyramid, on the stream it ran on
    yavo::LkParams P;
};

extern "C" {

int yv_lk_create(yv_ctx* ctx, int max_images, int H, int W, int win, int max_level, yv_lk** out) {
    if (!ctx || !out || max_images <= 0 || H < 1 || W < 1 || win < 3 || win > 22 || max_level < 0 ||
        max_level >= yavo::kLkMaxLevels || (int64_t)H * W >= (1ll << 31))
        return YV_ERR_INVALID;
    *out = nullptr;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    yv_lk* lk = new (std::nothrow) yv_lk();
    if (!lk) return YV_ERR_INVALID;
    lk->ctx = ctx;
    lk->max_images = max_images;
    lk->H = H;
    lk->W = W;
    yavo::LkParams& P = lk->P;
    P.win = win;
    P.h[0] = H;
    P.w[0] = W;
    // buildOpticalFlowPyramid: stop when the next level would be <= winSize in either dimension
    int levels = 0;
    for (int l = 0; l < max_level; ++l) {
        const int h = (P.h[l] + 1) / 2, w = (P.w[l] + 1) / 2;
        if (w <= win || h <= win) break;
        P.h[l + 1] = h;
        P.w[l + 1] = w;
        levels = l + 1;
    }
    P.levels = levels;
    int64_t off = 0, doff = 0;
    for (int l = 0; l <= levels; ++l) {
        P.ps[l] = (P.w[l] + 63) & ~63;
        P.ds[l] = (P.w[l] + 15) & ~15;
        if (l >= 1) {
            P.off[l] = off;
            off += ((int64_t)P.h[l] * P.ps[l] + 255) & ~(int64_t)255;
        }
    }
    doff = (int64_t)P.h[0] * P.ds[0] * 2;  // yv_lk_level's one-level derivative image (level 0 is the largest)
    P.pyr_pitch = std::max<int64_t>(off, 256);
    P.der_pitch = doff;
    if (dalloc(&P.pyr, (size_t)P.pyr_pitch * max_images) != YV_OK ||
        dalloc(&P.der, (size_t)P.der_pitch * sizeof(int16_t)) != YV_OK ||
        hipEventCreateWithFlags(&lk->built, hipEventDisableTiming) != hipSuccess) {
        if (P.pyr) (void)hipFree(P.pyr);
        if (P.der) (void)hipFree(P.der);
        lk->built = nullptr;
        delete lk;
        return YV_ERR_HIP;
    }
    *out = lk;
    return YV_OK;
}

void yv_lk_destroy(yv_lk* lk) {
    if (!lk) return;
    (void)hipSetDevice(lk->ctx->device);
    (void)hipDeviceSynchronize();
    if (lk->P.pyr) (void)hipFree(lk->P.pyr);
    if (lk->P.der) (void)hipFree(lk->P.der);
    if (lk->built) (void)hipEventDestroy(lk->built);
    delete lk;
}

int yv_lk_levels(const yv_lk* lk) { return lk ? lk->P.levels : YV_ERR_INVALID; }

int yv_lk_level(yv_lk* lk, int image, int level, const uint8_t** d_img, int* img_stride, const int16_t** d_deriv,
                int* deriv_stride, int* H, int* W) {
    if (!lk || !lk->P.img0 || image < 0 || image >= lk->built_images || level < 0 || level > lk->P.levels ||
        !d_img || !img_stride || !d_deriv || !deriv_stride || !H || !W)
        return YV_ERR_INVALID;
    if (set_device(lk->ctx) != YV_OK) return YV_ERR_HIP;
    const yavo::LkParams& P = lk->P;
    // the level's derivatives into the workspace's one-level image, complete on return.  The pyramid may have been
    // built on a caller stream (the batch's LK mode passes its track stream): wait for that build first
    if (hipStreamWaitEvent(lk->ctx->stream, lk->built, 0) != hipSuccess) return YV_ERR_HIP;
    yavo::launch_lk_derivs(P, image, level, P.der, lk->ctx->stream);
    if (check_launch() != YV_OK || hipStreamSynchronize(lk->ctx->stream) != hipSuccess) return YV_ERR_HIP;
    if (level == 0) {
        *d_img = P.img0 + image * P.pitch0;
        *img_stride = P.stride0;
    } else {
        *d_img = P.pyr + image * P.pyr_pitch + P.off[level];
        *img_stride = P.ps[level];
    }
    *d_deriv = P.der;
    *deriv_stride = P.ds[level];
    *H = P.h[level];
    *W = P.w[level];
    return YV_OK;
}

int yv_lk_build(yv_lk* lk, const uint8_t* d_images, int n_images, int stride, int64_t image_pitch, void* stream) {
    if (!lk || !d_images || n_images <= 0 || n_images > lk->max_images || stride < lk->W ||
        image_pitch < (int64_t)stride * (lk->H - 1) + lk->W)
        return YV_ERR_INVALID;
    if (set_device(lk->ctx) != YV_OK) return YV_ERR_HIP;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : lk->ctx->stream;
    lk->P.img0 = d_images;
    lk->P.stride0 = stride;
    lk->P.pitch0 = image_pitch;
    lk->built_images = n_images;
    yavo::launch_lk_pyramid(lk->P, n_images, s);
    if (check_launch() != YV_OK || hipEventRecord(lk->built, s) != hipSuccess) return YV_ERR_HIP;
    return YV_OK;
}

int yv_lk_track_batch(yv_lk* lk, const int32_t* d_pairs, int n_pairs, const float* d_pts, const int32_t* d_counts,
                      int pts_stride, int max_count, double eps, double min_eig, float* d_next, uint8_t* d_status,
                      float* d_err, void* stream) {
    if (!lk || !lk->P.img0 || n_pairs < 0 || pts_stride < 0 ||
        (n_pairs > 0 && (!d_pairs || !d_pts || !d_counts || !d_next || !d_status || !d_err)))
        return YV_ERR_INVALID;
    if (n_pairs == 0 || pts_stride == 0) return YV_OK;
    if (set_device(lk->ctx) != YV_OK) return YV_ERR_HIP;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : lk->ctx->stream;
    yavo::LkParams P = lk->P;
    // TermCriteria handling of SparsePyrLKOpticalFlowImpl: maxCount clipped to [0, 100], eps to [0, 10], squared
    P.max_count = std::min(std::max(max_count, 0), 100);
    const double e = std::min(std::max(eps, 0.), 10.);
    P.eps2 = e * e;
    P.min_eig = min_eig;
    yavo::launch_lk_track(P, d_pairs, n_pairs, d_pts, d_counts, pts_stride, pts_stride, d_next, d_status, d_err, s);
    return check_launch();
}

int yv_calc_optical_flow_pyr_lk(yv_ctx* ctx, const uint8_t* prev, const uint8_t* next, int H, int W, int stride,
                                const float* prev_pts, int n, int win, int max_level, int max_count, double eps,
                                double min_eig, float* next_pts, uint8_t* status, float* err) {
    if (!ctx || !prev || !next || n < 0 || (n > 0 && (!prev_pts || !next_pts || !status || !err)) || stride < W)
        return YV_ERR_INVALID;
    if (n > 65536) return YV_ERR_CAPACITY;
    if (n == 0) return YV_OK;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    const int64_t pitch = (int64_t)H * W;
    const int key[4] = {H, W, win, max_level};
    if (!ctx->lk_cache || !std::equal(key, key + 4, ctx->lk_key)) {
        if (ctx->lk_cache) yv_lk_destroy(ctx->lk_cache);
        ctx->lk_cache = nullptr;
        if (ctx->lk_img_d) (void)hipFree(ctx->lk_img_d);
        if (ctx->lk_img_h) (void)hipHostFree(ctx->lk_img_h);
        ctx->lk_img_d = ctx->lk_img_h = nullptr;
        ctx->lk_last = -1;
        int rc = yv_lk_create(ctx, 2, H, W, win, max_level, &ctx->lk_cache);
        if (rc != YV_OK) {
            ctx->lk_cache = nullptr;
            return rc;
        }
        if (hipMalloc(reinterpret_cast<void**>(&ctx->lk_img_d), (size_t)(2 * pitch + 64)) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&ctx->lk_img_h), (size_t)(2 * pitch)) != hipSuccess) {
            yv_lk_destroy(ctx->lk_cache);
            ctx->lk_cache = nullptr;
            if (ctx->lk_img_d) (void)hipFree(ctx->lk_img_d);
            ctx->lk_img_d = ctx->lk_img_h = nullptr;
            return YV_ERR_HIP;
        }
        std::copy(key, key + 4, ctx->lk_key);
    }
    yv_lk* lk = ctx->lk_cache;
    hipStream_t s = ctx->stream;
    // the image slots: prev is found in the slot the previous call left its next image in when the bytes are equal
    // (its pyramid is still in that slot too); otherwise both images go up and both pyramids are built
    auto same_image = [&](const uint8_t* img, const uint8_t* slot) {
        if (stride == W) return std::memcmp(img, slot, (size_t)pitch) == 0;
        for (int r = 0; r < H; ++r)
            if (std::memcmp(img + (size_t)r * stride, slot + (size_t)r * W, (size_t)W) != 0) return false;
        return true;
    };
    auto put_image = [&](const uint8_t* img, int slot) -> hipError_t {
        uint8_t* h = ctx->lk_img_h + slot * pitch;
        if (stride == W) std::memcpy(h, img, (size_t)pitch);
        else
            for (int r = 0; r < H; ++r) std::memcpy(h + (size_t)r * W, img + (size_t)r * stride, (size_t)W);
        return hipMemcpyAsync(ctx->lk_img_d + slot * pitch, h, (size_t)pitch, hipMemcpyHostToDevice, s);
    };
    // next goes to the slot the previous call's next is not in; its upload runs while prev is compared with that one
    const int ns = ctx->lk_last >= 0 ? 1 - ctx->lk_last : 1, ps = 1 - ns;
    const bool had = ctx->lk_last >= 0;
    ctx->lk_last = -1;  // until this call has completed
    if (put_image(next, ns) != hipSuccess) return YV_ERR_HIP;
    const bool reuse = had && same_image(prev, ctx->lk_img_h + ps * pitch);
    Arena a{ctx};
    float *dpts, *dnext, *derr;
    int32_t *dpair, *dcnt;
    uint8_t* dst;
    // points read once, outputs written once: in the pinned mirror (the images have their own slots)
    a.add_host(&dpts, 2 * (size_t)n);
    a.add_host(&dnext, 2 * (size_t)n);
    a.add_host(&derr, (size_t)n);
    a.add_host(&dpair, 2);
    a.add_host(&dcnt, 1);
    a.add_host(&dst, (size_t)n);
    if (a.commit() != YV_OK) return YV_ERR_HIP;
    const int32_t pair[3] = {ps, ns, n};
    a.in(dpts, prev_pts, sizeof(float) * 2 * n);
    a.in(dpair, pair, 2 * sizeof(int32_t));
    a.in(dcnt, pair + 2, sizeof(int32_t));
    if ((!reuse && put_image(prev, ps) != hipSuccess) || a.upload(s) != hipSuccess) return YV_ERR_HIP;
    yavo::LkParams& P = lk->P;
    P.img0 = ctx->lk_img_d;
    P.stride0 = W;
    P.pitch0 = pitch;
    lk->built_images = 2;
    if (reuse) {  // only the new image's pyramid (slot ns)
        yavo::LkParams P1 = P;
        P1.img0 = ctx->lk_img_d + ns * pitch;
        P1.pyr = P.pyr + ns * P.pyr_pitch;
        yavo::launch_lk_pyramid(P1, 1, s);
    } else {
        yavo::launch_lk_pyramid(P, 2, s);
    }
    if (check_launch() != YV_OK || hipEventRecord(lk->built, s) != hipSuccess) return YV_ERR_HIP;
    int status_rc = yv_lk_track_batch(lk, dpair, 1, dpts, dcnt, n, max_count, eps, min_eig, dnext, dst, derr, nullptr);
    if (status_rc != YV_OK) return status_rc;
    a.out(next_pts, dnext, sizeof(float) * 2 * n);
    a.out(status, dst, (size_t)n);
    a.out(err, derr, sizeof(float) * n);
    if (a.fetch(s) != hipSuccess) return YV_ERR_HIP;
    ctx->lk_last = ns;
    return YV_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// cv::findEssentialMat (RANSAC) + cv::recoverPose (yavo_geom.h)
// ------------------------------------------------------------------------------------------------
struct yv_essential {
    yv_ctx* ctx = nullptr;
    yavo::EssParams P;
};

namespace {
void essential_free(yv_essential* es) {
    if (!es) return;
    yavo::EssParams& P = es->P;
    void* ptrs[] = {P.m1, P.m2, P.idx, P.models, P.nmod, P.good, P.state, P.best, P.cand, P.cgood, P.rng_tab};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete es;
}
}  // namespace

extern "C" {

int yv_essential_create(yv_ctx* ctx, int max_pairs, int max_points, int max_iters, yv_essential** out) {
    if (!ctx || !out || max_pairs <= 0 || max_points < 5 || max_points > (1 << 20) || max_iters <= 0 ||
        max_iters > 100000)
        return YV_ERR_INVALID;
    *out = nullptr;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    yv_essential* es = new (std::nothrow) yv_essential();
    if (!es) return YV_ERR_INVALID;
    es->ctx = ctx;
    yavo::EssParams& P = es->P;
    P.max_pairs = max_pairs;
    P.max_points = max_points;
    P.max_iters = max_iters;
    P.chunk = yavo::ess_chunk_for(max_pairs);
    const size_t np = (size_t)max_pairs;
    if (dalloc(&P.m1, np * max_points * 2) != YV_OK || dalloc(&P.m2, np * max_points * 2) != YV_OK ||
        dalloc(&P.idx, np * max_iters * 5) != YV_OK || dalloc(&P.models, np * P.chunk * 90) != YV_OK ||
        dalloc(&P.nmod, np * P.chunk) != YV_OK || dalloc(&P.good, np * P.chunk * 10) != YV_OK ||
        dalloc(&P.state, np * 8) != YV_OK || dalloc(&P.best, np * 9) != YV_OK || dalloc(&P.cand, np * 48) != YV_OK ||
        dalloc(&P.cgood, np * 4) != YV_OK) {
        essential_free(es);
        return YV_ERR_HIP;
    }
    if (P.chunk == yavo::kEssChunkWide) {
        // cv::RNG((uint64)-1) states after 1 .. len draws: five per iteration plus room for the duplicate re-draws
        const int len = 5 * max_iters + 2048;
        std::vector<uint64_t> tab((size_t)len);
        uint64_t st = ~0ull;
        for (int k = 0; k < len; ++k) {
            st = (uint64_t)(uint32_t)st * 4164903690ull + (st >> 32);  // cv::RNG::next (CV_RNG_COEFF)
            tab[(size_t)k] = st;
        }
        if (dalloc(&P.rng_tab, (size_t)len) != YV_OK ||
            hipMemcpy(P.rng_tab, tab.data(), sizeof(uint64_t) * (size_t)len, hipMemcpyHostToDevice) != hipSuccess) {
            essential_free(es);
            return YV_ERR_HIP;
        }
        P.rng_len = len;
    }
    *out = es;
    return YV_OK;
}

void yv_essential_destroy(yv_essential* es) {
    if (!es) return;
    (void)hipSetDevice(es->ctx->device);
    (void)hipDeviceSynchronize();
    essential_free(es);
}

int yv_find_essential_batch(yv_essential* es, const float* d_pts1, const float* d_pts2, const int32_t* d_counts,
                            int n_pairs, int pts_stride, double focal, double ppx, double ppy, double prob,
                            double threshold, double* d_E, uint8_t* d_mask, int32_t* d_found, int32_t* d_stats,
                            void* stream) {
    if (!es || n_pairs < 0 || n_pairs > es->P.max_pairs || pts_stride < 0 || pts_stride > es->P.max_points ||
        (n_pairs > 0 && (!d_pts1 || !d_pts2 || !d_counts || !d_E || !d_found)) || !(focal != 0.0) ||
        !(prob > 0.0 && prob < 1.0))
        return YV_ERR_INVALID;
    if (n_pairs == 0) return YV_OK;
    if (set_device(es->ctx) != YV_OK) return YV_ERR_HIP;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : es->ctx->stream;
    // a list holds at most pts_stride (<= max_points) points: longer counts are clipped on the device
    yavo::EssRun r{focal, ppx, ppy, prob, threshold, es->P.max_iters};
    yavo::launch_find_essential(es->P, r, d_pts1, d_pts2, d_counts, n_pairs, pts_stride, d_E, d_mask, d_found,
                                d_stats, s);
    return check_launch();
}

int yv_recover_pose_batch(yv_essential* es, const double* d_E, const float* d_pts1, const float* d_pts2,
                          const int32_t* d_counts, int n_pairs, int pts_stride, const double K[9], double* d_R,
                          double* d_t, int32_t* d_good, void* stream) {
    if (!es || !K || n_pairs < 0 || n_pairs > es->P.max_pairs || pts_stride < 0 || pts_stride > es->P.max_points ||
        (n_pairs > 0 && (!d_E || !d_pts1 || !d_pts2 || !d_counts || !d_R || !d_t)) || !(K[0] != 0.0) ||
        !(K[4] != 0.0))
        return YV_ERR_INVALID;
    if (n_pairs == 0) return YV_OK;
    if (set_device(es->ctx) != YV_OK) return YV_ERR_HIP;
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : es->ctx->stream;
    yavo::Mat3 k;
    for (int i = 0; i < 9; ++i) k.v[i] = K[i];
    yavo::launch_recover_pose(es->P, d_E, d_pts1, d_pts2, d_counts, n_pairs, pts_stride, k, d_R, d_t, d_good, s);
    return check_launch();
}

// the context's cached one-list essential workspace with room for `points` points and `iters` RANSAC iterations
static int ctx_essential(yv_ctx* ctx, int points, int iters, yv_essential** out) {
    yv_essential* es = ctx->ess_cache;
    if (!es || es->P.max_points < points || es->P.max_iters < iters) {
        if (es) yv_essential_destroy(es);
        ctx->ess_cache = nullptr;
        const int rc = yv_essential_create(ctx, 1, std::max(points, 2048), std::max(iters, 1000), &ctx->ess_cache);
        if (rc != YV_OK) {
            ctx->ess_cache = nullptr;
            return rc;
        }
    }
    *out = ctx->ess_cache;
    return YV_OK;
}

int yv_find_essential(yv_ctx* ctx, const float* pts1, const float* pts2, int n, double focal, double ppx, double ppy,
                      double prob, double threshold, double E[9], uint8_t* mask, int* found) {
    if (!ctx || !E || !found || n < 0 || (n > 0 && (!pts1 || !pts2))) return YV_ERR_INVALID;
    if (n > 65536) return YV_ERR_CAPACITY;
    *found = 0;
    for (int i = 0; i < 9; ++i) E[i] = 0.0;
    if (n < 5) {
        if (mask)
            for (int i = 0; i < n; ++i) mask[i] = 0;
        return YV_OK;
    }
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    yv_essential* es = nullptr;
    int rc = ctx_essential(ctx, n, 1000, &es);
    if (rc != YV_OK) return rc;
    hipStream_t s = ctx->stream;
    Arena a{ctx};
    float *d1, *d2;
    double* dE;
    uint8_t* dm;
    int32_t *dcnt, *dfound;
    // the points are read once (ess_prepare_kernel normalises them into the workspace), the outputs written once: all
    // in the pinned mirror, no DMA
    a.add_host(&d1, 2 * (size_t)n);
    a.add_host(&d2, 2 * (size_t)n);
    a.add_host(&dE, 9);
    a.add_host(&dm, (size_t)n);
    a.add_host(&dcnt, 1);
    a.add_host(&dfound, 1);
    if (a.commit() != YV_OK) return YV_ERR_HIP;
    int st = YV_OK;
    do {
        a.in(d1, pts1, sizeof(float) * 2 * n);
        a.in(d2, pts2, sizeof(float) * 2 * n);
        a.in(dcnt, &n, sizeof(int32_t));
        if (a.upload(s) != hipSuccess) {
            st = YV_ERR_HIP;
            break;
        }
        st = yv_find_essential_batch(es, d1, d2, dcnt, 1, n, focal, ppx, ppy, prob, threshold, dE, dm, dfound,
                                     nullptr, nullptr);
        if (st != YV_OK) break;
        a.out(E, dE, sizeof(double) * 9);
        a.out(found, dfound, sizeof(int32_t));
        if (mask) a.out(mask, dm, (size_t)n);
        if (a.fetch(s) != hipSuccess) st = YV_ERR_HIP;
    } while (0);
    return st;
}

int yv_recover_pose(yv_ctx* ctx, const double E[9], const float* pts1, const float* pts2, int n, const double K[9],
                    double R[9], double t[3], int* good) {
    if (!ctx || !E || !K || !R || !t || !good || n < 0 || (n > 0 && (!pts1 || !pts2))) return YV_ERR_INVALID;
    if (n > 65536) return YV_ERR_CAPACITY;
    if (set_device(ctx) != YV_OK) return YV_ERR_HIP;
    StageScope stage_scope(ctx);
    yv_essential* es = nullptr;
    int rc = ctx_essential(ctx, std::max(n, 5), 1, &es);
    if (rc != YV_OK) return rc;
    hipStream_t s = ctx->stream;
    Arena a{ctx};
    float *d1, *d2;
    double *dE, *dR, *dt;
    int32_t *dcnt, *dgood;
    // each point is read by its four candidate lanes once: all in the pinned mirror, no DMA
    a.add_host(&d1, 2 * (size_t)std::max(n, 1));
    a.add_host(&d2, 2 * (size_t)std::max(n, 1));
    a.add_host(&dE, 9);
    a.add_host(&dR, 9);
    a.add_host(&dt, 3);
    a.add_host(&dcnt, 1);
    a.add_host(&dgood, 1);
    if (a.commit() != YV_OK) return YV_ERR_HIP;
    int st = YV_OK;
    do {
        if (n > 0) {
            a.in(d1, pts1, sizeof(float) * 2 * n);
            a.in(d2, pts2, sizeof(float) * 2 * n);
        }
        a.in(dE, E, sizeof(double) * 9);
        a.in(dcnt, &n, sizeof(int32_t));
        if (a.upload(s) != hipSuccess) {
            st = YV_ERR_HIP;
            break;
        }
        st = yv_recover_pose_batch(es, dE, d1, d2, dcnt, 1, std::max(n, 5), K, dR, dt, dgood, nullptr);
        if (st != YV_OK) break;
        a.out(R, dR, sizeof(double) * 9);
        a.out(t, dt, sizeof(double) * 3);
        a.out(good, dgood, sizeof(int32_t));
        if (a.fetch(s) != hipSuccess) st = YV_ERR_HIP;
    } while (0);
    return st;
}

}  // extern "C"
