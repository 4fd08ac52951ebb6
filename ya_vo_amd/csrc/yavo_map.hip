// yavo_map.hip -- the shared map (include/yavo/yavo_map.h): per-chunk blocks of keyframes
// and landmarks (the reference's Map::insertKeyFrame / insertMapPoint, src/Map.cc:9-40) built on the device after
// the chunk's pose LM, and their placement in world coordinates after the all-gather. Restated by
// oracle/yavo_oracle_map.c (or_map_chunk / or_map_place) expression for expression; built with -ffp-contract=off.
//
//   map_chain_kernel      one lane: L_k = L_{k-1} * rel_k over the chunk (Sophus products), the header and the
//                         keyframe records (global index % kf_every == 0)
//   map_landmarks_kernel  one 256-thread workgroup per keyframe: its LM inliers in edge order (ballot compaction)
//   map_anchor_kernel     one lane: A_0 = base, A_{r+1} = A_r * C_r over the gathered blocks; base <- A_world
//   map_place_kernel      one workgroup per (block, keyframe): T_wc = A_r * L_k, X_w = T_wc * X (a sequence shard's
//                         export, placed = 2: T_wc = A_r * T, X_w = A_r * X)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>

#include "../../include/yavo/yavo.h"
#include "../../include/yavo/yavo_map.h"
#include "yavo_internal.h"
#include "yavo_se3.h"

namespace yavo {
namespace map {

using se3::se3_act;
using se3::se3_mul;

constexpr int kNT = 256;
static_assert(sizeof(yv_map_header) == 128 && sizeof(yv_keyframe) == 72 && sizeof(yv_landmark) == 32,
              "block record layouts (ya_vo_amd/map.py dtypes)");

__host__ __device__ inline int64_t round256(int64_t x) { return (x + 255) & ~int64_t(255); }
__host__ __device__ inline int64_t kf_offset() { return (int64_t)sizeof(yv_map_header); }
__host__ __device__ inline int64_t lm_offset(int max_kf) {
    return round256(kf_offset() + (int64_t)max_kf * (int64_t)sizeof(yv_keyframe));
}
__host__ __device__ inline int64_t block_bytes(int max_kf, int lm_stride) {
    return round256(lm_offset(max_kf) + (int64_t)max_kf * lm_stride * (int64_t)sizeof(yv_landmark));
}

__global__ void map_chain_kernel(const double* rel, int n, int64_t first_frame, int kf_every, int lm_stride,
                                 int max_kf, uint8_t* block) {
    if (threadIdx.x != 0) return;
    yv_map_header* h = reinterpret_cast<yv_map_header*>(block);
    yv_keyframe* kf = reinterpret_cast<yv_keyframe*>(block + kf_offset());
    double L[7] = {0, 0, 0, 1, 0, 0, 0};
    int n_kf = 0;
    for (int k = 0; k < n; ++k) {
        double T[7];
        if (k == 0) {
            for (int i = 0; i < 7; ++i) T[i] = rel[i];
        } else {
            se3_mul(L, rel + 7 * k, T);
        }
        for (int i = 0; i < 7; ++i) L[i] = T[i];
        const int64_t g = first_frame + k;
        if (g % kf_every == 0 && n_kf < max_kf) {
            kf[n_kf].frame_id = g;
            for (int i = 0; i < 7; ++i) kf[n_kf].T[i] = L[i];
            kf[n_kf].n_landmarks = 0;
            kf[n_kf].pad = 0;
            ++n_kf;
        }
    }
    for (int i = 0; i < 7; ++i) h->chunk[i] = n > 0 ? L[i] : (i == 3 ? 1.0 : 0.0);
    h->first_frame = first_frame;
    h->n_frames = n;
    h->n_kf = n_kf;
    h->kf_every = kf_every;
    h->lm_stride = lm_stride;
    h->max_kf = max_kf;
    h->placed = 0;
    for (int i = 0; i < 5; ++i) h->pad[i] = 0.0;
}

// keyframe j's LM inliers, edge order kept: per 256 edges, wave ballots + LDS wave offsets
__global__ __launch_bounds__(kNT) void map_landmarks_kernel(const int32_t* edge_count, const double* edge_X,
                                                            const uint8_t* edge_outlier, int max_kp, uint8_t* block) {
    __shared__ int s_wave[kNT / 64];
    __shared__ int s_base;
    const yv_map_header* h = reinterpret_cast<const yv_map_header*>(block);
    const int j = blockIdx.x;
    if (j >= h->n_kf) return;
    yv_keyframe* kf = reinterpret_cast<yv_keyframe*>(block + kf_offset()) + j;
    yv_landmark* lm = reinterpret_cast<yv_landmark*>(block + lm_offset(h->max_kf)) + (int64_t)j * h->lm_stride;
    const int64_t g = kf->frame_id;
    const int k = (int)(g - h->first_frame);  // the track of this frame
    const int cnt = edge_count[k];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) s_base = 0;
    __syncthreads();
    for (int e0 = 0; e0 < cnt; e0 += kNT) {
        const int e = e0 + t;
        const bool keep = e < cnt && edge_outlier[(int64_t)k * max_kp + e] == 0;
        const unsigned long long m = __ballot(keep);
        if (lane == 0) s_wave[w] = __popcll(m);
        __syncthreads();
        int off = s_base;
        for (int q = 0; q < w; ++q) off += s_wave[q];
        off += __popcll(m & ((1ull << lane) - 1ull));
        if (keep) {
            const double* X = edge_X + ((int64_t)k * max_kp + e) * 3;
            lm[off].id = (g << 16) | (int64_t)e;
            lm[off].X[0] = X[0];
            lm[off].X[1] = X[1];
            lm[off].X[2] = X[2];
        }
        __syncthreads();
        if (t == 0) s_base += s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        __syncthreads();
    }
    if (t == 0) kf->n_landmarks = s_base;
}

__global__ void map_anchor_kernel(const uint8_t* blocks, int world, int64_t bb, double* base, double* anchors) {
    if (threadIdx.x != 0) return;
    double A[7];
    for (int i = 0; i < 7; ++i) A[i] = base[i];
    for (int r = 0; r < world; ++r) {
        const yv_map_header* h = reinterpret_cast<const yv_map_header*>(blocks + r * bb);
        for (int i = 0; i < 7; ++i) anchors[7 * r + i] = A[i];
        if (h->n_frames > 0) {
            double T[7];
            se3_mul(A, h->chunk, T);
            for (int i = 0; i < 7; ++i) A[i] = T[i];
        }
    }
    for (int i = 0; i < 7; ++i) base[i] = A[i];
}

// keyframes j = blockIdx.x, blockIdx.x + gridDim.x, ... of block blockIdx.y (n_kf is a device value; the grid is
// sized by the host to cover the usual count without launching a workgroup per possible keyframe)
__global__ __launch_bounds__(kNT) void map_place_kernel(uint8_t* blocks, int64_t bb, const double* anchors) {
    const int r = blockIdx.y;
    uint8_t* block = blocks + r * bb;
    yv_map_header* h = reinterpret_cast<yv_map_header*>(block);
    const int n_kf = h->n_kf;
    for (int j = blockIdx.x; j < n_kf; j += gridDim.x) {
        yv_keyframe* kf = reinterpret_cast<yv_keyframe*>(block + kf_offset()) + j;
        yv_landmark* lm = reinterpret_cast<yv_landmark*>(block + lm_offset(h->max_kf)) + (int64_t)j * h->lm_stride;
        double Lk[7], T[7], A[7];
        for (int i = 0; i < 7; ++i) Lk[i] = kf->T[i];
        for (int i = 0; i < 7; ++i) A[i] = anchors[7 * r + i];
        se3_mul(A, Lk, T);
        const int n = kf->n_landmarks;
        // a sequence shard's export (2, or 3 once a workgroup placed it -- other workgroups may read it after that
        // write): X_w = A_r X (the shard's own world frame)
        const bool shard_world = h->placed >= 2;
        __syncthreads();  // every lane has read L_k
        if (threadIdx.x == 0) {
            for (int i = 0; i < 7; ++i) kf->T[i] = T[i];
            if (j == 0) h->placed = shard_world ? 3 : 1;
        }
        for (int q = threadIdx.x; q < n; q += kNT) {
            double Xc[3] = {lm[q].X[0], lm[q].X[1], lm[q].X[2]}, Xw[3];
            se3_act(shard_world ? A : T, Xc, Xw);
            lm[q].X[0] = Xw[0];
            lm[q].X[1] = Xw[1];
            lm[q].X[2] = Xw[2];
        }
    }
}

}  // namespace map

void launch_map_chunk(const double* rel, int n, int64_t first_frame, int kf_every, const int32_t* edge_count,
                      const double* edge_X, const uint8_t* edge_outlier, int max_kp, int max_kf, void* block,
                      hipStream_t s) {
    uint8_t* blk = static_cast<uint8_t*>(block);
    hipLaunchKernelGGL(map::map_chain_kernel, dim3(1), dim3(64), 0, s, rel, n, first_frame, kf_every, max_kp, max_kf,
                       blk);
    hipLaunchKernelGGL(map::map_landmarks_kernel, dim3(max_kf), dim3(map::kNT), 0, s, edge_count, edge_X,
                       edge_outlier, max_kp, blk);
}

}  // namespace yavo

extern "C" int64_t yv_map_block_bytes(int max_kf, int lm_stride) {
    if (max_kf < 1 || lm_stride < 1) return -1;
    return yavo::map::block_bytes(max_kf, lm_stride);
}

extern "C" int yv_map_place(yv_ctx* ctx, void* d_blocks, int world, int64_t block_bytes, double* d_base,
                            double* d_anchors, void* stream) {
    if (!ctx || !d_blocks || world < 1 || block_bytes <= 0 || (block_bytes & 255) || !d_base || !d_anchors)
        return YV_ERR_INVALID;
    if (hipSetDevice(yavo::ctx_device(ctx)) != hipSuccess) return YV_ERR_HIP;
    // the header's max_kf (a device value) bounds the grid: the block size bounds it from above
    const int64_t per_kf = (int64_t)sizeof(yv_keyframe) + sizeof(yv_landmark);
    // (one workgroup per possible keyframe was up to 65535 mostly empty workgroups per block: 0.14 ms of dispatch for
    // a 1024-frame chunk's 256 keyframes; 512 covers that count in one pass and loops beyond it)
    const int grid_kf = (int)std::min<int64_t>(block_bytes / per_kf, 512);
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : yavo::ctx_stream(ctx);
    uint8_t* blk = static_cast<uint8_t*>(d_blocks);
    hipLaunchKernelGGL(yavo::map::map_anchor_kernel, dim3(1), dim3(64), 0, s, blk, world, block_bytes, d_base,
                       d_anchors);
    hipLaunchKernelGGL(yavo::map::map_place_kernel, dim3(grid_kf, world), dim3(yavo::map::kNT), 0, s, blk,
                       block_bytes, d_anchors);
    return hipGetLastError() == hipSuccess ? YV_OK : YV_ERR_HIP;
}
