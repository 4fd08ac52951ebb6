// yavo_kernels.hip -- gfx950 (CDNA4) kernels for the YA_VO detect / describe / match hot path.
//
// Built with -ffp-contract=off: the Harris eigen solve and response must round operation-for-operation
// like the reference's x86-64 build (no FMA contraction), see DESIGN.md "Float parity".
//
// Reference functions restated (file:line in /root/reference):
//   fast_harris_kernel  FastDetector::getFastFeatures loop      src/FastDetector.cc:298-335
//                       checkInBetween / checkContiguousPixels  src/FastDetector.cc:135-161
//                       preComputeHarris + Harris response      src/FastDetector.cc:164-214, 244-273
//   topk_kernel         std::sort + top-2000 cut                src/FastDetector.cc:343-368
//                       Brief::checkBoundry                     src/BriefDescriptor.cc:128-136
//   blur9_kernel        cv::GaussianBlur(9x9, 2.5) call         src/BriefDescriptor.cc:90
//   brief_kernel        Brief::computeBrief                     src/BriefDescriptor.cc:86-124
//   match_kernel        Brief::matchFeatures / hammingDistance  src/BriefDescriptor.cc:139-183
//   match_finalize      Matches records + removeOutliers        src/BriefDescriptor.cc:163-231
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "yavo_xlane.h"
#include "yavo_internal.h"


namespace yavo {

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Inclusive scan across one 64-lane wave, all in DPP (no LDS permutes): Hillis-Steele inside each 16-lane row
// (row_shr 1, 2, 4, 8; lanes without a source add the `old` 0), then row_bcast:15 adds row 0's total to row 1 and
// row 2's to row 3, and row_bcast:31 adds rows 0-1's total to rows 2 and 3 (GFX9 DPP).
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// Exclusive scan over the whole block (blockDim.x = NT, multiple of 64, <= 1024).  s_tmp >= 16 ints.
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* s_tmp, int* total) {
    const int lane = lane_id();
    const int wave = (int)threadIdx.x >> 6;
    constexpr int NW = NT / 64;
    int incl = wave_incl_scan(v);
    if (lane == 63) s_tmp[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        int w = lane < NW ? s_tmp[lane] : 0;
        int wi = wave_incl_scan(w);
        if (lane < NW) s_tmp[lane] = wi - w;  // exclusive wave offsets
        if (lane == NW - 1) s_tmp[NW] = wi;
    }
    __syncthreads();
    int res = s_tmp[wave] + incl - v;
    if (total) *total = s_tmp[NW];
    __syncthreads();
    return res;
}

// ------------------------------------------------------------------------------------------------
// FAST-12 + Harris
// ------------------------------------------------------------------------------------------------
// Ring order of FastDetector::getBresenhamCirclePoints (src/FastDetector.cc:50-112) as (drow, dcol);
// pinned by tests/test_oracle_fast.py against the reference's testBresenham.png fixture.
#define YV_RING_DR {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1}
#define YV_RING_DC {-3, -3, -2, -1, 0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3}

// OpenCV lapack.cpp hypot<float>: a*sqrt(1+(b/a)^2) (used by JacobiImpl_).
__device__ __forceinline__ float cv_hypotf(float a, float b) {
    a = fabsf(a);
    b = fabsf(b);
    if (a > b) {
        b /= a;
        return a * sqrtf(1.0f + b * b);
    }
    if (b > 0.0f) {
        a /= b;
        return b * sqrtf(1.0f + a * a);
    }
    return 0.0f;
}

// cv::eigen in an OpenCV built with HAVE_EIGEN: Eigen 3.4 SelfAdjointEigenSolver<MatrixXf> on the 2x2 (oracle
// or_eigen_selfadjoint2_f32 states the derivation): scale by the largest |entry|, implicit Wilkinson-shift QR steps
// until (e / FLT_EPSILON)^2 <= |d0| + |d1| (or |e| < FLT_MIN), at most 60; ascending sort, scale back.  Returns
// (w0 >= w1).  Every float operation in the oracle's order (-ffp-contract=off, IEEE div / sqrt).
__device__ __forceinline__ float eig_hypotf(float x, float y) {
    x = fabsf(x);
    y = fabsf(y);
    if (isinf(x) || isinf(y)) return __builtin_inff();
    if (isnan(x) || isnan(y)) return __builtin_nanf("");
    const float p = x > y ? x : y;
    if (p == 0.0f) return 0.0f;
    const float qp = (y < x ? y : x) / p;
    return p * sqrtf(1.0f + qp * qp);
}

__device__ void eig_selfadjoint2(float m00, float m01, float m11, float& w0, float& w1) {
    float scale = fabsf(m00);
    if (fabsf(m01) > scale) scale = fabsf(m01);
    if (fabsf(m11) > scale) scale = fabsf(m11);
    if (scale == 0.0f) scale = 1.0f;
    float d0 = m00 / scale, d1 = m11 / scale, e = m01 / scale;
    int iter = 0, ok = 1;
    while (true) {
        if (fabsf(e) < 1.17549435082228750797e-38f) {
            e = 0.0f;
        } else {
            const float se = 8388608.0f * e;
            if (se * se <= (fabsf(d0) + fabsf(d1))) e = 0.0f;
        }
        if (e == 0.0f) break;
        if (++iter > 60) { ok = 0; break; }
        const float td = (d0 - d1) * 0.5f;
        float mu = d1;
        if (td == 0.0f) {
            mu -= fabsf(e);
        } else {
            const float e2 = e * e;
            const float h = eig_hypotf(td, e);
            if (e2 == 0.0f) mu -= e / ((td + (td > 0.0f ? h : -h)) / e);
            else mu -= e2 / (td + (td > 0.0f ? h : -h));
        }
        const float x = d0 - mu, z = e;
        float c, sn;
        if (x == 0.0f) {  // makeGivens(x, z) with z != 0
            c = 0.0f;
            sn = z < 0.0f ? 1.0f : -1.0f;
        } else if (fabsf(x) > fabsf(z)) {
            const float t = z / x;
            float u = sqrtf(1.0f + t * t);
            if (x < 0.0f) u = -u;
            c = 1.0f / u;
            sn = -t * c;
        } else {
            const float t = x / z;
            float u = sqrtf(1.0f + t * t);
            if (z < 0.0f) u = -u;
            sn = -1.0f / u;
            c = -t * sn;
        }
        const float sdk = sn * d0 + c * e;
        const float dkp1 = sn * e + c * d1;
        const float nd0 = c * (c * d0 - sn * e) - sn * (c * e - sn * d1);
        const float nd1 = sn * sdk + c * dkp1;
        const float ne = c * sdk - sn * dkp1;
        d0 = nd0;
        d1 = nd1;
        e = ne;
    }
    if (ok && d1 < d0) { const float t = d0; d0 = d1; d1 = t; }
    d0 *= scale;
    d1 *= scale;
    w0 = d1;
    w1 = d0;
}

// cv::eigen on the 2x2 float structure tensor (eig = 0: JacobiImpl_<float>(n=2): one rotation unless
// |m01| <= FLT_EPSILON, then a descending sort; eig = 1: the HAVE_EIGEN solver above), followed by the response
// expression of src/FastDetector.cc:270 evaluated in double and rounded to float.
__device__ __forceinline__ float harris_response(float a, float b, float d, int eig) {
    float w0 = a, w1 = d;
    if (eig == 1) {
        eig_selfadjoint2(a, b, d, w0, w1);
    } else if (!(fabsf(b) <= 1.1920928955078125e-07f)) {
        const float p = b;
        const float y = (float)((double)(w1 - w0) * 0.5);
        float t = fabsf(y) + cv_hypotf(p, y);
        float s = cv_hypotf(p, t);
        // c = t / s is only used to rotate off-diagonal entries, none remain for n = 2
        s = p / s;
        t = (p / t) * p;
        if (y < 0.0f) { s = -s; t = -t; }
        w0 -= t;
        w1 += t;
    }
    if (eig != 1 && w0 < w1) { float tmp = w0; w0 = w1; w1 = tmp; }
    const float prod = w0 * w1;
    const float sum = w1 + w0;
    const double sq = (double)sum * (double)sum;
    const double r = (double)prod - 0.04 * sq;
    return (float)r;
}

// Order-preserving key: ascending key == (response descending, row-major index ascending).
__device__ __forceinline__ uint64_t make_key(float resp, uint32_t idx) {
    if (resp == 0.0f) resp = 0.0f;  // -0 and +0 compare equal in the reference's sort
    uint32_t u = __float_as_uint(resp);
    uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((uint64_t)(~ord) << 32) | (uint64_t)idx;
}
__device__ __forceinline__ float key_resp(uint64_t key) {
    uint32_t ord = ~(uint32_t)(key >> 32);
    uint32_t u = (ord & 0x80000000u) ? (ord & 0x7fffffffu) : ~ord;
    return __uint_as_float(u);
}

struct K9 {
    uint32_t k[9];
    // horizontal pass: output column j (0..3) of a 4-column item is dot4(d0, kh[j][0]) + dot4(d1, kh[j][1]) +
    // dot4(d2, kh[j][2]) over the row's 3 aligned LDS dwords d0..d2 (bytes 0..11): byte i of kh[j][m] is tap
    // 4m + i - j (0 outside 0..8), so no byte of the row is shifted or extracted in VALU
    uint32_t kh[4][3];
    // vertical pass over row-pair dwords P_t = {h[2m + 2t] (lo16), h[2m + 2t + 1] (hi16)}, t = 0..4:
    // even output row 2m = sum_t dot2(P_t, kve[t]), odd row 2m + 1 = sum_t dot2(P_t, kvo[t])
    uint32_t kve[5];  // (k0,k1) (k2,k3) (k4,k5) (k6,k7) (k8,0)
    uint32_t kvo[5];  // (0,k0) (k1,k2) (k3,k4) (k5,k6) (k7,k8)
    // sum of the taps <= 256: every rounded output (acc + 2^15) >> 16 is <= 255 and acc < 2^24, so the output byte
    // is byte 2 of the accumulator and needs no clamp (OpenCV's bit-exact kernels sum to exactly 256)
    int byte2;
    // horizontal pass on the int8 matrix cores (every tap <= 127): pixels enter as p - 128, so the sums are offset by
    // 128 * (sum of the taps), the accumulators' start value
    int mfma;
    int hbias;
};

static K9 make_k9(const uint16_t* k9) {
    K9 kw = {};
    uint32_t sum = 0;
    for (int i = 0; i < 9; ++i) {
        kw.k[i] = k9[i];
        sum += k9[i];
    }
    auto tap = [&](int t) -> uint32_t { return (t >= 0 && t <= 8) ? (uint32_t)k9[t] : 0u; };
    for (int j = 0; j < 4; ++j)
        for (int m = 0; m < 3; ++m)
            for (int i = 0; i < 4; ++i) kw.kh[j][m] |= tap(4 * m + i - j) << (8 * i);
    for (int t = 0; t < 5; ++t) {
        kw.kve[t] = tap(2 * t) | (tap(2 * t + 1) << 16);
        kw.kvo[t] = tap(2 * t - 1) | (tap(2 * t) << 16);
    }
    kw.byte2 = sum <= 256 ? 1 : 0;
    uint32_t mx = 0;
    for (int i = 0; i < 9; ++i) mx = k9[i] > mx ? k9[i] : mx;
    kw.mfma = mx <= 127 ? 1 : 0;
    kw.hbias = (int)(128 * sum);
    return kw;
}

__device__ __forceinline__ int reflect101(int p, int len) {
    // cv::borderInterpolate(BORDER_REFLECT_101); callers clamp p to [-(len-1), 2*len-2]
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - p - 2;
    return p;
}

// Fused per-tile detector: FAST-12 candidate test + Harris response (src/FastDetector.cc:298-335) and the
// 9x9 fixed-point Gaussian of the same tile (src/BriefDescriptor.cc:90), so the image is read from HBM
// once.  One 256-thread workgroup per 64 x 32 output tile, the tile plus a 4-pixel halo staged in LDS
// (BORDER_REFLECT_101 values outside the image: the blur needs them, no FAST candidate ever reads them).
// Candidates are staged in LDS and appended with ONE global atomic per workgroup.
// YAVO_LM_PROFILE builds (tools/det_profile.py): detect phase cycles of lane 0 of every workgroup, summed
#ifdef YAVO_LM_PROFILE
constexpr int kDetProfSlots = 131072;
__device__ unsigned long long g_det_prof[kDetProfSlots][6];
#define DP_DECL unsigned long long dp_acc[6] = {0, 0, 0, 0, 0, 0}; unsigned long long dp_t = __builtin_readcyclecounter();
#define DP_MARK(k) do { const unsigned long long t_ = __builtin_readcyclecounter(); dp_acc[k] += t_ - dp_t; dp_t = t_; } while (0)
#define DP_STORE() do { \
        const unsigned slot_ = blockIdx.x; \
        if (threadIdx.x == 0 && slot_ < kDetProfSlots) for (int q_ = 0; q_ < 6; ++q_) g_det_prof[slot_][q_] = dp_acc[q_]; \
    } while (0)
#else
#define DP_DECL
#define DP_MARK(k) do {} while (0)
#define DP_STORE() do {} while (0)
#endif
#ifdef YAVO_LM_PROFILE
constexpr int kBriefProfSlots = 16384;
__device__ unsigned long long g_brief_prof[kBriefProfSlots][6];
#define BP_DECL unsigned long long bp_acc[4] = {0, 0, 0, 0}; unsigned long long bp_t = __builtin_readcyclecounter(); \
    const unsigned long long bp_rt0 = __builtin_amdgcn_s_memrealtime();
#define BP_MARK(k) do { const unsigned long long t_ = __builtin_readcyclecounter(); bp_acc[k] += t_ - bp_t; bp_t = t_; } while (0)
#define BP_STORE() do { \
        if (threadIdx.x == 0 && blockIdx.x < kBriefProfSlots) { \
            g_brief_prof[blockIdx.x][0] = bp_acc[0] + bp_acc[1]; g_brief_prof[blockIdx.x][1] = bp_acc[2]; \
            g_brief_prof[blockIdx.x][2] = bp_rt0; \
            g_brief_prof[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime(); \
            g_brief_prof[blockIdx.x][4] = (unsigned long long)__builtin_amdgcn_s_getreg(0xF804); \
            g_brief_prof[blockIdx.x][5] = (unsigned long long)__builtin_amdgcn_s_getreg(0xF814); \
        } \
    } while (0)
#else
#define BP_DECL
#define BP_MARK(k) do {} while (0)
#define BP_STORE() do {} while (0)
#endif
constexpr int FT_W = kFastTileW;        // 64 output columns per tile (one wave-row)
constexpr int FT_H = kFastTileH;        // 56 output rows per tile
constexpr int FT_R = 4;                 // halo: blur radius 4 (ring radius 3, Sobel + 3x3 window radius 2)
constexpr int FT_LW = FT_W + 2 * FT_R;  // 72 bytes per LDS row
constexpr int FT_LH = FT_H + 2 * FT_R;  // 64 LDS rows

template <bool kBlur>
__global__ __launch_bounds__(256) void detect_kernel(const uint8_t* __restrict__ imgs, int H, int W, int stride,
                                                     int64_t pitch, int thr, int eig, uint64_t* __restrict__ cand_keys,
                                                     int64_t cap, uint32_t* __restrict__ cand_count, K9 kw,
                                                     uint8_t* __restrict__ blur) {
    __shared__ __align__(16) uint8_t tile[FT_LH * FT_LW];
    // the pretest survivors (phases 1-2) and the horizontal blur (from the barrier after phase 2) share LDS
    constexpr int kPreDw = FT_W * FT_H / 2, kHbufDw = kBlur ? (FT_LH / 2) * FT_W : 0;
    __shared__ __align__(16) uint32_t s_share[kPreDw > kHbufDw ? kPreDw : kHbufDw];
    uint16_t* s_pre = reinterpret_cast<uint16_t*>(s_share);
    uint32_t* hbuf = s_share;
    __shared__ uint16_t s_pos[FT_W * FT_H];
    __shared__ uint32_t s_n, s_npre, s_base;
    __shared__ uint32_t s_band[4 * 9];  // kh[r][M] at r * 9 + M + 3 for M in -3 .. 5 (0 outside 0 .. 2): the B operand
    DP_DECL
    // 1-D grid, XCD-aware: an image's tiles (and the halo rows neighbouring tiles share) stay in one XCD's L2
    const int ntx = (W + FT_W - 1) / FT_W, nty = (H + FT_H - 1) / FT_H;
    const int lb = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
    const int img = lb / (ntx * nty), tyx = lb - img * (ntx * nty);
    const int r0 = (tyx / ntx) * FT_H, c0 = (tyx % ntx) * FT_W;
    const uint8_t* src = imgs + (int64_t)img * pitch;
    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wave = tid >> 6;
    if (tid == 0) {
        s_n = 0;
        s_npre = 0;
    }
    if (kBlur && tid < 4 * 9) {
        const int r = tid / 9, M = tid - 9 * r - 3;
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int m = 0; m < 3; ++m)
                if (r == j && M == m) v = kw.kh[j][m];
        s_band[tid] = v;
    }

    // stage (FT_H + 8) x (FT_W + 8) = 64 x 72 bytes, one LDS dword per load: 5 per thread, all in flight before the
    // LDS writes.  Interior tiles (every source byte inside the image): each LDS dword is one unaligned dword load
    // (the hardware's unaligned mode splits it), no alignment arithmetic in VALU.  Border tiles (36% of a KITTI
    // image's 140 tiles): REFLECT_101 rows are whole source rows, so a dword whose 4 columns are inside the image is
    // still one dword load from the reflected row; only the dwords that cross the left / right edge gather their
    // 4 reflected columns byte by byte.
    {
        constexpr int kDw = FT_LW / 4;               // 18 LDS dwords per row
        constexpr int kSlots = FT_LH * kDw;          // 1152
        constexpr int kPer = (kSlots + 255) / 256;   // 5
        const bool interior = (c0 >= FT_R) && (c0 + FT_W + FT_R <= W) && (r0 >= FT_R) && (r0 + FT_H + FT_R < H);
        uint32_t v[kPer];
        if (interior) {
            // one wave-uniform base (SGPRs) and a 32-bit lane offset: slot t + 256 is 14 rows and 4 dwords on, or 15
            // rows and 14 dwords back when the dword index wraps past 18 (256 = 14 * 18 + 4), so one division for
            // the first slot and a compare + select + add for each further one (the same slots as the division form)
            const uint8_t* base = src + (int64_t)(r0 - FT_R) * stride + (c0 - FT_R);
            const int lr0 = tid / kDw, j0 = tid - lr0 * kDw;
            uint32_t off = (uint32_t)(lr0 * stride + 4 * j0);
            int j = j0;
            const uint32_t step = (uint32_t)(14 * stride + 16), wrap = (uint32_t)(15 * stride - 56);
            const uint32_t last = (uint32_t)((kSlots - 1) / kDw * stride + 4 * ((kSlots - 1) % kDw));
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                // slots past the tile (t >= kSlots, last pass only) read the last slot again; their store is skipped
                const uint32_t o = (256 * u + 255 >= kSlots && tid + 256 * u >= kSlots) ? last : off;
                __builtin_memcpy(&v[u], base + o, 4);
                const bool c = j + 4 >= kDw;
                off += c ? wrap : step;
                j += c ? 4 - kDw : 4;
            }
        } else {
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int t = min(tid + 256 * u, kSlots - 1);
                const int lr = t / kDw, j = t - lr * kDw;
                const int r = reflect101(min(max(r0 - FT_R + lr, -(H - 1)), 2 * H - 2), H);
                const uint8_t* row = src + (int64_t)r * stride;
                const int cc = c0 - FT_R + 4 * j;
                if (cc >= 0 && cc + 4 <= W) {
                    __builtin_memcpy(&v[u], row + cc, 4);
                } else {
                    uint32_t w = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        w |= (uint32_t)row[reflect101(min(max(cc + b, -(W - 1)), 2 * W - 2), W)] << (8 * b);
                    v[u] = w;
                }
            }
        }
        uint32_t* tile32 = reinterpret_cast<uint32_t*>(tile);
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int t = tid + 256 * u;
            if (t < kSlots) tile32[t] = v[u];
        }
    }
    __syncthreads();
    DP_MARK(0);

    constexpr int ring_dr[16] = YV_RING_DR;
    constexpr int ring_dc[16] = YV_RING_DC;
    const uint32_t neg_thr = (uint32_t)(-thr);
    // checkInBetween(cent, p) <=> cent > p - thr && cent < p + thr <=> |cent - p| - thr < 0: v_sad_u8 gives
    // |cent - p| + (-thr) in one instruction; its sign bit is "similar"
    // phase 1: the reference's pretest on ring pixels 0, 7 and (4 | 12) (src/FastDetector.cc:304-317) for
    // every pixel; each lane keeps a mask of its passing rows and the survivors are compacted into s_pre
    // once per wave (one scan, one LDS atomic)
    const int tx = lane;
    const int ty = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: the row bookkeeping below stays scalar
    const int c = c0 + tx;
    constexpr int kRowIters = FT_H / 4;
    // pixel (r, c) is tested iff 4 <= r < H - 4 and 4 <= c < W - 4: rows are wave-uniform, so the row test is one
    // scalar mask over the row iterations and the column test one compare
    uint32_t row_ok = 0;
#pragma unroll
    for (int u = 0; u < kRowIters; ++u) row_ok |= (uint32_t)((unsigned)(r0 + ty + 4 * u - 4) < (unsigned)(H - 8)) << u;
    // The reference's corner test is pre && run12 with pre = diff0 && diff7 && (diff4 || diff12)
    // (src/FastDetector.cc:304-317) and run12 = 12 consecutive "different" ring pixels without wrap
    // (checkContiguousPixels).  Any such run covers ring indices 4..11, so run12 implies diff7 and diff4, and
    // pre && run12 == diff0 && run12.  Phase 1 therefore filters on diff0 && diff4 && diff8 && diff11 (left, bottom,
    // right and top of the ring: a necessary condition, ~7% survivors against the pretest's ~18%) and phase 2
    // evaluates run12 exactly; the corner set is the reference's.
    // "similar" is the sign bit of sad(c, p) - thr, so the filter holds iff the sign bit of d0 | d4 | d8 | d11 is
    // clear; the sign bits are shifted into nmask (bit u = filtered out) with v_alignbit.  Every LDS read is one base
    // register (the 7 x 7 window's top-left of row iteration 0) plus a constant non-negative offset, so the
    // addresses cost no VALU.
    uint32_t nmask = 0;
    const uint8_t* wbase = &tile[(ty + FT_R - 3) * FT_LW + tx + FT_R - 3];
#pragma unroll
    for (int u = kRowIters - 1; u >= 0; --u) {
        const uint8_t* t0 = wbase + 4 * u * FT_LW;
        const uint32_t cent = t0[3 * FT_LW + 3];
        auto d = [&](int k) {
            return __builtin_amdgcn_sad_u8(cent, (uint32_t)t0[(ring_dr[k] + 3) * FT_LW + ring_dc[k] + 3], neg_thr);
        };
        const uint32_t v = (d(0) | d(4)) | (d(8) | d(11));
        nmask = __builtin_amdgcn_alignbit(nmask, v, 31);  // (nmask << 1) | (v >> 31)
    }
    uint32_t pmask = (unsigned)(c - 4) < (unsigned)(W - 8) ? (~nmask & row_ok) : 0u;
    {
        // survivors (~1 per lane) compacted into s_pre: a loop over the set bits, not one masked store per row
        const int cnt = __popc(pmask);
        const int incl = wave_incl_scan(cnt);
        const int total = __shfl(incl, 63, 64);
        uint32_t base = 0;
        if (lane == 0 && total > 0) base = atomicAdd(&s_npre, (uint32_t)total);
        base = __shfl(base, 0, 64);
        uint32_t off = base + (uint32_t)(incl - cnt);
        while (pmask) {
            const int u = __builtin_ctz(pmask);
            s_pre[off++] = (uint16_t)((ty + 4 * u) * FT_W + tx);
            pmask &= pmask - 1;
        }
    }
    __syncthreads();
    DP_MARK(1);
    // phase 2: the full 16-pixel test (>= 12 consecutive "different" ring pixels, no wrap:
    // checkContiguousPixels) densely over the pretest survivors; corners are staged in s_pos
    const uint32_t npre = s_npre;
    for (uint32_t i0 = 0; i0 < npre; i0 += 256) {  // uniform trip count: the ballots below see whole waves
        const uint32_t i = i0 + tid;
        bool cand = false;
        int pos = 0;
        if (i < npre) {
            pos = s_pre[i];
            // the 7 x 7 window's top-left: every ring read is this base plus a constant non-negative offset
            const uint8_t* t0 = &tile[((pos >> 6) + FT_R - 3) * FT_LW + (pos & 63) + FT_R - 3];
            const uint32_t cent = t0[3 * FT_LW + 3];
            // similar bits in reverse ring order (bit 15 - k for ring pixel k), one v_alignbit each; a run of
            // 12 consecutive bits without wrap is the same test in either order
            uint32_t sim = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                sim = __builtin_amdgcn_alignbit(
                    sim, __builtin_amdgcn_sad_u8(cent, (uint32_t)t0[(ring_dr[k] + 3) * FT_LW + ring_dc[k] + 3], neg_thr),
                    31);
            const uint32_t mask = ~sim & 0xFFFFu;  // "different" ring pixels
            const uint32_t a2 = mask & (mask >> 1);
            const uint32_t a4 = a2 & (a2 >> 2);
            const uint32_t a8 = a4 & (a4 >> 4);
            const uint32_t a12 = a8 & (a4 >> 8);
            cand = a12 != 0u;
        }
        const uint64_t bal = __ballot(cand);
        if (bal == 0) continue;
        const int leader = __ffsll((long long)bal) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&s_n, (uint32_t)__popcll(bal));
        base = __shfl(base, leader, 64);
        if (cand) s_pos[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)pos;
    }
    __syncthreads();
    DP_MARK(2);
    const uint32_t n = s_n;
    // one global atomic per workgroup reserves the output range of this tile's corners
    if (tid == 0 && n > 0) s_base = atomicAdd(&cand_count[img], n);
    if (kBlur && kw.mfma) {
        // horizontal pass on the int8 matrix cores: the 64 x 64 h of the tile (all 64 LDS rows, the 64 output
        // columns) is 4 x 4 blocks of 16 x 16, block (rb, cb) = A (tile rows 16 rb .., LDS columns 16 cb .. 16 cb + 63,
        // as p - 128) x B (the banded taps: B[k][n] = tap(k - n)), one v_mfma_i32_16x16x64_i8 each, wave rb taking
        // row block rb.  Exact: |products| and sums are integers far inside i32, and the accumulators start at
        // 128 * sum(taps), so acc = sum_t tap(t) p[x + t] (<= 65280: 16 bits).  A lane (n, g) of K-block g holds
        // bytes 16 g .. 16 g + 15 of its row / column for A and B alike (the pairing is by K index, the same for
        // both); B's dword jj is kh[n & 3][4 g + jj - (n >> 2)] (0 outside 0 .. 2), read from s_band.  LDS columns
        // past 71 (cb = 3) meet zero taps.  Output lane (n, g) holds rows 4 g .. 4 g + 3 of column n: rows 4g, 4g + 1
        // pack into h row pair 8 rb + 2 g, as the vertical pass reads them.  VALU per wave: 4 x (4 xor + 2 packs)
        // where the v_dot4 form took ~60: detect alone 2.766 -> 2.743 ms (profiles/r06/c41).  The four lane groups'
        // row pairs share banks (4-way conflicts on these 8 stores); a 72-dword row-pair stride cost 1 KB of LDS and
        // the 8th workgroup per CU (2.92 ms), an XOR swizzle of the column groups cost the vertical pass more VALU than
        // the conflicts (2.82 ms; c42-c44).
        typedef int dt_v4i __attribute__((ext_vector_type(4)));
        const int n = lane & 15, g = lane >> 4;
        dt_v4i B;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int M = 4 * g + jj - (n >> 2);
            B[jj] = (M >= -3 && M <= 5) ? (int)s_band[(n & 3) * 9 + M + 3] : 0;
        }
        const dt_v4i C = {kw.hbias, kw.hbias, kw.hbias, kw.hbias};
        const int rb = ty;
        const uint8_t* arow = &tile[(16 * rb + n) * FT_LW + 16 * g];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            const uint2 lo = *reinterpret_cast<const uint2*>(arow + 16 * cb);
            const uint2 hi = *reinterpret_cast<const uint2*>(arow + 16 * cb + 8);
            const dt_v4i A = {(int)(lo.x ^ 0x80808080u), (int)(lo.y ^ 0x80808080u), (int)(hi.x ^ 0x80808080u),
                              (int)(hi.y ^ 0x80808080u)};
            const dt_v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, C, 0, 0, 0);
            const int q = 8 * rb + 2 * g, x = 16 * cb + n;
            hbuf[q * FT_W + x] = (uint32_t)acc[0] | ((uint32_t)acc[1] << 16);
            hbuf[(q + 1) * FT_W + x] = (uint32_t)acc[2] | ((uint32_t)acc[3] << 16);
        }
    } else if (kBlur) {
        // horizontal pass, exact: h = sum_j k_j * p[x + j] as two v_dot4_u32_u8 + one mad on the byte row
        // (rows start 4-byte aligned: FT_LW = 72).  h <= 255 * 256 fits 16 bits; rows 2q and 2q+1 are
        // packed into one dword so the vertical pass can use v_dot2_u32_u16.  One item = 4 adjacent
        // columns of a row pair: 3 LDS dwords per row feed all 4 outputs, one 16-B LDS store.
        const uint32_t* trow = reinterpret_cast<const uint32_t*>(tile);
        constexpr int kItems = (FT_LH / 2) * (FT_W / 4);
        for (int i = tid; i < kItems; i += 256) {
            const int q = i >> 4, xq = (i & 15) * 4;
            uint32_t hv[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t* wr = trow + ((2 * q + h) * FT_LW >> 2) + (xq >> 2);
                const uint32_t d0 = wr[0], d1 = wr[1], d2 = wr[2];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    uint32_t acc = __builtin_amdgcn_udot4(d0, kw.kh[j][0], 0u, false);
                    acc = __builtin_amdgcn_udot4(d1, kw.kh[j][1], acc, false);
                    hv[h][j] = __builtin_amdgcn_udot4(d2, kw.kh[j][2], acc, false);
                }
            }
            *reinterpret_cast<uint4*>(&hbuf[q * FT_W + xq]) =
                make_uint4(hv[0][0] | (hv[1][0] << 16), hv[0][1] | (hv[1][1] << 16), hv[0][2] | (hv[1][2] << 16),
                           hv[0][3] | (hv[1][3] << 16));
        }
    }
    __syncthreads();
    DP_MARK(3);
    // Harris response of every staged corner, one lane per corner (no divergence across FAST lanes);
    // consecutive lanes write consecutive keys
    if (n > 0) {
        uint64_t* out = cand_keys + (int64_t)img * cap + s_base;
        for (uint32_t i = tid; i < n; i += 256) {
            const int pos = s_pos[i];
            const int prr = pos >> 6, ptx = pos & 63;
            // the 5 x 5 patch's top-left: every read is this base plus a constant non-negative offset
            const uint8_t* t0 = &tile[(prr + FT_R - 2) * FT_LW + ptx + FT_R - 2];
            // Sobel Ix / Iy (3x3 correlation) at the 3x3 window around the corner, from the 5x5 patch.
            int sxx = 0, sxy = 0, syy = 0;
#pragma unroll
            for (int ii = -1; ii <= 1; ++ii) {
#pragma unroll
                for (int j = -1; j <= 1; ++j) {
                    const uint8_t* q = t0 + (ii + 2) * FT_LW + j + 2;
                    const int pmm = q[-FT_LW - 1], pm0 = q[-FT_LW], pmp = q[-FT_LW + 1];
                    const int p0m = q[-1], p0p = q[1];
                    const int ppm = q[FT_LW - 1], pp0 = q[FT_LW], ppp = q[FT_LW + 1];
                    const int gx = (pmp - pmm) + 2 * (p0p - p0m) + (ppp - ppm);
                    const int gy = (ppm - pmm) + 2 * (pp0 - pm0) + (ppp - pmp);
                    sxx += gx * gx;
                    sxy += gx * gy;
                    syy += gy * gy;
                }
            }
            // all partial sums are integers < 2^24: exact in float, as in the reference
            const float resp = harris_response((float)sxx, (float)sxy, (float)syy, eig);
            out[i] = make_key(resp, (uint32_t)((r0 + prr) * W + (c0 + ptx)));  // cap >= every pixel: in range
        }
    }
    DP_MARK(4);
    if (kBlur) {
        // vertical pass, exact u32: rows 2m and 2m+1 of columns xq..xq+3 from the row-pair dwords P_m .. P_{m+4}
        // (one 16-B LDS read per row pair); each row's 4 bytes go out as one dword store, so 16 lanes write a
        // tile row's 64-B segment of the 128-B aligned pitched image (columns past W land in the row padding)
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        const int bp = blur_pitch(W);
        uint8_t* dst = blur + (int64_t)img * H * bp;
        for (int i = tid; i < (FT_H / 2) * (FT_W / 4); i += 256) {
            const int m = i >> 4, xq = (i & 15) * 4;
            uint4 P[5];
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                // one ds_read_b128 per row pair: 16 lanes cover a row pair's 64 dwords (every bank once).  The
                // volatile access keeps it whole: otherwise the compiler splits it into ds_read2_b32 pairs at a
                // 4-dword lane stride, 4-way bank conflicts (SQ_LDS_BANK_CONFLICT ~240 cycles per wave, r03 counters)
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                typedef const volatile __attribute__((address_space(3))) u32x4 lds_u32x4;
                const u32x4 q = *(lds_u32x4*)(&s_share[(m + t) * FT_W + xq]);
                P[t] = make_uint4(q.x, q.y, q.z, q.w);
            }
            // accumulators start at 2^15 (the rounding term of (acc + 2^15) >> 16)
            uint32_t ev[4], od[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                auto col = [&](const uint4& q) { return j == 0 ? q.x : j == 1 ? q.y : j == 2 ? q.z : q.w; };
                uint32_t e = 1u << 15, o = 1u << 15;
#pragma unroll
                for (int t = 0; t < 5; ++t) {
                    e = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, col(P[t])), __builtin_bit_cast(us2, kw.kve[t]), e, false);
                    o = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, col(P[t])), __builtin_bit_cast(us2, kw.kvo[t]), o, false);
                }
                ev[j] = e;
                od[j] = o;
            }
            uint32_t w0, w1;
            if (kw.byte2) {
                // output byte = byte 2 of each accumulator: two v_perm pick them pairwise, one v_perm joins the pairs
                w0 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(ev[3], ev[2], 0x0c0c0602u),
                                           __builtin_amdgcn_perm(ev[1], ev[0], 0x0c0c0602u), 0x05040100u);
                w1 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(od[3], od[2], 0x0c0c0602u),
                                           __builtin_amdgcn_perm(od[1], od[0], 0x0c0c0602u), 0x05040100u);
            } else {
                w0 = w1 = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    w0 |= min(ev[j] >> 16, 255u) << (8 * j);
                    w1 |= min(od[j] >> 16, 255u) << (8 * j);
                }
            }
            const int r = r0 + 2 * m, c = c0 + xq;
            if (r < H) *reinterpret_cast<uint32_t*>(&dst[(int64_t)r * bp + c]) = w0;
            if (r + 1 < H) *reinterpret_cast<uint32_t*>(&dst[(int64_t)(r + 1) * bp + c]) = w1;
        }
    }
    DP_MARK(5);
    DP_STORE();
}

void launch_fast_harris(const uint8_t* imgs, int n_images, int H, int W, int stride, int64_t pitch,
                        int thr, int eig, uint64_t* cand_keys, int64_t cap, uint32_t* cand_count, hipStream_t s) {
    dim3 grid(((W + FT_W - 1) / FT_W) * ((H + FT_H - 1) / FT_H) * n_images);
    K9 kw = {};
    hipLaunchKernelGGL(detect_kernel<false>, grid, dim3(256), 0, s, imgs, H, W, stride, pitch, thr, eig, cand_keys,
                       cap, cand_count, kw, (uint8_t*)nullptr);
}

void launch_detect_blur(const uint8_t* imgs, int n_images, int H, int W, int stride, int64_t pitch, int thr,
                        int eig, uint64_t* cand_keys, int64_t cap, uint32_t* cand_count, const uint16_t* k9_host,
                        uint8_t* blur, hipStream_t s) {
    dim3 grid(((W + FT_W - 1) / FT_W) * ((H + FT_H - 1) / FT_H) * n_images);
    const K9 kw = make_k9(k9_host);
    hipLaunchKernelGGL(detect_kernel<true>, grid, dim3(256), 0, s, imgs, H, W, stride, pitch, thr, eig, cand_keys, cap,
                       cand_count, kw, blur);
}

// ------------------------------------------------------------------------------------------------
// 9x9 fixed-point Gaussian blur (OpenCV GaussianBlurFixedPoint<uint8_t, ufixedpoint16>)
// ------------------------------------------------------------------------------------------------
constexpr int BL_W = 64, BL_H = 32, BL_R = 4;
constexpr int BL_LW = BL_W + 2 * BL_R;  // 72
constexpr int BL_LH = BL_H + 2 * BL_R;  // 40

__global__ __launch_bounds__(256) void blur9_kernel(const uint8_t* __restrict__ imgs, int H, int W, int stride,
                                                    int64_t pitch, K9 kw, uint8_t* __restrict__ blur) {
    __shared__ uint8_t tin[BL_LH * BL_LW];
    __shared__ uint32_t th[BL_LH * BL_W];
    const int img = blockIdx.z;
    const int r0 = blockIdx.y * BL_H, c0 = blockIdx.x * BL_W;
    const uint8_t* src = imgs + (int64_t)img * pitch;
    const int tid = threadIdx.x;
    for (int i = tid; i < BL_LH * BL_LW; i += 256) {
        const int lr = i / BL_LW, lc = i - lr * BL_LW;
        const int r = reflect101(min(max(r0 - BL_R + lr, -(H - 1)), 2 * H - 2), H);
        const int c = reflect101(min(max(c0 - BL_R + lc, -(W - 1)), 2 * W - 2), W);
        tin[i] = src[(int64_t)r * stride + c];
    }
    __syncthreads();
    // horizontal: exact u32 sums (<= 255 * 256)
    for (int i = tid; i < BL_LH * BL_W; i += 256) {
        const int lr = i >> 6, lc = i & 63;
        const uint8_t* q = &tin[lr * BL_LW + lc];
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < 9; ++j) acc += kw.k[j] * (uint32_t)q[j];
        th[i] = acc;
    }
    __syncthreads();
    const int tx = tid & 63, ty = tid >> 6;
    const int c = c0 + tx;
    for (int rr = ty; rr < BL_H; rr += 4) {
        const int r = r0 + rr;
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) acc += kw.k[i] * th[(rr + i) * BL_W + tx];
        uint32_t v = (acc + (1u << 15)) >> 16;
        if (r < H && c < W) blur[(int64_t)img * blur_image_bytes(H, W) + (int64_t)r * blur_pitch(W) + c] = (uint8_t)(v > 255u ? 255u : v);
    }
}

void launch_blur9(const uint8_t* imgs, int n_images, int H, int W, int stride, int64_t pitch,
                  const uint16_t* k9_host, uint8_t* blur, hipStream_t s) {
    const K9 kw = make_k9(k9_host);
    dim3 grid((W + BL_W - 1) / BL_W, (H + BL_H - 1) / BL_H, n_images);
    hipLaunchKernelGGL(blur9_kernel, grid, dim3(256), 0, s, imgs, H, W, stride, pitch, kw, blur);
}

// ------------------------------------------------------------------------------------------------
// top-K selection + sort + checkBoundry compaction (one 1024-thread workgroup per image)
// ------------------------------------------------------------------------------------------------
constexpr int TK_NT = 1024;

// checkBoundry(kp.y=col, kp.x=row, W, H): 8 <= col <= W-8 and 8 <= row <= H-8.
__device__ __forceinline__ bool brief_boundary(int row, int col, int H, int W) {
    return !(col - 8 < 0 || col + 8 > W) && !(row - 8 < 0 || row + 8 > H);
}

// Compacts points 0..K-1 (rc_at(i) -> int2 {row, col}) to those inside checkBoundry, keeping order;
// kp_src[slot] = {row, col, id = input index, 0}.  Chunks of 4 * NT points, 4 consecutive per thread.  The kept
// points are also bucketed by BRIEF band (row / kBandRows): kp_band = {row, col, id, slot} grouped by band,
// band_off[b] = the first entry of band b, band_off[nb] = the count (nb = bands of H rows).  Inside a band the points
// are grouped by the LDS bank of their patch centre in brief_kernel's band layout (bank_classes(nb) classes), which
// deals each 32-lane group of its descriptor waves keypoints of distinct banks (any order inside a class).  A second
// pass recomputes the same flags and slots and places each point after its (band, class) counter.
__host__ __device__ constexpr int bank_classes(int nb) { return nb <= kBandCounters / 32 ? 32 : 1; }

template <int NT, class RcAt>
__device__ void boundary_compact(RcAt rc_at, int K, int H, int W, int32_t* kp_src, int32_t* kp_count,
                                 int32_t* kp_band, int32_t* band_off, int* s_tmp, int* s_band) {
    const int tid = threadIdx.x;
    const int nb = (H + kBandRows - 1) / kBandRows;
    const int C = bank_classes(nb), nbc = nb * C;
    const int LS = brief_lds_stride(W);
    // (band, class) of a point: the dword bank of its centre byte (row - r0 + 8) * LS + col in the band's LDS copy
    auto bucket = [&](int row, int col) -> int {
        const int band = row / kBandRows;
        const int cls = C == 1 ? 0 : ((((row - band * kBandRows + 8) * LS + col) >> 2) & 31);
        return band * C + cls;
    };
    for (int b = tid; b < nbc; b += NT) s_band[b] = 0;
    __syncthreads();
    int base = 0;
    for (int pass = 0; pass < 2; ++pass) {
        base = 0;
        for (int c0 = 0; c0 < K; c0 += 4 * NT) {
            int flags[4];
            int2 rcs[4];
            int cnt = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = c0 + tid * 4 + u;
                flags[u] = 0;
                rcs[u] = make_int2(0, 0);
                if (i < K) {
                    rcs[u] = rc_at(i);
                    flags[u] = brief_boundary(rcs[u].x, rcs[u].y, H, W) ? 1 : 0;
                }
                cnt += flags[u];
            }
            int total = 0;
            int off = base + block_excl_scan<NT>(cnt, s_tmp, &total);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = c0 + tid * 4 + u;
                if (flags[u]) {
                    const int bk = bucket(rcs[u].x, rcs[u].y);
                    if (pass == 0) {
                        reinterpret_cast<int4*>(kp_src)[off] = make_int4(rcs[u].x, rcs[u].y, i, 0);
                        atomicAdd(&s_band[bk], 1);
                    } else {
                        const int pos = atomicAdd(&s_band[bk], 1);
                        reinterpret_cast<int4*>(kp_band)[pos] = make_int4(rcs[u].x, rcs[u].y, i, off);
                    }
                    off++;
                }
            }
            base += total;
        }
        __syncthreads();
        if (pass == 0) {
            // (band, class) counts -> first entries (the second pass's cursors) and the band offsets table
            int acc = 0;
            for (int b0 = 0; b0 < nbc; b0 += NT) {
                const int j = b0 + tid;
                const int c = j < nbc ? s_band[j] : 0;
                int tot = 0;
                const int first = acc + block_excl_scan<NT>(c, s_tmp, &tot);
                if (j < nbc) {
                    s_band[j] = first;
                    if (j % C == 0) band_off[j / C] = first;
                }
                acc += tot;
            }
            if (tid == 0) band_off[nb] = acc;
        }
        __syncthreads();
    }
    if (tid == 0) *kp_count = base;
}

// top-K per image: one workgroup of NT threads per image.  512 threads: same-box A/B in the headline step (r03 c32,
// two runs each) 1024 -> 206.0k fps, 512 -> 209.7k, 256 -> 207.3k; in-step top-K 757 -> 488 us per dispatch (half
// the waves at each of its ~80 workgroup barriers, twice the per-thread work in the sort stages).
constexpr int TK_SEL_NT = 512;
static_assert(TK_SEL_NT >= 256 && TK_SEL_NT % 64 == 0, "the radix-select histogram scan uses the first 256 threads");
template <int NT>
__global__ __launch_bounds__(NT) void topk_kernel(const uint64_t* __restrict__ cand_keys, int64_t cap,
                                                     uint32_t* __restrict__ cand_count, uint32_t* __restrict__ cand_seen,
                                                     int H, int W, int max_kp, int keep, int32_t* __restrict__ det_rc,
                                                     float* __restrict__ det_resp, int32_t* __restrict__ det_count,
                                                     int32_t* __restrict__ kp_src, int32_t* __restrict__ kp_count,
                                                     int32_t* __restrict__ kp_band, int32_t* __restrict__ band_off) {
    __shared__ uint64_t s_keys[kMaxKp];
    __shared__ uint32_t s_hist[256];
    __shared__ int s_tmp[40];
    __shared__ int s_band[kBandCounters];
    __shared__ uint64_t s_prefix, s_mask;
    __shared__ int s_krem, s_done, s_n;

    const int img = blockIdx.x;
    const int tid = threadIdx.x;
    const uint64_t* keys = cand_keys + (int64_t)img * cap;
    int64_t C64 = (int64_t)cand_count[img];
    if (C64 > cap) C64 = cap;
    const int C = (int)C64;
    const int K = C < keep ? C : keep;
    __syncthreads();
    if (tid == 0) {
        cand_seen[img] = (uint32_t)C;  // corners before the cut, kept for the caller
        cand_count[img] = 0;           // consumed: ready for the next detection into this slot
    }
    int32_t* rc_out = det_rc + (int64_t)img * max_kp * 2;
    float* resp_out = det_resp + (int64_t)img * max_kp;

    if (K == 0) {  // no corners (or max_kp == 0): nothing to select
        const int nb = (H + kBandRows - 1) / kBandRows;
        for (int b = tid; b <= nb; b += NT) band_off[(int64_t)img * (kMaxBands + 1) + b] = 0;
        if (tid == 0) { det_count[img] = 0; kp_count[img] = 0; }
        return;
    }
    uint64_t sel_mask = 0, sel_prefix = ~0ull;  // selection: (key & sel_mask) <= sel_prefix
    if (C > K) {
        if (tid == 0) { s_prefix = 0; s_mask = 0; s_krem = K; s_done = 0; }
        __syncthreads();
        for (int shift = 56; shift >= 0; shift -= 8) {
            // state of the previous pass is read before the barrier that precedes any rewrite of it
            const uint64_t pm = s_mask, pp = s_prefix;
            const int krem = s_krem;
            if (tid < 256) s_hist[tid] = 0;
            __syncthreads();
            for (int i = tid; i < C; i += NT) {
                const uint64_t k = keys[i];
                if ((k & pm) == pp) atomicAdd(&s_hist[(k >> shift) & 255u], 1u);
            }
            __syncthreads();
            // find the bucket holding the krem-th smallest key (256-entry scan by the first 4 waves)
            int h = 0, incl = 0;
            if (tid < 256) {
                h = (int)s_hist[tid];
                incl = wave_incl_scan(h);
                if ((tid & 63) == 63) s_tmp[tid >> 6] = incl;
            }
            __syncthreads();
            if (tid < 256) {
                int base = 0;
                for (int w = 0; w < (tid >> 6); ++w) base += s_tmp[w];
                incl += base;
                if (incl >= krem && incl - h < krem) {
                    const int nk = krem - (incl - h);
                    s_prefix = pp | ((uint64_t)tid << shift);
                    s_mask = pm | (0xFFull << shift);
                    s_krem = nk;
                    s_done = (h == nk);
                }
            }
            __syncthreads();
            if (s_done) break;
        }
        sel_mask = s_mask;
        sel_prefix = s_prefix;
    }
    // collect the K selected keys into LDS (any order), pad to a power of two, bitonic sort
    if (tid == 0) s_n = 0;
    __syncthreads();
    for (int i = tid; i < C; i += NT) {
        const uint64_t k = keys[i];
        if ((k & sel_mask) <= sel_prefix) {
            const int p = atomicAdd(&s_n, 1);
            if (p < kMaxKp) s_keys[p] = k;
        }
    }
    __syncthreads();
    int P2 = 1;
    while (P2 < K) P2 <<= 1;
    for (int i = K + tid; i < P2; i += NT) s_keys[i] = ~0ull;
    __syncthreads();
    for (int size = 2; size <= P2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < (P2 >> 1); t += NT) {
                const int i = 2 * t - (t & (stride - 1));
                const int j = i + stride;
                const bool up = ((i & size) == 0);
                const uint64_t a = s_keys[i], b = s_keys[j];
                if ((a > b) == up) { s_keys[i] = b; s_keys[j] = a; }
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < K; i += NT) {
        const uint64_t k = s_keys[i];
        const uint32_t idx = (uint32_t)k;
        const int row = (int)(idx / (uint32_t)W), col = (int)(idx - (uint32_t)row * (uint32_t)W);
        rc_out[2 * i] = row;
        rc_out[2 * i + 1] = col;
        resp_out[i] = key_resp(k);
    }
    if (tid == 0) det_count[img] = K;
    const uint32_t Wu = (uint32_t)W;
    auto rc_from_lds = [&](int i) -> int2 {
        const uint32_t idx = (uint32_t)s_keys[i];
        const uint32_t row = idx / Wu;
        return make_int2((int)row, (int)(idx - row * Wu));
    };
    boundary_compact<NT>(rc_from_lds, K, H, W, kp_src + (int64_t)img * max_kp * 4, kp_count + img,
                         kp_band + (int64_t)img * max_kp * 4, band_off + (int64_t)img * (kMaxBands + 1), s_tmp, s_band);
}

__global__ __launch_bounds__(TK_NT) void kp_boundary_kernel(const int32_t* __restrict__ det_rc,
                                                            const int32_t* __restrict__ det_count, int H, int W,
                                                            int max_kp, int32_t* __restrict__ kp_src,
                                                            int32_t* __restrict__ kp_count, int32_t* __restrict__ kp_band,
                                                            int32_t* __restrict__ band_off) {
    __shared__ int s_tmp[40];
    __shared__ int s_band[kBandCounters];
    const int img = blockIdx.x;
    int K = det_count[img];
    if (K > max_kp) K = max_kp;
    const int32_t* rc = det_rc + (int64_t)img * max_kp * 2;
    auto rc_from_global = [&](int i) -> int2 { return make_int2(rc[2 * i], rc[2 * i + 1]); };
    boundary_compact<TK_NT>(rc_from_global, K, H, W, kp_src + (int64_t)img * max_kp * 4, kp_count + img,
                            kp_band + (int64_t)img * max_kp * 4, band_off + (int64_t)img * (kMaxBands + 1), s_tmp,
                            s_band);
}

void launch_topk(const uint64_t* cand_keys, int64_t cap, uint32_t* cand_count, uint32_t* cand_seen, int n_images,
                 int H, int W, int max_kp, int keep, int32_t* det_rc, float* det_resp, int32_t* det_count, int32_t* kp_src,
                 int32_t* kp_count, int32_t* kp_band, int32_t* band_off, hipStream_t s) {
    hipLaunchKernelGGL(topk_kernel<TK_SEL_NT>, dim3(n_images), dim3(TK_SEL_NT), 0, s, cand_keys, cap, cand_count,
                       cand_seen, H, W, max_kp, keep, det_rc, det_resp, det_count, kp_src, kp_count, kp_band, band_off);
}

void launch_kp_boundary(const int32_t* det_rc, const int32_t* det_count, int n_images, int H, int W, int max_kp,
                        int32_t* kp_src, int32_t* kp_count, int32_t* kp_band, int32_t* band_off, hipStream_t s) {
    hipLaunchKernelGGL(kp_boundary_kernel, dim3(n_images), dim3(TK_NT), 0, s, det_rc, det_count, H, W, max_kp,
                       kp_src, kp_count, kp_band, band_off);
}

// ------------------------------------------------------------------------------------------------
// BRIEF
// ------------------------------------------------------------------------------------------------

// One workgroup per (32-row band, image): the band's keypoints (rows [r0, r0 + 32)) read their 17 x 17
// patches from an LDS copy of the blurred rows [r0 - 8, r0 + 41) with row stride LS = brief_lds_stride(W) >= W + 1.
// The reference samples getPixelVal at the linear index (row + dr) * W + (col + dc) (src/BriefDescriptor.cc:
// 100-118, src/Image.cc:15-17).  checkBoundry keeps 8 <= row <= H - 8 and 8 <= col <= W - 8, and |dr|, |dc| <= 8
// (yv_set_brief_offsets), so a sample is pixel (row + dr, col + dc) except (a) col + dc == W, which wraps to the
// first pixel of the next row, and (b) any index past the image end (row + dr == H, or row + dr == H - 1 at
// col + dc == W), which the reference reads out of bounds (UB; both paths read 0).  The band therefore holds in
// LDS column W of each row the next row's first pixel, and zero rows past the image: every sample is then
// s_band[(row + dr - (r0 - 8)) * LS + col + dc] with no test.  Lanes = keypoints: a wave takes 64 keypoints and
// one quarter (64) of the tests, whose sample offsets are wave-uniform scalars (loff).
constexpr int BR_BAND = kBandRows;
constexpr int BR_ROWS = BR_BAND + 17;  // rows r0-8 .. r0+40 (the last one for the wrap of col + 8 == W)
// 16 waves share one staged band: the ~61 KB band limits a CU to 2 workgroups, so the workgroup is as wide as
// the 64-VGPR budget of 8 waves per SIMD allows
constexpr int BR_NT = 1024;
constexpr int BR_NW = BR_NT / 64;
// the band's keypoint records are loaded as 4 per thread (kq below): a band may hold every keypoint of the image.
// (A loop over any further records would lift this bound but takes the kernel from 46 to 64 VGPRs, and at <= 48 one
// BRIEF wave per SIMD still fits beside the side stream's two pose-LM waves: 2 x 232 of 512.)
static_assert(4 * BR_NT >= kMaxKp, "brief_kernel loads at most 4 * BR_NT band records");

__global__ __launch_bounds__(BR_NT) void brief_kernel(const uint8_t* __restrict__ blur, int H, int W,
                                                    const int32_t* __restrict__ kp_src,
                                                    const int32_t* __restrict__ kp_band,
                                                    const int32_t* __restrict__ band_off, int max_kp,
                                                    yv_keypoint* __restrict__ keypoints, Desc* __restrict__ desc,
                                                    const int2* __restrict__ loff) {
    // All of the workgroup's LDS is dynamic, from a 16-B aligned base: static __shared__ variables would precede the
    // dynamic region unpadded (16,388 B of them put the band at 4 mod 16), and the band's 16-B LDS-DMA and zero-word
    // stores then run off their natural alignment.  Layout: the band (BR_ROWS * LS bytes, LS a multiple of 16), this
    // band's keypoints packed (index << 16) | (col << 5) | (row - r0) (index < 4096, col < 2048, 32-row band), the
    // count (launch_brief sizes the region).
    extern __shared__ __attribute__((aligned(16))) uint8_t s_band[];
    uint32_t* s_list = reinterpret_cast<uint32_t*>(s_band + BR_ROWS * brief_lds_stride(W));
    int& s_n = *reinterpret_cast<int*>(s_list + kMaxKp);
    BP_DECL
    // 1-D grid, XCD-aware: neighbouring bands of an image (17 shared rows) stay in one XCD's L2
    const int nbands = (H + BR_BAND - 1) / BR_BAND;
    const int lb = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
    const int img = lb / nbands;
    const int band = lb - img * nbands;
    const int r0 = band * BR_BAND;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int4* src = reinterpret_cast<const int4*>(kp_src) + (int64_t)img * max_kp;
    // this band's keypoints, bucketed by top-K (kp_band {row, col, id, slot}, band_off): the workgroup reads its own
    // ~K / bands records, not the image's whole list
    const int32_t* bo = band_off + (int64_t)img * (kMaxBands + 1);
    const int lo = bo[band], nbk = bo[band + 1] - lo;
    const int4* kb = reinterpret_cast<const int4*>(kp_band) + (int64_t)img * max_kp + lo;
    // Every global load of the workgroup is issued up front: the band's keypoint records (<= 4096 = 4 per thread),
    // then the band itself by LDS-DMA (global_load_lds_dwordx4: word k of the band lands at s4[k] with no VGPR
    // destination; the LDS address is the wave's base + 16 x lane, and word k = tid + u BR_NT is lane-linear).  Staging
    // the band through registers held 16 VGPRs per thread across the loads: the kernel took 46, and beside two pose-LM
    // waves on a SIMD (2 x 168 of 512 registers) a 16-wave BRIEF workgroup fits only at <= 40.
    // (unconditional loads from a valid record -- the image's first when the band has none -- so no branch merge
    // waits for them before the band's loads are issued; lanes past nbk ignore theirs)
    int4 kq[4];
    const int4* kbv = nbk > 0 ? kb : reinterpret_cast<const int4*>(kp_band) + (int64_t)img * max_kp;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = u * BR_NT + tid;
        kq[u] = kbv[j < nbk ? j : 0];
    }
    // band: rows rb .. rb + BR_ROWS - 1 (rb = r0 - 8) of the pitched blurred image as 16-B words, LS bytes per row
    // (LS <= the pitch: inside the row); column W of row r is patched with pixel (r + 1, 0) (0 past the image), rows
    // outside [0, H) are zero
    const int bp = blur_pitch(W), LS = brief_lds_stride(W);
    const uint8_t* b = blur + (int64_t)img * H * bp;
    const int rb = r0 - 8;
    const int wpr = LS >> 4;              // 16-B words per LDS row
    const int nw = BR_ROWS * wpr;
    const int kw_fix = W >> 4;
    uint4* s4 = reinterpret_cast<uint4*>(s_band);
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    const int wbase = tid & ~63;
    // the zero words first: an LDS store issued while LDS-DMA loads are in flight waits for them all
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int k = tid + u * BR_NT;
        const int r = rb + k / wpr;
        if (k < nw && (r < 0 || r >= H)) s4[k] = make_uint4(0, 0, 0, 0);
    }
    uint32_t nx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int k = tid + u * BR_NT;
        const int j = k / wpr, q = k - j * wpr;
        const int r = rb + j;
        nx[u] = 0u;
        if (k < nw && r >= 0 && r < H) {
            __builtin_amdgcn_global_load_lds(b + (int64_t)r * bp + 16 * q, (lds_ptr_t)(s4 + wbase + u * BR_NT), 16, 0,
                                             0);
            if (q == kw_fix && r + 1 < H) nx[u] = (uint32_t)b[(int64_t)(r + 1) * bp];
        }
    }
    // every load is in flight: one wait for all of them (consumed earlier, the records were waited for one by one)
    __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) asm volatile("" : "+v"(kq[u].x), "+v"(kq[u].y), "+v"(kq[u].w), "+v"(nx[u]));
    // 1. this band's keypoints (any order: each keypoint's outputs go to its own slot)
    if (tid == 0) s_n = nbk;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = u * BR_NT + tid;
        if (j < nbk)
            s_list[j] = ((uint32_t)kq[u].w << 16) | ((uint32_t)kq[u].y << 5) | (uint32_t)(kq[u].x - r0);
    }
    // 2. column W of each row: the byte after the row's last pixel takes the next row's first pixel, written by the
    // lane whose LDS-DMA word holds it, after its own loads have landed
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int k = tid + u * BR_NT;
        const int j = k / wpr, q = k - j * wpr;
        const int r = rb + j;
        if (k < nw && q == kw_fix && r >= 0 && r < H) s_band[16 * k + (W & 15)] = (uint8_t)nx[u];
    }
    // wide images (W > 1320): the rest of the band, word by word through registers
    const int sh_fix = 8 * (W & 3), dw_fix = (W >> 2) & 3;
    for (int k = tid + 4 * BR_NT; k < nw; k += BR_NT) {
        const int j = k / wpr, q = k - j * wpr;
        const int r = rb + j;
        uint4 w = make_uint4(0, 0, 0, 0);
        if (r >= 0 && r < H) {
            w = reinterpret_cast<const uint4*>(b + (int64_t)r * bp)[q];
            if (q == kw_fix) {
                const uint32_t nxx = r + 1 < H ? (uint32_t)b[(int64_t)(r + 1) * bp] : 0u;
                const uint32_t m = ~(0xFFu << sh_fix);
                if (dw_fix == 0) w.x = (w.x & m) | (nxx << sh_fix);
                else if (dw_fix == 1) w.y = (w.y & m) | (nxx << sh_fix);
                else if (dw_fix == 2) w.z = (w.z & m) | (nxx << sh_fix);
                else w.w = (w.w & m) | (nxx << sh_fix);
            }
        }
        s4[k] = w;
    }
    __syncthreads();
    const int nb = s_n;
    BP_MARK(1);
    if (nb == 0) {
        BP_STORE();
        return;
    }
    // 3. descriptors, lanes = keypoints: wave item = (block of 64 keypoints, group g of 64 tests).  The tests'
    // offsets are wave-uniform (loff, scalar loads), so a test costs each lane two LDS byte reads, two address adds,
    // a subtraction and one v_alignbit that shifts the result bit in: 4 VALU per test and keypoint, against ~110
    // VALU of per-keypoint ballot / emit work per wave in the lanes = tests form.
    uint8_t* rec_b = reinterpret_cast<uint8_t*>(keypoints + (int64_t)img * max_kp);
    Desc* d_base = desc + (int64_t)img * max_kp;
    // s_list is grouped by the bank of the patch centre (boundary_compact's classes, ~G entries each): lane kd of the
    // dealt order takes entry (kd % 32) * G + kd / 32, so the 32 lanes of a group take entries G apart, about one per
    // class -- distinct banks for every test's uniform offset, up to a carry -- where neighbouring entries share one
    const int G = (nb + 31) >> 5;
    const int nitems = ((32 * G + 63) >> 6) * 4;
    // the item index in an SGPR (tid >> 6 is not known to be wave-uniform): loff then comes by scalar loads
    for (int item = __builtin_amdgcn_readfirstlane(wave); item < nitems; item += BR_NW) {
        const int g = item & 3, kd = (item >> 2) * 64 + lane;
        const int k = (kd & 31) * G + (kd >> 5);
        const bool act = (kd >> 5) < G && k < nb;
        const uint32_t e = s_list[act ? k : nb - 1];
        const int i = (int)(e >> 16), row = r0 + (int)(e & 31u), col = (int)((e >> 5) & 2047u);
        const int id = (act && g == 0) ? src[i].z : 0;
        const int la = (row - rb) * LS + col;
        const int2* lo = loff + 64 * g;
        uint32_t w[2] = {0u, 0u};
        // tests 64g + 63 down to 64g: w[h] = (w[h] << 1) | (p1 > p2), so bit j of w[h] is test 64g + 32h + j; eight
        // tests (16 LDS reads in flight) per iteration keep the lane within the 64 VGPRs of 8 waves per SIMD
#pragma unroll 1
        for (int c = 7; c >= 0; --c) {
            const int2* oc = lo + 8 * c;
            uint32_t acc = w[c >> 2];
#pragma unroll
            for (int j = 7; j >= 0; --j) {
                const int2 o = oc[j];
                const uint32_t p1 = s_band[la + o.x], p2 = s_band[la + o.y];
                acc = __builtin_amdgcn_alignbit(acc, p2 - p1, 31);  // p2 - p1 < 0 iff p1 > p2
            }
            if (c >= 4) w[1] = acc;
            else w[0] = acc;
        }
        if (act) {
            reinterpret_cast<uint2*>(d_base + i)[g] = make_uint2(w[0], w[1]);
            // the 48-B record {row, col, id, matched = 0, featVec[32], 3 pad bytes}: featVec bytes 8g .. 8g + 7 at
            // record byte 13 + 8g (byte, short, dword, byte: the natural alignments of 13 + 8g ...)
            uint8_t* r = rec_b + (int64_t)i * 48;
            if (g == 0) {
                reinterpret_cast<int32_t*>(r)[0] = row;
                reinterpret_cast<int32_t*>(r)[1] = col;
                reinterpret_cast<int32_t*>(r)[2] = id;
                r[12] = 0;
            }
            r[13 + 8 * g] = (uint8_t)w[0];
            *reinterpret_cast<uint16_t*>(r + 14 + 8 * g) = (uint16_t)(w[0] >> 8);
            *reinterpret_cast<uint32_t*>(r + 16 + 8 * g) = (w[0] >> 24) | (w[1] << 8);
            r[20 + 8 * g] = (uint8_t)(w[1] >> 24);
            if (g == 3) {
                r[45] = 0;
                *reinterpret_cast<uint16_t*>(r + 46) = 0;
            }
        }
    }
    BP_MARK(2);
    BP_STORE();
}

// the 256 tests' sample offsets in the band's LDS layout: loff[t] = {dr1 * LS + dc1, dr2 * LS + dc2}
__global__ void brief_loff_kernel(const int8_t* __restrict__ offsets, int LS, int2* __restrict__ loff) {
    const int t = threadIdx.x;
    const int8_t* o = offsets + 4 * t;
    loff[t] = make_int2((int)o[0] * LS + (int)o[1], (int)o[2] * LS + (int)o[3]);
}

void launch_brief(const uint8_t* blur, int n_images, int H, int W, const int8_t* offsets, const int32_t* kp_src,
                  const int32_t* kp_band, const int32_t* band_off, int max_kp, yv_keypoint* keypoints, Desc* desc,
                  int32_t* loff, bool new_loff, hipStream_t s) {
    dim3 grid(((H + BR_BAND - 1) / BR_BAND) * n_images);
    const size_t lds = (size_t)BR_ROWS * brief_lds_stride(W) + sizeof(uint32_t) * kMaxKp + 16;
    int2* lo = reinterpret_cast<int2*>(loff);
    if (new_loff) hipLaunchKernelGGL(brief_loff_kernel, dim3(1), dim3(256), 0, s, offsets, brief_lds_stride(W), lo);
    hipLaunchKernelGGL(brief_kernel, grid, dim3(BR_NT), lds, s, blur, H, W, kp_src, kp_band, band_off, max_kp,
                       keypoints, desc, lo);
}

__global__ void pack_desc_kernel(const yv_keypoint* __restrict__ keypoints, const int32_t* __restrict__ kp_count,
                                 int max_kp, Desc* __restrict__ desc) {
    const int slot = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kp_count[slot] || i >= max_kp) return;
    const uint8_t* rec = reinterpret_cast<const uint8_t*>(keypoints + (int64_t)slot * max_kp + i);
    Desc d;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        d.w[q] = (uint32_t)rec[13 + 4 * q] | ((uint32_t)rec[14 + 4 * q] << 8) | ((uint32_t)rec[15 + 4 * q] << 16) |
                 ((uint32_t)rec[16 + 4 * q] << 24);
    }
    desc[(int64_t)slot * max_kp + i] = d;
}

void launch_pack_desc(const yv_keypoint* keypoints, const int32_t* kp_count, int n_slots, int max_kp, Desc* desc,
                      hipStream_t s) {
    dim3 grid((max_kp + 255) / 256, n_slots);
    hipLaunchKernelGGL(pack_desc_kernel, grid, dim3(256), 0, s, keypoints, kp_count, max_kp, desc);
}

// ------------------------------------------------------------------------------------------------
// Brute-force Hamming matcher on the int8 matrix cores
// ------------------------------------------------------------------------------------------------
// With every descriptor bit b mapped to the int8 value 2b - 1 (+1 / -1), the dot product of two 256-bit
// descriptors is 256 - 2 * Hamming exactly, so a pair's whole distance matrix is an int8 GEMM
// (queries x 256) . (256 x trains) with int32 accumulation: v_mfma_i32_16x16x64_i8 computes a 16 x 16
// distance tile per K-step, four K-steps per tile.  Per query the first minimum (strict <, as
// Brief::matchFeatures) is the maximum of the key (dot << 16) | (0xFFFF - j): larger dot, then smaller j.
// A and B fragments place descriptor element k = 64 s + 16 (lane >> 4) + j in byte j of K-step s of
// their lane, for both operands alike, so the products pair matching bits whatever the hardware's k
// order inside an instruction is.
typedef int mm_v4i __attribute__((ext_vector_type(4)));
constexpr int MM_QT = 8;                  // 16-row query tiles per wave
constexpr int MM_QB = 4 * MM_QT * 16;     // queries per workgroup (4 waves)
constexpr int MM_TC = 128;                // train descriptors per LDS chunk
constexpr int MM_ROW = 17;                // uint4 per expanded train row (16 + 1 pad: conflict-free b128 reads)

// 4 descriptor bits -> 4 bytes of +1 (bit set) / -1 (bit clear), bit i in byte i
__device__ __forceinline__ uint32_t expand_pm1(uint32_t nib) {
    const uint32_t spread = (nib * 0x00204081u) & 0x01010101u;
    return ~(spread * 0xFEu);
}

__device__ __forceinline__ uint4 expand16_pm1(uint32_t bits) {
    return make_uint4(expand_pm1(bits & 0xF), expand_pm1((bits >> 4) & 0xF), expand_pm1((bits >> 8) & 0xF),
                      expand_pm1((bits >> 12) & 0xF));
}

__device__ __forceinline__ int desc_popcount(const Desc& d) {
    int c = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) c += __popc(d.w[w]);
    return c;
}

// Train lists above 2048 (up to kMaxKp; lists <= 2048 take the FP4 kernel below): the +-1 encoding, dot = 256 -
// 2 Hamming, key = (dot << 16) + 0xFFFF - j formed per element.
__global__ __launch_bounds__(256) void match_kernel(const Desc* __restrict__ desc, const int32_t* __restrict__ kp_count,
                                                    const int32_t* __restrict__ pairs, int max_kp,
                                                    uint32_t* __restrict__ match_key) {
    __shared__ uint4 s_t[2][MM_TC * MM_ROW];
    const int pair = blockIdx.y;
    const int qi = pairs[2 * pair], ti = pairs[2 * pair + 1];
    const int nq = kp_count[qi], nt = kp_count[ti];
    const int q0 = blockIdx.x * MM_QB;
    if (q0 >= nq) return;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int col = lane & 15, g = lane >> 4;
    const Desc* qd = desc + (int64_t)qi * max_kp;
    const uint32_t* tw = reinterpret_cast<const uint32_t*>(desc + (int64_t)ti * max_kp);

    // query fragments: tile qt row (lane & 15) = query q0 + 16 MM_QT wave + 16 qt + (lane & 15)
    mm_v4i A[MM_QT][4];
#pragma unroll
    for (int qt = 0; qt < MM_QT; ++qt) {
        const int q = q0 + 16 * MM_QT * wave + 16 * qt + col;
        const Desc d = qd[q < nq ? q : 0];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint32_t hi_mask = 0u - (uint32_t)(g >> 1);  // blend, not an index: keeps d in registers
            const uint32_t w = d.w[2 * s] ^ ((d.w[2 * s] ^ d.w[2 * s + 1]) & hi_mask);
            const uint32_t bits = (w >> (16 * (g & 1))) & 0xFFFFu;
            const uint4 e = expand16_pm1(bits);
            A[qt][s] = mm_v4i{(int)e.x, (int)e.y, (int)e.z, (int)e.w};
        }
    }
    int best[MM_QT][4];
#pragma unroll
    for (int qt = 0; qt < MM_QT; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) best[qt][r] = INT_MIN;

    // staging: thread -> (train tt = idx >> 4, 16-bit field u = idx & 15), kF fields per thread per chunk
    constexpr int kF = MM_TC * 16 / 256;  // 16-bit fields per thread per chunk
    uint32_t pre[kF];
    auto fetch = [&](int t0) {
#pragma unroll
        for (int k = 0; k < kF; ++k) {
            const int idx = tid + 256 * k, tt = idx >> 4, u = idx & 15;
            const int t = t0 + tt;
            pre[k] = t < nt ? tw[(int64_t)t * 8 + (u >> 1)] : 0u;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int k = 0; k < kF; ++k) {
            const int idx = tid + 256 * k, tt = idx >> 4, u = idx & 15;
            const uint32_t bits = (pre[k] >> (16 * (u & 1))) & 0xFFFFu;
            s_t[buf][tt * MM_ROW + u] = expand16_pm1(bits);
        }
    };
    if (nt > 0) {
        fetch(0);
        store(0);
    }
    int buf = 0;
    for (int t0 = 0; t0 < nt; t0 += MM_TC) {
        const bool more = t0 + MM_TC < nt;
        if (more) fetch(t0 + MM_TC);
        __syncthreads();
        // two 16-column train tiles per pass: four independent MFMA chains, and one v_max3 folds both tiles' keys
        // into the running maximum
#pragma unroll
        for (int tt0 = 0; tt0 < MM_TC; tt0 += 32) {
            if (t0 + tt0 >= nt) break;
            mm_v4i Ba[4], Bb[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const uint4 va = s_t[buf][(tt0 + col) * MM_ROW + 4 * s + g];
                const uint4 vb = s_t[buf][(tt0 + 16 + col) * MM_ROW + 4 * s + g];
                Ba[s] = mm_v4i{(int)va.x, (int)va.y, (int)va.z, (int)va.w};
                Bb[s] = mm_v4i{(int)vb.x, (int)vb.y, (int)vb.z, (int)vb.w};
            }
            // a column past nt (including the whole second tile at the end of the list) gets -2^30, below every
            // real key and above INT_MIN, so no per-element select and no branch are needed
            const int ja = t0 + tt0 + col, jb = ja + 16;
            {
                // key = (dot << 16) + bias: bias = 0xFFFF - j for a real train column
                const int bias_a = ja < nt ? 0xFFFF - ja : -(1 << 30);
                const int bias_b = jb < nt ? 0xFFFF - jb : -(1 << 30);
#pragma unroll
                for (int qt = 0; qt < MM_QT; qt += 2) {
                    mm_v4i a0 = {0, 0, 0, 0}, b0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0}, b1 = {0, 0, 0, 0};
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        a0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[qt][s], Ba[s], a0, 0, 0, 0);
                        b0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[qt][s], Bb[s], b0, 0, 0, 0);
                        a1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[qt + 1][s], Ba[s], a1, 0, 0, 0);
                        b1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[qt + 1][s], Bb[s], b1, 0, 0, 0);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        best[qt][r] = max(best[qt][r], max((int)(((uint32_t)a0[r] << 16) + (uint32_t)bias_a),
                                                           (int)(((uint32_t)b0[r] << 16) + (uint32_t)bias_b)));
                        best[qt + 1][r] = max(best[qt + 1][r],
                                              max((int)(((uint32_t)a1[r] << 16) + (uint32_t)bias_a),
                                                  (int)(((uint32_t)b1[r] << 16) + (uint32_t)bias_b)));
                    }
                }
            }
        }
        if (more) {
            store(buf ^ 1);  // the other buffer: last read before the barrier at the top of this chunk
            buf ^= 1;
        }
    }
    // per query row: max over the 16 lanes (train columns) of its lane group
#pragma unroll
    for (int qt = 0; qt < MM_QT; ++qt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int v = best[qt][r];
            v = max(v, xl::xor_row_i32<8>(v));  // DPP butterflies inside the 16-lane group (yavo_xlane.h)
            v = max(v, xl::xor_row_i32<4>(v));
            v = max(v, xl::xor_row_i32<2>(v));
            v = max(v, xl::xor_row_i32<1>(v));
            const int q = q0 + 16 * MM_QT * wave + 16 * qt + 4 * g + r;
            if (col == r && q < nq) {
                uint32_t key = 0xFFFFFFFFu;  // empty train set (nt >= 1 always leaves a real key in the row max)
                if (v != INT_MIN) {
                    const int dot = v >> 16;
                    const uint32_t d = (uint32_t)((256 - dot) >> 1);
                    const uint32_t jj = 0xFFFFu - ((uint32_t)v & 0xFFFFu);
                    key = (d << 16) | jj;
                }
                match_key[(int64_t)pair * max_kp + q] = key;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// The same matcher on the FP4 matrix cores (train lists <= 2048)
// ------------------------------------------------------------------------------------------------
// v_mfma_scale_f32_32x32x64_f8f6f4 with both operands FP4 (e2m1): every descriptor bit becomes the FP4 value b
// (nibble 0b0010 = 1.0, 0b0000 = 0) and both E8M0 block scales are 2^6, so every product is 4096 * a_k * b_k: exact.
// The accumulator is f32 and every partial sum an integer of magnitude < 2^22 (the chain starts from
// c_j = (2047 - j) - 2048 * popcount(b_j) + 2^21 and adds 4096 * popcount(a & b) <= 2^20), so every sum is exact in
// any order and the chain ends at the int8 kernel's key plus 2^21 exactly:
//   key' = 2048 * (pa - Hamming) + (2047 - j) + 2^21 >= 2^21 - 2^19.
// Every key' is a positive float (a train row past the list starts at 0 and, its staged descriptor being zero, stays
// 0), and positive floats order as their bit patterns, so the running maximum is v_max3_u32 on the raw bits (a float
// max would first canonicalise both MFMA results).
//
// Train descriptors are the A operand (rows), queries B (columns).  A 32 x 32 x 64 tile takes 32 cycles and holds
// the SIMD's vector issue for 8 of them, where the 16 x 16 x 128 form holds 8 of 16 (MI355X_MICROARCH.md), so the
// running maxima and the staging get 24 free issue cycles per MFMA instead of 8 (tools/mfma_fp4_probe.hip: both
// forms alone 0.91-0.96 of the FP4 peak at 3 waves per SIMD, their matcher loops without LDS 0.83-0.84; the kernel
// 1.48 -> 1.43 ms per 4096-pair step, profiles/r06/c12, c14).  With the train list on the rows, a lane's 16
// accumulators are 16 train descriptors of ONE query, so each query tile keeps one running maximum per lane (the two
// lane halves merge at the end), and the chain start C(row) = c_j is four ds_read_b128 of the staged c row per
// 32-train block, shared by every query tile of the wave (no broadcast moves).  Lane (n, h = lane >> 5) of a K-step s
// holds descriptor dword 2 s + h of its train row / query column, for A and B alike; inside a dword the nibble order
// is a fixed permutation of the bits (the same for A and B), so the products pair matching bits.
constexpr int MF_TC = 128;               // train descriptors per LDS chunk
constexpr int MF_ROW = 9;                // uint4 per expanded train row (8 + 1 pad)

// 32 descriptor bits -> 32 FP4 nibbles (1.0 / 0) in four dwords: bit 4i + k lands in bit 1 of nibble i of dword k,
// one mask per dword (and a shift for three of them): 7 VALU per descriptor dword, where spreading each byte
// with two v_mul_u32_u24 took 34
__device__ __forceinline__ uint4 expand32_fp4(uint32_t w) {
    constexpr uint32_t kBit1 = 0x22222222u;
    return make_uint4((w << 1) & kBit1, w & kBit1, (w >> 1) & kBit1, (w >> 2) & kBit1);
}

typedef int mf_v8i __attribute__((ext_vector_type(8)));
typedef float mf_v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ mf_v16f mfma_fp4_32(const mm_v4i& a, const mm_v4i& b, const mf_v16f& c) {
    // FP4 operands use 4 of the 8 operand registers (the backend narrows them); scales 133 = 2^(133-127) = 64
    const mf_v8i a8 = __builtin_shufflevector(a, a, 0, 1, 2, 3, -1, -1, -1, -1);
    const mf_v8i b8 = __builtin_shufflevector(b, b, 0, 1, 2, 3, -1, -1, -1, -1);
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 133, 0, 133);
}

// running maximum of the 16 keys' of one accumulator (positive floats: bit patterns order as the values)
__device__ __forceinline__ uint32_t max16_u32(uint32_t best, const mf_v16f& a) {
    auto u = [&](int i) { return __float_as_uint(a[i]); };
    const uint32_t m0 = max(u(0), max(u(1), u(2))), m1 = max(u(3), max(u(4), u(5)));
    const uint32_t m2 = max(u(6), max(u(7), u(8))), m3 = max(u(9), max(u(10), u(11)));
    const uint32_t m4 = max(u(12), max(u(13), u(14)));
    const uint32_t m5 = max(m0, max(m1, m2)), m6 = max(m3, max(m4, u(15)));
    return max(best, max(m5, m6));
}

template <int QT, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void match_fp4_kernel(
    const Desc* __restrict__ desc, const int32_t* __restrict__ kp_count, const int32_t* __restrict__ pairs, int max_kp,
    uint32_t* __restrict__ match_key) {
    constexpr int QB = 4 * QT * 32;  // queries per workgroup
    __shared__ uint4 s_t[2][MF_TC * MF_ROW];
    __shared__ float s_c[2][MF_TC];  // c_j = (2047 - j) - 2048 popcount(b_j) + 2^21, 0 past the list
    const int pair = blockIdx.y;
    const int qi = pairs[2 * pair], ti = pairs[2 * pair + 1];
    const int nq = kp_count[qi], nt = kp_count[ti];
    const int q0 = blockIdx.x * QB;
    if (q0 >= nq) return;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int n = lane & 31, h = lane >> 5;
    const uint32_t* qw = reinterpret_cast<const uint32_t*>(desc + (int64_t)qi * max_kp);
    const uint32_t* tw = reinterpret_cast<const uint32_t*>(desc + (int64_t)ti * max_kp);

    // query fragments: tile qt column n = query q0 + 32 QT wave + 32 qt + n; the lane loads only its own four dwords
    // (a whole-descriptor load with a lane-dependent pick went through scratch)
    mm_v4i B[QT][4];
    uint32_t raw[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int q = q0 + 32 * QT * wave + 32 * qt + n;
        const uint32_t* w = qw + (int64_t)(q < nq ? q : 0) * 8 + h;
#pragma unroll
        for (int s = 0; s < 4; ++s) raw[qt][s] = w[2 * s];
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint4 e = expand32_fp4(raw[qt][s]);
            B[qt][s] = mm_v4i{(int)e.x, (int)e.y, (int)e.z, (int)e.w};
        }
    uint32_t best[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) best[qt] = 0u;

    // staging: thread -> (train tt = idx >> 3, descriptor dword u = idx & 7), kF dwords per thread per chunk; train
    // tt's chain start c_j from the popcounts of its 8 dwords, summed over their 8 consecutive lanes by DPP (waves 0-1
    // re-reading the chunk's descriptors for it stalled the workgroup on those loads at every chunk)
    constexpr int kF = MF_TC * 8 / 256;
    uint32_t pre[kF];
    auto fetch = [&](int t0) {
#pragma unroll
        for (int k = 0; k < kF; ++k) {
            const int idx = tid + 256 * k, tt = idx >> 3, u = idx & 7;
            const int t = t0 + tt;
            pre[k] = t < nt ? tw[(int64_t)t * 8 + u] : 0u;
        }
    };
    auto store = [&](int buf, int t0) {
#pragma unroll
        for (int k = 0; k < kF; ++k) {
            const int idx = tid + 256 * k, tt = idx >> 3, u = idx & 7;
            s_t[buf][tt * MF_ROW + u] = expand32_fp4(pre[k]);
            uint32_t pc = __builtin_popcount(pre[k]);
            pc += xl::dpp<0xB1>(pc);
            pc += xl::dpp<0x4E>(pc);
            pc += xl::dpp<0x141>(pc);
            const int t = t0 + tt;
            if (u == 0) s_c[buf][tt] = t < nt ? (float)((2047 - t) - 2048 * (int)pc + (1 << 21)) : 0.f;
        }
    };
    if (nt > 0) {
        fetch(0);
        store(0, 0);
    }
    int buf = 0;
    for (int t0 = 0; t0 < nt; t0 += MF_TC) {
        const bool more = t0 + MF_TC < nt;
        if (more) fetch(t0 + MF_TC);
        __syncthreads();
#pragma unroll
        for (int tt0 = 0; tt0 < MF_TC; tt0 += 32) {
            if (t0 + tt0 >= nt) break;
            mm_v4i A[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const uint4 v = s_t[buf][(tt0 + n) * MF_ROW + 2 * s + h];
                A[s] = mm_v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
            }
            // C(row, :) = c of train tt0 + row; accumulator i is row 8 (i >> 2) + 4 h + (i & 3)
            mf_v16f C;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 c4 = *reinterpret_cast<const float4*>(&s_c[buf][tt0 + 8 * k + 4 * h]);
                C[4 * k] = c4.x;
                C[4 * k + 1] = c4.y;
                C[4 * k + 2] = c4.z;
                C[4 * k + 3] = c4.w;
            }
#pragma unroll
            for (int qt = 0; qt < QT; qt += 2) {
                mf_v16f a0 = mfma_fp4_32(A[0], B[qt][0], C);
                mf_v16f a1 = mfma_fp4_32(A[0], B[qt + 1][0], C);
#pragma unroll
                for (int s = 1; s < 4; ++s) {
                    a0 = mfma_fp4_32(A[s], B[qt][s], a0);
                    a1 = mfma_fp4_32(A[s], B[qt + 1][s], a1);
                }
                best[qt] = max16_u32(best[qt], a0);
                best[qt + 1] = max16_u32(best[qt + 1], a1);
            }
        }
        if (more) {
            store(buf ^ 1, t0 + MF_TC);  // the other buffer: last read before the barrier at the top of this chunk
            buf ^= 1;
        }
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        uint32_t v = best[qt];
        v = max(v, (uint32_t)__shfl_xor((int)v, 32, 64));  // the other lane half's 16 rows of each train block
        // the query's popcount: its expanded fragments hold one set bit per descriptor bit, half in each lane half
        int pa = 0;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int r = 0; r < 4; ++r) pa += __popc((uint32_t)B[qt][s][r]);
        pa += __shfl_xor(pa, 32, 64);
        const int q = q0 + 32 * QT * wave + 32 * qt + n;
        if (h == 0 && q < nq) {
            uint32_t key = 0xFFFFFFFFu;  // empty train set
            if (nt > 0) {
                const int iv = (int)__uint_as_float(v) - (1 << 21);
                const uint32_t d = (uint32_t)(pa - (iv >> 11));
                const uint32_t jj = 2047u - ((uint32_t)iv & 2047u);
                key = (d << 16) | jj;
            }
            match_key[(int64_t)pair * max_kp + q] = key;
        }
    }
}

namespace {
template <int QT, int WPE>
void launch_fp4(const Desc* desc, const int32_t* kp_count, const int32_t* pairs, int n_pairs, int max_kp,
                uint32_t* match_key, hipStream_t s) {
    constexpr int QB = 4 * QT * 32;
    dim3 grid((max_kp + QB - 1) / QB, n_pairs);
    hipLaunchKernelGGL((match_fp4_kernel<QT, WPE>), grid, dim3(256), 0, s, desc, kp_count, pairs, max_kp, match_key);
}
}  // namespace

void launch_match(const Desc* desc, const int32_t* kp_count, const int32_t* pairs, int n_pairs, int max_kp,
                  int max_train, uint32_t* match_key, hipStream_t s) {
    if (max_train > 2048) {
        dim3 grid((max_kp + MM_QB - 1) / MM_QB, n_pairs);
        hipLaunchKernelGGL(match_kernel, grid, dim3(256), 0, s, desc, kp_count, pairs, max_kp, match_key);
        return;
    }
    // FP4: 4 query tiles of 32 per wave, 3 waves per SIMD (168 VGPRs; 2 tiles at 4 waves per SIMD: 1.60 ms vs 1.43,
    // profiles/r06/c14)
    launch_fp4<4, 3>(desc, kp_count, pairs, n_pairs, max_kp, match_key, s);
}

// ------------------------------------------------------------------------------------------------
// Matches records + removeOutliers (one 1024-thread workgroup per pair)
// ------------------------------------------------------------------------------------------------
constexpr int FZ_NT = 1024;
constexpr int REC_DW = 25;  // 100-B Matches record = 25 dwords

__device__ __forceinline__ int block_min_int(int v, int* s_tmp) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
    const int wave = (int)threadIdx.x >> 6;
    if (lane_id() == 0) s_tmp[wave] = v;
    __syncthreads();
    int r = s_tmp[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = min(r, s_tmp[w]);
    __syncthreads();
    return r;
}

// removeOutliers limit: max(2*min_dist, thr) with the reference's int wrap-around.
__device__ __forceinline__ int outlier_limit(int min_d, int thr) {
    const int twice = (int)((uint32_t)min_d * 2u);
    return twice > thr ? twice : thr;
}

__global__ __launch_bounds__(FZ_NT) void match_finalize_kernel(
    uint32_t* __restrict__ match_key, const yv_keypoint* __restrict__ keypoints,
    const int32_t* __restrict__ kp_count, const int32_t* __restrict__ pairs, int max_kp, int thr,
    yv_match* __restrict__ matches, int32_t* __restrict__ match_count, yv_match* __restrict__ filtered,
    int32_t* __restrict__ filt_count, int2* __restrict__ match_dj, int32_t* __restrict__ match_lim,
    int32_t* __restrict__ kp_count_copy, int n_slots) {
    __shared__ int s_dist[kMaxKp];
    // the edge build's copy of the run's keypoint counts (the last writer of kp_count, top-K, ran before this kernel)
    if (kp_count_copy && blockIdx.x == 0)
        for (int i = (int)threadIdx.x; i < n_slots; i += FZ_NT) kp_count_copy[i] = kp_count[i];
    __shared__ int s_j[kMaxKp];
    __shared__ int s_pos[kMaxKp];
    __shared__ int s_tmp[40];
    const int pair = blockIdx.x;
    const int tid = threadIdx.x;
    const int qi = pairs[2 * pair], ti = pairs[2 * pair + 1];
    const int nq = kp_count[qi];
    uint32_t* keys = match_key + (int64_t)pair * max_kp;
    int local_min = 0x7fffffff;
    for (int i = tid; i < nq; i += FZ_NT) {
        const uint32_t k = keys[i];
        keys[i] = 0xFFFFFFFFu;  // consumed: ready for the next match into this pair slot
        const int d = (k == 0xFFFFFFFFu) ? 0x7fffffff : (int)(k >> 16);
        s_dist[i] = d;
        s_j[i] = (k == 0xFFFFFFFFu) ? -1 : (int)(k & 0xFFFFu);
        local_min = min(local_min, d);
    }
    const int min_d = block_min_int(local_min, s_tmp);
    const int lim = outlier_limit(min_d, thr);
    int flags[4], cnt = 0;
    int2* dj = match_dj + (int64_t)pair * max_kp;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid * 4 + u;
        flags[u] = (i < nq && s_dist[i] < lim) ? 1 : 0;
        cnt += flags[u];
        if (i < nq) dj[i] = make_int2(s_dist[i], s_j[i]);
    }
    int total = 0;
    int off = block_excl_scan<FZ_NT>(cnt, s_tmp, &total);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid * 4 + u;
        if (i < nq) s_pos[i] = flags[u] ? off : -1;
        off += flags[u];
    }
    __syncthreads();
    const uint32_t* qrec = reinterpret_cast<const uint32_t*>(keypoints + (int64_t)qi * max_kp);
    const uint32_t* trec = reinterpret_cast<const uint32_t*>(keypoints + (int64_t)ti * max_kp);
    uint32_t* out_all = reinterpret_cast<uint32_t*>(matches + (int64_t)pair * max_kp);
    uint32_t* out_f = reinterpret_cast<uint32_t*>(filtered + (int64_t)pair * max_kp);
    const int ndw = nq * REC_DW;
    // Branch-free record assembly: every lane issues one load per record dword from an address that is always
    // valid (query record dword f < 12; train record dword min(f - 12, 2) of train j, or of train 0 when j < 0; the
    // value is then selected), FZ_U dwords per thread with every load in flight before the stores.  A wave's 64
    // consecutive dwords span ~2.5 records, so per-field branches ran all three paths with a load wait in each
    // (0.83 -> 0.67 ms per 2048-frame step, profiles/r03/c54).
    constexpr int FZ_U = 4;
    for (int dw0 = tid; dw0 < ndw; dw0 += FZ_U * FZ_NT) {
        uint32_t v[FZ_U];
        int ii[FZ_U], ff[FZ_U];
#pragma unroll
        for (int u = 0; u < FZ_U; ++u) {
            const int dw = min(dw0 + u * FZ_NT, ndw - 1);
            const int i = dw / REC_DW, f = dw - i * REC_DW;
            const int j = s_j[i];
            const uint32_t* src = f < 12 ? qrec + (int64_t)i * 12 + f : trec + (int64_t)max(j, 0) * 12 + min(f - 12, 2);
            v[u] = *src;
            ii[u] = i;
            ff[u] = f;
        }
#pragma unroll
        for (int u = 0; u < FZ_U; ++u) {
            const int dw = dw0 + u * FZ_NT;
            if (dw >= ndw) break;
            const int i = ii[u], f = ff[u];
            uint32_t x = v[u];
            if (f == 11) x &= 0xFFu;                         // featVec[31]; the 3 pad bytes are always written as 0
            else if (f >= 12 && (f >= 15 || s_j[i] < 0)) x = 0;  // pt2: x, y, id of the train keypoint only
            if (f == 24) x = (uint32_t)s_dist[i];
            out_all[dw] = x;
            const int p = s_pos[i];
            if (p >= 0) {
                if (f == 3 || f == 15) x = (x & ~0xFFu) | 1u;  // matched = true on both copies
                out_f[(int64_t)p * REC_DW + f] = x;
            }
        }
    }
    if (tid == 0) {
        match_count[pair] = nq;
        filt_count[pair] = total;
        match_lim[pair] = lim;
    }
}

void launch_match_finalize(uint32_t* match_key, const yv_keypoint* keypoints, const int32_t* kp_count,
                           const int32_t* pairs, int n_pairs, int max_kp, int thr, yv_match* matches,
                           int32_t* match_count, yv_match* filtered, int32_t* filt_count, int2* match_dj,
                           int32_t* match_lim, hipStream_t s, int32_t* kp_count_copy, int n_slots) {
    hipLaunchKernelGGL(match_finalize_kernel, dim3(n_pairs), dim3(FZ_NT), 0, s, match_key, keypoints, kp_count,
                       pairs, max_kp, thr, matches, match_count, filtered, filt_count, match_dj, match_lim,
                       kp_count_copy, n_slots);
}

// removeOutliers over a caller-supplied Matches list (n <= kMaxKp), one workgroup.
__global__ __launch_bounds__(FZ_NT) void filter_records_kernel(const yv_match* __restrict__ in, int n, int thr,
                                                               yv_match* __restrict__ out,
                                                               int32_t* __restrict__ out_count) {
    __shared__ int s_pos[kMaxKp];
    __shared__ int s_tmp[40];
    const int tid = threadIdx.x;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(in);
    int local_min = 0x7fffffff;
    for (int i = tid; i < n; i += FZ_NT) local_min = min(local_min, (int)src[(int64_t)i * REC_DW + 24]);
    const int min_d = block_min_int(local_min, s_tmp);
    const int lim = outlier_limit(min_d, thr);
    int flags[4], cnt = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid * 4 + u;
        flags[u] = (i < n && (int)src[(int64_t)i * REC_DW + 24] < lim) ? 1 : 0;
        cnt += flags[u];
    }
    int total = 0;
    int off = block_excl_scan<FZ_NT>(cnt, s_tmp, &total);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid * 4 + u;
        if (i < n) s_pos[i] = flags[u] ? off : -1;
        off += flags[u];
    }
    __syncthreads();
    uint32_t* dst = reinterpret_cast<uint32_t*>(out);
    for (int dw = tid; dw < n * REC_DW; dw += FZ_NT) {
        const int i = dw / REC_DW;
        const int f = dw - i * REC_DW;
        const int p = s_pos[i];
        if (p < 0) continue;
        uint32_t v = src[dw];
        if (f == 3 || f == 15) v = (v & ~0xFFu) | 1u;
        dst[(int64_t)p * REC_DW + f] = v;
    }
    if (tid == 0) *out_count = total;
}

void launch_filter_records(const yv_match* in, int n, int thr, yv_match* out, int32_t* out_count, hipStream_t s) {
    hipLaunchKernelGGL(filter_records_kernel, dim3(1), dim3(FZ_NT), 0, s, in, n, thr, out, out_count);
}

}  // namespace yavo

#ifdef YAVO_LM_PROFILE
extern "C" int yv_debug_brief_prof(unsigned long long* out /* [16384][6] */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(yavo::g_brief_prof), sizeof(unsigned long long) * 16384 * 6) ==
                   hipSuccess ? 0 : -2;
}
extern "C" int yv_debug_det_prof(unsigned long long* out /* [131072][6] */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(yavo::g_det_prof), sizeof(unsigned long long) * 131072 * 6) ==
                   hipSuccess ? 0 : -2;
}
#endif

// yavo_xlane.h self-check (tests/test_gpu_xlane.py): rows 0-3 = lane ^ {1, 2, 4, 8} through the DPP butterflies;
// rows 4-5 / 6-7 = the permlane16 / permlane32 half exchange of (lo = lane, hi = 100 + lane).
namespace yavo {
__global__ void xlane_check_kernel(int32_t* out) {
    const int l = threadIdx.x;
    out[0 * 64 + l] = xl::xor_row_i32<1>(l);
    out[1 * 64 + l] = xl::xor_row_i32<2>(l);
    out[2 * 64 + l] = xl::xor_row_i32<4>(l);
    out[3 * 64 + l] = xl::xor_row_i32<8>(l);
    uint32_t a = (uint32_t)l, b = 100u + (uint32_t)l;
    xl::swap_halves<16>(a, b);
    out[4 * 64 + l] = (int32_t)a;
    out[5 * 64 + l] = (int32_t)b;
    a = (uint32_t)l;
    b = 100u + (uint32_t)l;
    xl::swap_halves<32>(a, b);
    out[6 * 64 + l] = (int32_t)a;
    out[7 * 64 + l] = (int32_t)b;
}
}  // namespace yavo

extern "C" int yv_debug_xlane(int32_t* d_out /* [8][64] */, void* stream) {
    if (!d_out) return -1;
    hipLaunchKernelGGL(yavo::xlane_check_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), d_out);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
