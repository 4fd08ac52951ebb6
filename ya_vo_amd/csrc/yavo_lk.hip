// yavo_lk.hip -- gfx950 kernels for cv::calcOpticalFlowPyrLK as the reference calls it (SURVEY.md 8f row 1;
// src/LoopHandler.cc:372-375: winSize 11x11, maxLevel 3, TermCriteria(COUNT+EPS, 30, 0.01), flags 0,
// minEigThreshold 0.001).  Restates OpenCV's lkpyramid.cpp (scalar path) like oracle/yavo_oracle_lk.c:
//
//   pyr_down_kernel   cv::pyrDown CV_8U, 5x5 [1 4 6 4 1]^2 / 256, BORDER_REFLECT_101 (exact integers); 4
//                     output pixels x 4 rows per lane, packed-u16 sums over aligned 16-byte source-row loads
//   scharr_kernel     calcSharrDeriv: int16 (dx, dy), REFLECT_101 rows / columns; 4 pixels x 4 rows per lane,
//                     one aligned 16-byte store per output row
//   lk_kernel         LKTrackerInvoker for every level of one point per 16-lane DPP row (4 points per wave):
//                     each lane owns an S x S task of the window (S = ceil(win / 4)); bilinear samples (14-bit
//                     weights, CV_DESCALE) straight from the level images (REFLECT_101 image border, zero
//                     derivative border) with 24-bit multiply-adds; window sums as float partials per lane then
//                     a row butterfly (the oracle's sum_mode 1) that leaves the sum in all 16 lanes, so every
//                     lane computes the same Newton step
//
// Built with -ffp-contract=off like the rest: each float op rounds as the oracle's.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "yavo_internal.h"

namespace yavo {
namespace lk {

__device__ __forceinline__ int refl(int p, int len) {
    // cv::borderInterpolate(BORDER_REFLECT_101) for |p| < 2 len (all callers)
    if (len == 1) return 0;
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - p - 2;
    return p;
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Both kernels split a level into interior lanes, which read their source columns straight from the row, and border
// lanes (x0 = 0 and x0 >= x1), whose columns reflect.  The interior covers output columns [4, x1) in workgroups of
// 4 waves x 256 columns; one extra workgroup column packs the border lanes 8 groups x 8 row bands per wave, so
// the reflection's byte loads never run in an interior wave (a border lane there would make the whole wave run
// both forms).  Inside a wave the source rows are uniform (the wave index comes through readfirstlane, so the row
// arithmetic is scalar), and so is each row's dword misalignment: x0 is a multiple of 4.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 pair(uint16_t lo, uint16_t hi) {
    u16x2 v = {lo, hi};
    return v;
}

constexpr int kBorderGroups = 8;  // border lanes per row band: x0 = 0 and up to 7 groups at the right

// ------------------------------------------------------------------------------------------------
// pyrDown: a lane makes output pixels x0 .. x0 + 3 of PD_R output rows from source columns 2 x0 - 2 .. 2 x0 + 8 of
// rows 2 oy - 2 .. 2 oy + 2.  Interior lanes: one aligned dwordx4 per source row, the bytes split into even / odd
// columns as packed u16 pairs (w & 0x00FF00FF, (w >> 8) & 0x00FF00FF), the vertical [1 4 6 4 1] as packed
// multiply-adds, the horizontal one on pairs of outputs (a sum of 16 bytes <= 65280 fits a u16 lane), rounding
// and the byte pack in three ops.  The 5x5 sum is exact in integers, so any order gives cv::pyrDown's bytes.
// ------------------------------------------------------------------------------------------------
constexpr int PD_TW = 256;

// interior x0 < pd_x1(W): 2 x0 + 13 < W, so the aligned 16 bytes of every source row stay inside it
__host__ __device__ __forceinline__ int pd_x1(int W) {
    const int xm = W >= 22 ? ((W - 14) / 2) & ~3 : 0;  // last interior x0
    return xm >= 4 ? xm + 4 : 4;
}

template <int PD_R>
__global__ __launch_bounds__(256) void pyr_down_kernel(const uint8_t* __restrict__ src, int H, int W, int sstride,
                                                       int64_t spitch, uint8_t* __restrict__ dst, int dstride,
                                                       int64_t dpitch) {
    constexpr int PD_SR = 2 * PD_R + 3;  // source rows per lane
    const int img = blockIdx.z;
    const int Hd = (H + 1) / 2, Wd = (W + 1) / 2;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x1 = pd_x1(W);
    const uint8_t* s = src + (int64_t)img * spitch;
    uint8_t* d = dst + (int64_t)img * dpitch;
    if (blockIdx.x != gridDim.x - 1) {
        const int x0 = 4 + blockIdx.x * PD_TW + lane * 4;
        const int oy0 = (blockIdx.y * 4 + wave) * PD_R;
        if (x0 >= x1 || oy0 >= Hd) return;
        const int c0 = 2 * x0 - 2;
        uint32_t raw[PD_SR][4];
        uint32_t mis[PD_SR];
#pragma unroll
        for (int r = 0; r < PD_SR; ++r) {
            const uint8_t* row = s + (int64_t)refl(min(2 * oy0 - 2 + r, 2 * H - 2), H) * sstride;
            mis[r] = ((uint32_t)(uintptr_t)row + 2u) & 3u;  // (row + c0) & 3, c0 = 6 mod 8
            __builtin_memcpy(raw[r], __builtin_assume_aligned(row + c0 - mis[r], 4), 16);
        }
        // vertical sums of even (e) / odd (o) columns: e[m] = column c0 + 4m, c0 + 4m + 2; o[m] = the next ones
        u16x2 ve[PD_R][3], vo[PD_R][3];
#pragma unroll
        for (int i = 0; i < PD_R; ++i)
#pragma unroll
            for (int m = 0; m < 3; ++m) ve[i][m] = vo[i][m] = pair(0, 0);
#pragma unroll
        for (int r = 0; r < PD_SR; ++r) {
            u16x2 e[3], o[3];
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                const uint32_t w = __builtin_amdgcn_alignbyte(raw[r][m + 1], raw[r][m], mis[r]);
                e[m] = as_u16x2(w & 0x00FF00FFu);
                o[m] = as_u16x2((w >> 8) & 0x00FF00FFu);
            }
#pragma unroll
            for (int i = 0; i < PD_R; ++i) {
                const int t = r - 2 * i;  // tap of source row r for output row i
                if (t < 0 || t > 4) continue;
                const uint16_t c = (t == 0 || t == 4) ? 1 : (t == 2 ? 6 : 4);
#pragma unroll
                for (int m = 0; m < 3; ++m) {
                    ve[i][m] += e[m] * pair(c, c);
                    vo[i][m] += o[m] * pair(c, c);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < PD_R; ++i) {
            const int oy = oy0 + i;
            if (oy >= Hd) break;
            // outputs (2p, 2p + 1): e[p] + 4 o[p] + 6 e'[p] + 4 o'[p] + e[p + 1], e' = (e[p].hi, e[p + 1].lo)
            uint32_t q[2];
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const u16x2 es = as_u16x2(__builtin_amdgcn_alignbit(as_u32(ve[i][p + 1]), as_u32(ve[i][p]), 16));
                const u16x2 os = as_u16x2(__builtin_amdgcn_alignbit(as_u32(vo[i][p + 1]), as_u32(vo[i][p]), 16));
                const u16x2 acc = ve[i][p] + vo[i][p] * pair(4, 4) + es * pair(6, 6) + os * pair(4, 4) +
                                  ve[i][p + 1] + pair(128, 128);
                q[p] = as_u32(acc) >> 8;  // bytes 0 and 2: the two outputs
            }
            const uint32_t packed = __builtin_amdgcn_perm(q[1], q[0], 0x06040200u);
            // the row padding (stride >= Wd rounded up to 64) takes the bytes past Wd
            __builtin_memcpy(__builtin_assume_aligned(d + (int64_t)oy * dstride + x0, 4), &packed, 4);
        }
        return;
    }
    // border workgroup: lane = (row band, group)
    const int g = lane % kBorderGroups;
    const int x0 = g == 0 ? 0 : x1 + 4 * (g - 1);
    const int oy0 = ((blockIdx.y * 4 + wave) * (64 / kBorderGroups) + lane / kBorderGroups) * PD_R;
    if (x0 >= Wd || oy0 >= Hd) return;
    const int c0 = 2 * x0 - 2;
    int v[PD_R][11];
#pragma unroll
    for (int i = 0; i < PD_R; ++i)
#pragma unroll
        for (int k = 0; k < 11; ++k) v[i][k] = 0;
    int cols[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) cols[k] = refl(min(c0 + k, 2 * W - 2), W);
#pragma unroll
    for (int r = 0; r < PD_SR; ++r) {
        const uint8_t* row = s + (int64_t)refl(min(2 * oy0 - 2 + r, 2 * H - 2), H) * sstride;
        int b[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) b[k] = row[cols[k]];
#pragma unroll
        for (int i = 0; i < PD_R; ++i) {
            const int t = r - 2 * i;
            if (t < 0 || t > 4) continue;
            const int c = (t == 0 || t == 4) ? 1 : (t == 2 ? 6 : 4);
#pragma unroll
            for (int k = 0; k < 11; ++k) v[i][k] += c * b[k];
        }
    }
#pragma unroll
    for (int i = 0; i < PD_R; ++i) {
        const int oy = oy0 + i;
        if (oy >= Hd) break;
        uint32_t packed = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int acc = v[i][2 * j] + 4 * v[i][2 * j + 1] + 6 * v[i][2 * j + 2] + 4 * v[i][2 * j + 3] + v[i][2 * j + 4];
            packed |= (uint32_t)((acc + 128) >> 8) << (8 * j);
        }
        __builtin_memcpy(__builtin_assume_aligned(d + (int64_t)oy * dstride + x0, 4), &packed, 4);
    }
}

// ------------------------------------------------------------------------------------------------
// calcSharrDeriv: a lane makes pixels x0 .. x0 + 3 of SC_R rows from source columns x0 - 1 .. x0 + 4 of rows
// y0 - 1 .. y0 + SC_R (interior: one aligned dwordx3 per row); the 4 (dx, dy) int16 pairs of a row leave as one
// aligned 16-byte store (derivative rows are padded to 16 pixels).
// ------------------------------------------------------------------------------------------------
constexpr int SC_TW = 256;

// interior x0 < sc_x1(W): x0 + 10 < W, so the aligned 12 bytes of every source row stay inside it
__host__ __device__ __forceinline__ int sc_x1(int W) {
    const int xm = W >= 18 ? (W - 11) & ~3 : 0;
    return xm >= 4 ? xm + 4 : 4;
}

template <int SC_R>
__device__ __forceinline__ void scharr_rows(const int (&a)[SC_R + 2][6], int y0, int H, int x0, int dstride,
                                            int16_t* __restrict__ d) {
#pragma unroll
    for (int i = 0; i < SC_R; ++i) {
        const int y = y0 + i;
        if (y >= H) break;
        int t0[6], t1[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            t0[k] = (a[i][k] + a[i + 2][k]) * 3 + a[i + 1][k] * 10;
            t1[k] = a[i + 2][k] - a[i][k];
        }
        uint32_t out[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int dx = t0[j + 2] - t0[j], dy = (t1[j] + t1[j + 2]) * 3 + t1[j + 1] * 10;
            out[j] = (uint32_t)(uint16_t)dx | ((uint32_t)(uint16_t)dy << 16);
        }
        // pixels past W land in the row padding
        __builtin_memcpy(__builtin_assume_aligned(d + 2 * ((int64_t)y * dstride + x0), 16), out, 16);
    }
}

template <int SC_R>
__global__ __launch_bounds__(256) void scharr_kernel(const uint8_t* __restrict__ src, int H, int W, int sstride,
                                                     int64_t spitch, int16_t* __restrict__ der, int dstride,
                                                     int64_t dpitch) {
    const int img = blockIdx.z;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x1 = sc_x1(W);
    const uint8_t* s = src + (int64_t)img * spitch;
    int16_t* d = der + (int64_t)img * dpitch;
    int a[SC_R + 2][6];  // source (y0 - 1 + r, x0 - 1 + k)
    if (blockIdx.x != gridDim.x - 1) {
        const int x0 = 4 + blockIdx.x * SC_TW + lane * 4;
        const int y0 = (blockIdx.y * 4 + wave) * SC_R;
        if (x0 >= x1 || y0 >= H) return;
        uint32_t raw[SC_R + 2][3];
        uint32_t mis[SC_R + 2];
#pragma unroll
        for (int r = 0; r < SC_R + 2; ++r) {
            const uint8_t* row = s + (int64_t)refl(min(y0 - 1 + r, H), H) * sstride;
            mis[r] = ((uint32_t)(uintptr_t)row + 3u) & 3u;  // (row + x0 - 1) & 3
            __builtin_memcpy(raw[r], __builtin_assume_aligned(row + x0 - 1 - mis[r], 4), 12);
        }
#pragma unroll
        for (int r = 0; r < SC_R + 2; ++r) {
            const uint32_t w0 = __builtin_amdgcn_alignbyte(raw[r][1], raw[r][0], mis[r]);
            const uint32_t w1 = __builtin_amdgcn_alignbyte(raw[r][2], raw[r][1], mis[r]);
#pragma unroll
            for (int k = 0; k < 4; ++k) a[r][k] = (w0 >> (8 * k)) & 0xFF;
            a[r][4] = w1 & 0xFF;
            a[r][5] = (w1 >> 8) & 0xFF;
        }
        scharr_rows<SC_R>(a, y0, H, x0, dstride, d);
        return;
    }
    // border workgroup: lane = (row band, group)
    const int g = lane % kBorderGroups;
    const int x0 = g == 0 ? 0 : x1 + 4 * (g - 1);
    const int y0 = ((blockIdx.y * 4 + wave) * (64 / kBorderGroups) + lane / kBorderGroups) * SC_R;
    if (x0 >= W || y0 >= H) return;
    int cols[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) cols[k] = refl(min(x0 - 1 + k, W), W);
#pragma unroll
    for (int r = 0; r < SC_R + 2; ++r) {
        const uint8_t* row = s + (int64_t)refl(min(y0 - 1 + r, H), H) * sstride;
#pragma unroll
        for (int k = 0; k < 6; ++k) a[r][k] = row[cols[k]];
    }
    scharr_rows<SC_R>(a, y0, H, x0, dstride, d);
}

// ------------------------------------------------------------------------------------------------
// LK
// ------------------------------------------------------------------------------------------------
constexpr int kWBits = 14;
constexpr int kLkLanes = 16;                   // lanes per point: one DPP row
constexpr int kLkPtsPerBlock = 256 / kLkLanes;  // 16 points per 256-thread workgroup

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

__device__ __forceinline__ void weights(float a, float b, int* iw) {
    iw[0] = (int)__builtin_rintf((1.f - a) * (1.f - b) * (float)(1 << kWBits));
    iw[1] = (int)__builtin_rintf(a * (1.f - b) * (float)(1 << kWBits));
    iw[2] = (int)__builtin_rintf((1.f - a) * b * (float)(1 << kWBits));
    iw[3] = (1 << kWBits) - iw[0] - iw[1] - iw[2];
}


// row rotations read a lane of the same row for every lane, so no old value is needed (mov_dpp, bound_ctrl)
template <int kCtrl>
__device__ __forceinline__ float row_dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kCtrl, 0xF, 0xF, true));
}

// Sum over a point's 16 lanes (one DPP row) in the oracle's sum_mode 1 order: the butterfly q[l] + q[l ^ off],
// off = 8, 4, 2, 1, as row rotations (after the step with off the values have period off, so rotating by off / 2
// brings lane l ^ (off / 2)).  Lane 0 follows the tree p[l] += p[l + off]; every lane ends with the same bits
// (IEEE addition commutes), so the Newton step needs no broadcast.
// Butterfly steps as single v_add_f32 with the DPP row rotation on an operand (an opaque register copy keeps the
// two sums of a pair from being packed into v_pk_add_f32, which takes no DPP operand).
// two independent sums, their steps alternated so each DPP read finds its operand's write two instructions back
// (no s_nop for the VALU-write -> DPP-read hazard)
template <int kCtrl>
__device__ __forceinline__ void row_add_dpp2(float& p, float& q) {
    p = p + row_dpp<kCtrl>(p);
    q = q + row_dpp<kCtrl>(q);
    __asm__ volatile("" : "+v"(p), "+v"(q));
}

__device__ __forceinline__ void row_sum_dpp2(float& p, float& q) {
    row_add_dpp2<0x128>(p, q);  // row_ror:8
    row_add_dpp2<0x124>(p, q);  // row_ror:4
    row_add_dpp2<0x122>(p, q);  // row_ror:2
    row_add_dpp2<0x121>(p, q);  // row_ror:1
}

__device__ __forceinline__ float row_sum(float q) {
    q = q + row_dpp<0x128>(q);  // row_ror:8
    q = q + row_dpp<0x124>(q);  // row_ror:4
    q = q + row_dpp<0x122>(q);  // row_ror:2
    q = q + row_dpp<0x121>(q);  // row_ror:1
    return q;
}

// REFLECT_101 then clamped: task pixels past the window (never summed) may lie beyond one reflection on a small
// top level; their addresses stay in the image
__device__ __forceinline__ int refl_c(int p, int len) { return min(max(refl(p, len), 0), len - 1); }

// the (S + 1) x (S + 1) bilinear footprint of a lane's task, top-left (x0, y0), REFLECT_101 outside the image.
// Inside the image each row's S + 1 <= 4 bytes come from one dword-aligned dwordx2 and one v_alignbyte (the aligned
// 8 bytes stay inside the row: x0 + 7 < Wl); otherwise byte loads at reflected coordinates.
template <int S>
__device__ __forceinline__ void load_footprint(const uint8_t* __restrict__ J, int sJ, int Hl, int Wl, int x0, int y0,
                                               int (&v)[S + 1][S + 1]) {
    if (S <= 3 && x0 >= 0 && y0 >= 0 && x0 + 7 < Wl && y0 + S < Hl) {
        const uint32_t off = (uint32_t)(y0 * sJ + x0);
#pragma unroll
        for (int i = 0; i <= S; ++i) {
            const uint32_t o = off + (uint32_t)(i * sJ);
            const uint32_t mis = (uint32_t)((uintptr_t)J + o) & 3u;
            u32x2 a;  // one dwordx2 at 4-byte alignment
            __builtin_memcpy(&a, __builtin_assume_aligned(J + (o - mis), 4), 8);
            const uint32_t w = __builtin_amdgcn_alignbyte(a.y, a.x, mis);
#pragma unroll
            for (int j = 0; j <= S; ++j) v[i][j] = (w >> (8 * j)) & 0xFF;
        }
    } else if (x0 >= 0 && y0 >= 0 && x0 + S < Wl && y0 + S < Hl) {
        uint32_t row = (uint32_t)(y0 * sJ + x0);
#pragma unroll
        for (int i = 0; i <= S; ++i, row += (uint32_t)sJ)
#pragma unroll
            for (int j = 0; j <= S; ++j) v[i][j] = J[row + (uint32_t)j];
    } else {
        int r[S + 1], c[S + 1];
#pragma unroll
        for (int i = 0; i <= S; ++i) {
            r[i] = refl_c(y0 + i, Hl) * sJ;
            c[i] = refl_c(x0 + i, Wl);
        }
#pragma unroll
        for (int i = 0; i <= S; ++i)
#pragma unroll
            for (int j = 0; j <= S; ++j) v[i][j] = J[(uint32_t)(r[i] + c[j])];
    }
}

// calcSharrDeriv of the level image I at the (S + 1) x (S + 1) footprint positions (y0 + i, x0 + j), computed in
// place from I's (S + 3) x (S + 3) neighbourhood instead of read from a derivative pyramid: the same exact integers
// as scharr_kernel (REFLECT_101 on I), packed (dx, dy) as scharr_kernel stores them, and 0 at positions outside the
// image (the derivative border LK reads); the window's inside is also the I footprint of the level.  Inside the
// image one unaligned 8-byte load per window row; near a border, reflected byte loads.
template <int S>
__device__ __forceinline__ void scharr_footprint(const uint8_t* __restrict__ I, int sI, int Hl, int Wl, int x0,
                                                 int y0, int (&dv)[S + 1][S + 1], uint32_t (&ip)[S + 1][S]) {
    constexpr int N = S + 3, NW = (N + 3) / 4;
    uint32_t w[N][NW];  // bytes of I(y0 - 1 + r, x0 - 1 .. x0 + S + 1), packed 4 per dword
    if (S <= 3 && x0 >= 1 && y0 >= 1 && x0 + 8 <= Wl && y0 + S + 1 < Hl) {
        // one unaligned 4 NW-byte load per window row (x0 - 1 + 4 NW <= x0 + 7 < Wl: inside the row)
#pragma unroll
        for (int r = 0; r < N; ++r) {
            const uint32_t o = (uint32_t)((y0 - 1 + r) * sI + x0 - 1);
            __builtin_memcpy(w[r], I + o, 4 * NW);
        }
    } else {
        int cc[N];
#pragma unroll
        for (int k = 0; k < N; ++k) cc[k] = refl_c(x0 - 1 + k, Wl);
#pragma unroll
        for (int r = 0; r < N; ++r) {
            const uint32_t rr = (uint32_t)(refl_c(y0 - 1 + r, Hl) * sI);
#pragma unroll
            for (int q = 0; q < NW; ++q) w[r][q] = 0;
#pragma unroll
            for (int k = 0; k < N; ++k) w[r][k >> 2] |= (uint32_t)I[rr + (uint32_t)cc[k]] << (8 * (k & 3));
        }
    }
    // the window's inner (S + 1) x (S + 1) is the I footprint (refl_c at the borders, as load_footprint reads it),
    // as the horizontal pairs (I(i, j), I(i, j + 1)) of bilinear_dot2: bytes j + 1, j + 2 of window row i + 1
#pragma unroll
    for (int i = 0; i <= S; ++i)
#pragma unroll
        for (int j = 0; j < S; ++j) {
            constexpr int kLastW = NW - 1;
            const int q = (j + 1) >> 2, o = (j + 1) & 3;
            ip[i][j] = __builtin_amdgcn_perm(w[i + 1][q + 1 <= kLastW ? q + 1 : kLastW], w[i + 1][q],
                                             0x0C000C00u | ((uint32_t)(o + 1) << 16) | (uint32_t)o);
        }
#pragma unroll
    for (int i = 0; i <= S; ++i) {
        int t0[N], t1[N];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const int sh = 8 * (k & 3);
            const int a0 = (w[i][k >> 2] >> sh) & 0xFF, a1 = (w[i + 1][k >> 2] >> sh) & 0xFF;
            const int a2 = (w[i + 2][k >> 2] >> sh) & 0xFF;
            t0[k] = (a0 + a2) * 3 + a1 * 10;
            t1[k] = a2 - a0;
        }
        const bool rin = y0 + i >= 0 && y0 + i < Hl;
#pragma unroll
        for (int j = 0; j <= S; ++j) {
            const bool in = rin && x0 + j >= 0 && x0 + j < Wl;
            const int dx = t0[j + 2] - t0[j], dy = (t1[j] + t1[j + 2]) * 3 + t1[j + 1] * 10;
            dv[i][j] = in ? (int)((uint32_t)(uint16_t)dx | ((uint32_t)dy << 16)) : 0;  // as scharr_kernel packs
        }
    }
}

// The footprint as horizontal pairs p[i][j] = (v[i][j], v[i][j + 1]) packed 16-bit (v_perm from the row's dword
// inside the image), the operand form of v_dot2_i32_i16: the bilinear sum w0 J00 + w1 J01 + w2 J10 + w3 J11 + c is
// two signed dot2 on the pairs (w0, w1) / (w2, w3), exact integers like the mad24 chain.  Signed: w3 = 2^14 - w0 -
// w1 - w2 is -1 when all three round up (a b 2^14 < 1.5, e.g. a = 0.4995, b = 2^-14).
template <int S>
__device__ __forceinline__ void load_footprint_pairs(const uint8_t* __restrict__ J, int sJ, int Hl, int Wl, int x0,
                                                     int y0, uint32_t (&p)[S + 1][S]) {
    if (S <= 3 && x0 >= 0 && y0 >= 0 && x0 + 3 < Wl && y0 + S < Hl) {
        const uint32_t off = (uint32_t)(y0 * sJ + x0);
#pragma unroll
        for (int i = 0; i <= S; ++i) {
            const uint32_t o = off + (uint32_t)(i * sJ);
            // one byte-aligned dword load (the hardware's unaligned mode splits it), no alignment arithmetic in VALU
            uint32_t w;
            __builtin_memcpy(&w, J + o, 4);
#pragma unroll
            for (int j = 0; j < S; ++j)  // bytes j, j + 1 into the low bytes of the two halves (0x0C selects 0)
                p[i][j] = __builtin_amdgcn_perm(0u, w, 0x0C000C00u | ((uint32_t)(j + 1) << 16) | (uint32_t)j);
        }
    } else {
        int v[S + 1][S + 1];
        load_footprint<S>(J, sJ, Hl, Wl, x0, y0, v);
#pragma unroll
        for (int i = 0; i <= S; ++i)
#pragma unroll
            for (int j = 0; j < S; ++j) p[i][j] = (uint32_t)v[i][j] | ((uint32_t)v[i][j + 1] << 16);
    }
}

typedef int16_t lk_s2 __attribute__((ext_vector_type(2)));
typedef float lk_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int bilinear_dot2(uint32_t top, uint32_t bot, uint32_t w01, uint32_t w23, int c) {
    // clamp on the first dot2 (its sums stay far inside int32, so it never saturates) selects the three-operand
    // VOP3P form: the accumulate-in-place v_dot2c would need a copy of the loop-invariant c every time
    const int t = __builtin_amdgcn_sdot2(__builtin_bit_cast(lk_s2, bot), __builtin_bit_cast(lk_s2, w23), c, true);
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(lk_s2, top), __builtin_bit_cast(lk_s2, w01), t, false);
}

// One point per 16-lane row, 4 per wave.  Lane g of the row owns the S x S task at window rows S (g >> 2) ..,
// columns S (g & 3) .. (S = ceil(win / 4)); per level it keeps, for each task pixel, the I sample folded into the
// rounding constant of the J interpolation (ck = 2^8 - 2^9 iv, so (ck + sum w J) >> 9 = descale(.) - iv) and the
// derivatives as floats (zero for pixels past the window, which then add +0 to every sum).
template <int S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(S <= 2 ? 8 : (S == 3 ? 6 : 1)))) void lk_kernel(LkParams P, const int32_t* __restrict__ pairs,
                                                 const float* __restrict__ pts, const int32_t* __restrict__ counts,
                                                 int pts_stride, float* __restrict__ next_out,
                                                 uint8_t* __restrict__ status_out, float* __restrict__ err_out) {
    const int pair = blockIdx.y;
    const int g = threadIdx.x & (kLkLanes - 1);
    const int pi = blockIdx.x * kLkPtsPerBlock + (threadIdx.x >> 4);
    const int n = counts[pair];
    if (pi >= n) return;  // whole rows leave together
    const int ia = pairs[2 * pair], ib = pairs[2 * pair + 1];
    const int64_t po = (int64_t)pair * pts_stride + pi;
    const int win = P.win;
    const float halfw = (float)((win - 1) * 0.5f);
    const float px0 = pts[2 * po], py0 = pts[2 * po + 1];
    const int r0 = S * (g >> 2), c0 = S * (g & 3);
    float nxo = 0.f, nyo = 0.f;  // nextPts[ptidx]
    uint8_t status = 1;
    float err = 0.f;
    const float FLT_SCALE = 1.f / (1 << 20);
    for (int level = P.levels; level >= 0; --level) {
        const int Wl = P.w[level], Hl = P.h[level];
        const uint8_t* I = level == 0 ? P.img0 + (int64_t)ia * P.pitch0 : P.pyr + (int64_t)ia * P.pyr_pitch + P.off[level];
        const uint8_t* J = level == 0 ? P.img0 + (int64_t)ib * P.pitch0 : P.pyr + (int64_t)ib * P.pyr_pitch + P.off[level];
        const int sI = level == 0 ? P.stride0 : P.ps[level];
        const float scale = __builtin_ldexpf(1.f, -level);  // (float)(1. / (1 << level)), exact
        float px = px0 * scale, py = py0 * scale;
        float nx, ny;
        if (level == P.levels) {
            nx = px;
            ny = py;
        } else {
            nx = nxo * 2.f;
            ny = nyo * 2.f;
        }
        nxo = nx;
        nyo = ny;
        px -= halfw;
        py -= halfw;
        const int ipx = (int)floorf(px), ipy = (int)floorf(py);
        if (ipx < -win || ipx >= Wl || ipy < -win || ipy >= Hl) {
            if (level == 0) {
                status = 0;
                err = 0.f;
            }
            continue;
        }
        int iw[4];
        weights(px - (float)ipx, py - (float)ipy, iw);
        // I and (dx, dy) over the task footprint; the derivative image is zero outside [0, Hl) x [0, Wl)
        int dv[S + 1][S + 1];
        uint32_t ip[S + 1][S];
        scharr_footprint<S>(I, sI, Hl, Wl, ipx + c0, ipy + r0, dv, ip);
        const uint32_t iw01 = ((uint32_t)iw[0] & 0xFFFFu) | ((uint32_t)iw[1] << 16);
        const uint32_t iw23 = ((uint32_t)iw[2] & 0xFFFFu) | ((uint32_t)iw[3] << 16);
        int ck[S][S];
        float fx[S][S], fy[S][S];
        float a11 = 0.0f, a12 = 0.0f, a22 = 0.0f;
#pragma unroll
        for (int i = 0; i < S; ++i)
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const int ival = descale(bilinear_dot2(ip[i][j], ip[i + 1][j], iw01, iw23, 0), kWBits - 5);
                // the dx (low) / dy (high) halves of the packed derivatives as horizontal pairs, one v_perm each
                const uint32_t xt = __builtin_amdgcn_perm((uint32_t)dv[i][j + 1], (uint32_t)dv[i][j], 0x05040100u);
                const uint32_t xb = __builtin_amdgcn_perm((uint32_t)dv[i + 1][j + 1], (uint32_t)dv[i + 1][j], 0x05040100u);
                const uint32_t yt = __builtin_amdgcn_perm((uint32_t)dv[i][j + 1], (uint32_t)dv[i][j], 0x07060302u);
                const uint32_t yb = __builtin_amdgcn_perm((uint32_t)dv[i + 1][j + 1], (uint32_t)dv[i + 1][j], 0x07060302u);
                const int ixv = descale(bilinear_dot2(xt, xb, iw01, iw23, 0), kWBits);
                const int iyv = descale(bilinear_dot2(yt, yb, iw01, iw23, 0), kWBits);
                const bool in = r0 + i < win && c0 + j < win;
                ck[i][j] = (1 << (kWBits - 6)) - (ival << (kWBits - 5));
                fx[i][j] = in ? (float)ixv : 0.f;
                fy[i][j] = in ? (float)iyv : 0.f;
                // (float)(ixv * ixv) etc.: the products are < 2^24, exact as floats
                a11 = a11 + fx[i][j] * fx[i][j];
                a12 = a12 + fx[i][j] * fy[i][j];
                a22 = a22 + fy[i][j] * fy[i][j];
            }
        row_sum_dpp2(a11, a12);
        const float A11 = a11 * FLT_SCALE;
        const float A12 = a12 * FLT_SCALE;
        const float A22 = row_sum(a22) * FLT_SCALE;
        float Dd = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win * win);
        if (minEig < P.min_eig || Dd < FLT_EPSILON) {
            if (level == 0) status = 0;
            continue;
        }
        Dd = 1.f / Dd;
        nx -= halfw;
        ny -= halfw;
        float pdx = 0.f, pdy = 0.f;
        for (int it = 0; it < P.max_count; ++it) {
            const int inx = (int)floorf(nx), iny = (int)floorf(ny);
            if (inx < -win || inx >= Wl || iny < -win || iny >= Hl) {
                if (level == 0) status = 0;
                break;
            }
            weights(nx - (float)inx, ny - (float)iny, iw);
            const uint32_t w01 = ((uint32_t)iw[0] & 0xFFFFu) | ((uint32_t)iw[1] << 16);
            const uint32_t w23 = ((uint32_t)iw[2] & 0xFFFFu) | ((uint32_t)iw[3] << 16);
            uint32_t jp[S + 1][S];
            load_footprint_pairs<S>(J, sI, Hl, Wl, inx + c0, iny + r0, jp);
            // (b1, b2) as one packed pair: v_pk_mul_f32 / v_pk_add_f32 round each half like the scalar ops
            lk_f2 bb = {0.0f, 0.0f};
#pragma unroll
            for (int i = 0; i < S; ++i)
#pragma unroll
                for (int j = 0; j < S; ++j) {
                    const int acc = bilinear_dot2(jp[i][j], jp[i + 1][j], w01, w23, ck[i][j]);
                    // (float)(diff * ixv): |diff * ixv| < 2^27, one rounding either way
                    const float d = (float)(acc >> (kWBits - 5));
                    const lk_f2 dd = {d, d}, f = {fx[i][j], fy[i][j]};
                    bb = bb + dd * f;
                }
            float s1 = bb.x, s2 = bb.y;
            row_sum_dpp2(s1, s2);
            const float B1 = s1 * FLT_SCALE;
            const float B2 = s2 * FLT_SCALE;
            const float dx = (float)((A12 * B2 - A22 * B1) * Dd);
            const float dy = (float)((A12 * B1 - A11 * B2) * Dd);
            nx += dx;
            ny += dy;
            nxo = nx + halfw;
            nyo = ny + halfw;
            if ((double)dx * dx + (double)dy * dy <= P.eps2) break;
            // |v| < 0.01 (double) <=> |v| <= 0.01f: the float nearest 0.01 lies below it and the next one above
            if (it > 0 && fabsf(dx + pdx) <= 0.01f && fabsf(dy + pdy) <= 0.01f) {
                nxo -= dx * 0.5f;
                nyo -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }
        if (status && level == 0) {
            const float ex = nxo - halfw, ey = nyo - halfw;
            const int inx = (int)floorf(ex), iny = (int)floorf(ey);
            if (inx < -win || inx >= Wl || iny < -win || iny >= Hl) {
                status = 0;
            } else {
                weights(ex - (float)inx, ey - (float)iny, iw);
                const uint32_t w01 = ((uint32_t)iw[0] & 0xFFFFu) | ((uint32_t)iw[1] << 16);
                const uint32_t w23 = ((uint32_t)iw[2] & 0xFFFFu) | ((uint32_t)iw[3] << 16);
                uint32_t jp[S + 1][S];
                load_footprint_pairs<S>(J, sI, Hl, Wl, inx + c0, iny + r0, jp);
                float e = 0.0f;
#pragma unroll
                for (int i = 0; i < S; ++i)
#pragma unroll
                    for (int j = 0; j < S; ++j) {
                        const int acc = bilinear_dot2(jp[i][j], jp[i + 1][j], w01, w23, ck[i][j]);
                        const bool in = r0 + i < win && c0 + j < win;
                        e = e + (in ? fabsf((float)(acc >> (kWBits - 5))) : 0.f);
                    }
                err = row_sum(e) * 1.f / (float)(32 * win * win);
            }
        }
    }
    if (g == 0) {
        next_out[2 * po] = nxo;
        next_out[2 * po + 1] = nyo;
        status_out[po] = status;
        err_out[po] = err;
    }
}

}  // namespace lk

void launch_lk_pyramid(const LkParams& P, int n_images, hipStream_t s) {
    constexpr int kPdR = 4;  // output rows per lane
    // level l (>= 1) from level l-1 (the tracker computes the Scharr derivatives inside its windows); the grid is the
    // interior workgroup columns + one border column (whose workgroups cover 8x the rows: row tiles past the image
    // return at once)
    for (int l = 1; l <= P.levels; ++l) {
        const int Hs = P.h[l - 1], Ws = P.w[l - 1];
        const uint8_t* src = l == 1 ? P.img0 : P.pyr + P.off[l - 1];
        const int sstride = l == 1 ? P.stride0 : P.ps[l - 1];
        const int64_t spitch = l == 1 ? P.pitch0 : P.pyr_pitch;
        dim3 grid((lk::pd_x1(Ws) - 4 + lk::PD_TW - 1) / lk::PD_TW + 1, (P.h[l] + 4 * kPdR - 1) / (4 * kPdR), n_images);
        hipLaunchKernelGGL(lk::pyr_down_kernel<kPdR>, grid, dim3(256), 0, s, src, Hs, Ws, sstride, spitch,
                           P.pyr + P.off[l], P.ps[l], P.pyr_pitch);
    }
}

void launch_lk_derivs(const LkParams& P, int image, int level, int16_t* der, hipStream_t s) {
    // one level of one image into der (rows ds[level] pixels apart): the inspection path of yv_lk_level
    constexpr int kScR = 4;
    const uint8_t* src = level == 0 ? P.img0 + (int64_t)image * P.pitch0 : P.pyr + (int64_t)image * P.pyr_pitch + P.off[level];
    const int sstride = level == 0 ? P.stride0 : P.ps[level];
    dim3 grid((lk::sc_x1(P.w[level]) - 4 + lk::SC_TW - 1) / lk::SC_TW + 1, (P.h[level] + 4 * kScR - 1) / (4 * kScR), 1);
    hipLaunchKernelGGL(lk::scharr_kernel<kScR>, grid, dim3(256), 0, s, src, P.h[level], P.w[level], sstride, (int64_t)0,
                       der, P.ds[level], (int64_t)0);
}

void launch_lk_track(const LkParams& P, const int32_t* pairs, int n_pairs, const float* pts, const int32_t* counts,
                     int pts_stride, int max_pts, float* next_pts, uint8_t* status, float* err, hipStream_t s) {
    if (n_pairs <= 0 || max_pts <= 0) return;
    dim3 grid((max_pts + lk::kLkPtsPerBlock - 1) / lk::kLkPtsPerBlock, n_pairs);
    // S = ceil(win / 4) pixels per task side (win 3 .. 22)
    switch ((P.win + 3) / 4) {
#define YV_LK_CASE(S)                                                                                             \
    case S:                                                                                                       \
        hipLaunchKernelGGL(lk::lk_kernel<S>, grid, dim3(256), 0, s, P, pairs, pts, counts, pts_stride, next_pts, \
                           status, err);                                                                          \
        break;
        YV_LK_CASE(1)
        YV_LK_CASE(2)
        YV_LK_CASE(3)
        YV_LK_CASE(4)
        YV_LK_CASE(5)
        YV_LK_CASE(6)
#undef YV_LK_CASE
        default:
            break;
    }
}

}  // namespace yavo
