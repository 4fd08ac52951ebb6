// yavo_lk.hip -- gfx950 kernels for cv::calcOpticalFlowPyrLK as the reference calls it (SURVEY.md 8f row 1;
// src/LoopHandler.cc:372-375: winSize 11x11, maxLevel 3, TermCriteria(COUNT+EPS, 30, 0.01), flags 0,
// minEigThreshold 0.001).  Restates OpenCV's lkpyramid.cpp (scalar path) like oracle/yavo_oracle_lk.c:
//
//   pyr_down_kernel   cv::pyrDown CV_8U, 5x5 [1 4 6 4 1]^2 / 256, BORDER_REFLECT_101 (exact integers); a
//                     16 x 64 output tile per workgroup, its 35 x 131 source patch staged in LDS
//   scharr_kernel     calcSharrDeriv: int16 (dx, dy), REFLECT_101 rows / columns
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

// ------------------------------------------------------------------------------------------------
// pyrDown
// ------------------------------------------------------------------------------------------------
constexpr int PD_TH = 16, PD_TW = 64;                  // output tile
constexpr int PD_SH = 2 * PD_TH + 3, PD_SW = 2 * PD_TW + 3;  // source patch 35 x 131

__global__ __launch_bounds__(256) void pyr_down_kernel(const uint8_t* __restrict__ src, int H, int W, int sstride,
                                                       int64_t spitch, uint8_t* __restrict__ dst, int64_t dpitch) {
    __shared__ uint8_t s_src[PD_SH * PD_SW];
    __shared__ int s_h[PD_SH * PD_TW];
    const int img = blockIdx.z;
    const int Hd = (H + 1) / 2, Wd = (W + 1) / 2;
    const int oy0 = blockIdx.y * PD_TH, ox0 = blockIdx.x * PD_TW;
    const uint8_t* s = src + (int64_t)img * spitch;
    const int sy0 = 2 * oy0 - 2, sx0 = 2 * ox0 - 2;
    for (int i = threadIdx.x; i < PD_SH * PD_SW; i += 256) {
        const int r = i / PD_SW, c = i - r * PD_SW;
        const int y = refl(min(sy0 + r, 2 * H - 2), H), x = refl(min(sx0 + c, 2 * W - 2), W);
        s_src[i] = s[(int64_t)y * sstride + x];
    }
    __syncthreads();
    // horizontal: h(r, x) = src(r, 2x-2) + 4 src(r, 2x-1) + 6 src(r, 2x) + 4 src(r, 2x+1) + src(r, 2x+2)
    for (int i = threadIdx.x; i < PD_SH * PD_TW; i += 256) {
        const int r = i / PD_TW, x = i - r * PD_TW;
        const uint8_t* p = s_src + r * PD_SW + 2 * x;
        s_h[i] = p[0] + 4 * p[1] + 6 * p[2] + 4 * p[3] + p[4];
    }
    __syncthreads();
    uint8_t* d = dst + (int64_t)img * dpitch;
    for (int i = threadIdx.x; i < PD_TH * PD_TW; i += 256) {
        const int y = i / PD_TW, x = i - y * PD_TW;
        const int oy = oy0 + y, ox = ox0 + x;
        if (oy >= Hd || ox >= Wd) continue;
        const int* q = s_h + (2 * y) * PD_TW + x;
        const int acc = q[0] + 4 * q[PD_TW] + 6 * q[2 * PD_TW] + 4 * q[3 * PD_TW] + q[4 * PD_TW];
        d[(int64_t)oy * Wd + ox] = (uint8_t)((acc + 128) >> 8);
    }
}

// ------------------------------------------------------------------------------------------------
// calcSharrDeriv
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void scharr_kernel(const uint8_t* __restrict__ src, int H, int W, int sstride,
                                                     int64_t spitch, int16_t* __restrict__ der, int64_t dpitch) {
    const int img = blockIdx.z;
    const int y = blockIdx.y;
    const uint8_t* s = src + (int64_t)img * spitch;
    const uint8_t* s0 = s + (int64_t)refl(y - 1, H) * sstride;
    const uint8_t* s1 = s + (int64_t)y * sstride;
    const uint8_t* s2 = s + (int64_t)refl(y + 1, H) * sstride;
    int16_t* d = der + (int64_t)img * dpitch + (int64_t)y * W * 2;
    for (int x = blockIdx.x * 256 + threadIdx.x; x < W; x += gridDim.x * 256) {
        const int xl = refl(x - 1, W), xr = refl(x + 1, W);
        const int t0l = (s0[xl] + s2[xl]) * 3 + s1[xl] * 10, t0r = (s0[xr] + s2[xr]) * 3 + s1[xr] * 10;
        const int t1l = s2[xl] - s0[xl], t1r = s2[xr] - s0[xr], t1c = s2[x] - s0[x];
        const int dx = t0r - t0l, dy = (t1r + t1l) * 3 + t1c * 10;
        d[2 * x] = (int16_t)dx;
        d[2 * x + 1] = (int16_t)dy;
    }
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

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// a * b + c with |a|, |b| < 2^23 (v_mad_i32_i24): samples are u8 / int16, weights <= 2^14
__device__ __forceinline__ int mad24(int a, int b, int c) { return __mul24(a, b) + c; }

template <int kCtrl>
__device__ __forceinline__ float row_dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xF, 0xF, false));
}

// Sum over a point's 16 lanes (one DPP row) in the oracle's sum_mode 1 order: the butterfly q[l] + q[l ^ off],
// off = 8, 4, 2, 1, as row rotations (after the step with off the values have period off, so rotating by off / 2
// brings lane l ^ (off / 2)).  Lane 0 follows the tree p[l] += p[l + off]; every lane ends with the same bits
// (IEEE addition commutes), so the Newton step needs no broadcast.
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
        const int sI = level == 0 ? P.stride0 : Wl;
        const uint32_t* D = reinterpret_cast<const uint32_t*>(P.der + (int64_t)ia * P.der_pitch + P.der_off[level]);
        const float scale = (float)(1. / (1 << level));
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
        int iv8[S + 1][S + 1];
        load_footprint<S>(I, sI, Hl, Wl, ipx + c0, ipy + r0, iv8);
        int dv[S + 1][S + 1];
        if (S == 3 && ipx + c0 >= 0 && ipy + r0 >= 0 && ipx + c0 + S < Wl && ipy + r0 + S < Hl) {
            // all inside: one dwordx4 per footprint row
#pragma unroll
            for (int i = 0; i <= S; ++i) {
                u32x4 d;
                __builtin_memcpy(&d, __builtin_assume_aligned(D + (uint32_t)((ipy + r0 + i) * Wl + ipx + c0), 4), 16);
#pragma unroll
                for (int j = 0; j <= S; ++j) dv[i][j] = (int)d[j & 3];
            }
        } else {
            int r[S + 1], c[S + 1];
            bool rin[S + 1], cin[S + 1];
#pragma unroll
            for (int i = 0; i <= S; ++i) {
                const int y = ipy + r0 + i, x = ipx + c0 + i;
                rin[i] = y >= 0 && y < Hl;
                cin[i] = x >= 0 && x < Wl;
                r[i] = min(max(y, 0), Hl - 1) * Wl;
                c[i] = min(max(x, 0), Wl - 1);
            }
#pragma unroll
            for (int i = 0; i <= S; ++i)
#pragma unroll
                for (int j = 0; j <= S; ++j) {
                    const uint32_t d = D[(uint32_t)(r[i] + c[j])];
                    dv[i][j] = rin[i] && cin[j] ? (int)d : 0;
                }
        }
        int ck[S][S];
        float fx[S][S], fy[S][S];
        float a11 = 0.0f, a12 = 0.0f, a22 = 0.0f;
#pragma unroll
        for (int i = 0; i < S; ++i)
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const int ival = descale(mad24(iv8[i][j], iw[0], mad24(iv8[i][j + 1], iw[1],
                                         mad24(iv8[i + 1][j], iw[2], iv8[i + 1][j + 1] * iw[3]))), kWBits - 5);
                // (int16) low / high halves of the interleaved (dx, dy) derivative
                const int x00 = (int16_t)dv[i][j], x01 = (int16_t)dv[i][j + 1];
                const int x10 = (int16_t)dv[i + 1][j], x11 = (int16_t)dv[i + 1][j + 1];
                const int y00 = dv[i][j] >> 16, y01 = dv[i][j + 1] >> 16;
                const int y10 = dv[i + 1][j] >> 16, y11 = dv[i + 1][j + 1] >> 16;
                const int ixv = descale(mad24(x00, iw[0], mad24(x01, iw[1], mad24(x10, iw[2], __mul24(x11, iw[3])))), kWBits);
                const int iyv = descale(mad24(y00, iw[0], mad24(y01, iw[1], mad24(y10, iw[2], __mul24(y11, iw[3])))), kWBits);
                const bool in = r0 + i < win && c0 + j < win;
                ck[i][j] = (1 << (kWBits - 6)) - (ival << (kWBits - 5));
                fx[i][j] = in ? (float)ixv : 0.f;
                fy[i][j] = in ? (float)iyv : 0.f;
                // (float)(ixv * ixv) etc.: the products are < 2^24, exact as floats
                a11 = a11 + fx[i][j] * fx[i][j];
                a12 = a12 + fx[i][j] * fy[i][j];
                a22 = a22 + fy[i][j] * fy[i][j];
            }
        const float A11 = row_sum(a11) * FLT_SCALE;
        const float A12 = row_sum(a12) * FLT_SCALE;
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
            int jv[S + 1][S + 1];
            load_footprint<S>(J, sI, Hl, Wl, inx + c0, iny + r0, jv);
            float b1 = 0.0f, b2 = 0.0f;
#pragma unroll
            for (int i = 0; i < S; ++i)
#pragma unroll
                for (int j = 0; j < S; ++j) {
                    const int acc = mad24(jv[i][j], iw[0], mad24(jv[i][j + 1], iw[1],
                                    mad24(jv[i + 1][j], iw[2], mad24(jv[i + 1][j + 1], iw[3], ck[i][j]))));
                    // (float)(diff * ixv): |diff * ixv| < 2^27, one rounding either way
                    const float d = (float)(acc >> (kWBits - 5));
                    b1 = b1 + d * fx[i][j];
                    b2 = b2 + d * fy[i][j];
                }
            const float B1 = row_sum(b1) * FLT_SCALE;
            const float B2 = row_sum(b2) * FLT_SCALE;
            const float dx = (float)((A12 * B2 - A22 * B1) * Dd);
            const float dy = (float)((A12 * B1 - A11 * B2) * Dd);
            nx += dx;
            ny += dy;
            nxo = nx + halfw;
            nyo = ny + halfw;
            if ((double)dx * dx + (double)dy * dy <= P.eps2) break;
            if (it > 0 && fabsf(dx + pdx) < 0.01 && fabsf(dy + pdy) < 0.01) {
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
                int jv[S + 1][S + 1];
                load_footprint<S>(J, sI, Hl, Wl, inx + c0, iny + r0, jv);
                float e = 0.0f;
#pragma unroll
                for (int i = 0; i < S; ++i)
#pragma unroll
                    for (int j = 0; j < S; ++j) {
                        const int acc = mad24(jv[i][j], iw[0], mad24(jv[i][j + 1], iw[1],
                                        mad24(jv[i + 1][j], iw[2], mad24(jv[i + 1][j + 1], iw[3], ck[i][j]))));
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
    // level l (>= 1) from level l-1, then the derivatives of every level
    for (int l = 1; l <= P.levels; ++l) {
        const int Hs = P.h[l - 1], Ws = P.w[l - 1];
        const uint8_t* src = l == 1 ? P.img0 : P.pyr + P.off[l - 1];
        const int sstride = l == 1 ? P.stride0 : Ws;
        const int64_t spitch = l == 1 ? P.pitch0 : P.pyr_pitch;
        dim3 grid((P.w[l] + lk::PD_TW - 1) / lk::PD_TW, (P.h[l] + lk::PD_TH - 1) / lk::PD_TH, n_images);
        hipLaunchKernelGGL(lk::pyr_down_kernel, grid, dim3(256), 0, s, src, Hs, Ws, sstride, spitch,
                           P.pyr + P.off[l], P.pyr_pitch);
    }
    for (int l = 0; l <= P.levels; ++l) {
        const uint8_t* src = l == 0 ? P.img0 : P.pyr + P.off[l];
        const int sstride = l == 0 ? P.stride0 : P.w[l];
        const int64_t spitch = l == 0 ? P.pitch0 : P.pyr_pitch;
        dim3 grid((P.w[l] + 255) / 256, P.h[l], n_images);
        hipLaunchKernelGGL(lk::scharr_kernel, grid, dim3(256), 0, s, src, P.h[l], P.w[l], sstride, spitch,
                           P.der + P.der_off[l], P.der_pitch);
    }
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
