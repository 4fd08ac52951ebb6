// yavo_lk.hip -- gfx950 kernels for cv::calcOpticalFlowPyrLK as the reference calls it (SURVEY.md 8f row 1;
// src/LoopHandler.cc:372-375: winSize 11x11, maxLevel 3, TermCriteria(COUNT+EPS, 30, 0.01), flags 0,
// minEigThreshold 0.001).  Restates OpenCV's lkpyramid.cpp (scalar path) like oracle/yavo_oracle_lk.c:
//
//   pyr_down_kernel   cv::pyrDown CV_8U, 5x5 [1 4 6 4 1]^2 / 256, BORDER_REFLECT_101 (exact integers); a
//                     16 x 64 output tile per workgroup, its 35 x 131 source patch staged in LDS
//   scharr_kernel     calcSharrDeriv: int16 (dx, dy), REFLECT_101 rows / columns
//   lk_kernel         LKTrackerInvoker for every level of one point per wave: window pixel p = y * win + x
//                     lives on lane p mod 64; bilinear samples (14-bit weights, CV_DESCALE) straight from the
//                     level images (REFLECT_101 image border, zero derivative border); window sums as float
//                     partials per lane then a wave tree (the oracle's sum_mode 1); every lane computes the
//                     same Newton step from the broadcast sums
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
// window pixels per lane (MP): ceil(win^2 / 64) rounded to 2, 4 or 8 (win <= 22); the launch picks the smallest

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

__device__ __forceinline__ void weights(float a, float b, int* iw) {
    iw[0] = (int)__builtin_rintf((1.f - a) * (1.f - b) * (float)(1 << kWBits));
    iw[1] = (int)__builtin_rintf(a * (1.f - b) * (float)(1 << kWBits));
    iw[2] = (int)__builtin_rintf((1.f - a) * b * (float)(1 << kWBits));
    iw[3] = (1 << kWBits) - iw[0] - iw[1] - iw[2];
}

// Sum over the window in the oracle's sum_mode 1 order: lane partials from 0.0f, then p[l] += p[l + off] for
// off = 32 .. 1, all in registers: v_permlane32_swap / v_permlane16_swap bring lane l + 32 / l + 16 to lane l
// (the swapped second operand), DPP row_shl:off does l + off inside a 16-lane row; lane 0 holds the total.
__device__ __forceinline__ float wave_sum(float part) {
    float t = __uint_as_float(
        __builtin_amdgcn_permlane32_swap(__float_as_uint(part), __float_as_uint(part), false, false)[1]);
    part = part + t;  // lanes 0..31: p[l] + p[l + 32]
    t = __uint_as_float(
        __builtin_amdgcn_permlane16_swap(__float_as_uint(part), __float_as_uint(part), false, false)[1]);
    part = part + t;  // lanes 0..15 (of each half): + lane l + 16
    part = part + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(part), 0x108, 0xF, 0xF, false));
    part = part + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(part), 0x104, 0xF, 0xF, false));
    part = part + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(part), 0x102, 0xF, 0xF, false));
    part = part + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(part), 0x101, 0xF, 0xF, false));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(part)));
}

template <int kMaxPix>
__global__ __launch_bounds__(256) void lk_kernel(LkParams P, const int32_t* __restrict__ pairs,
                                                 const float* __restrict__ pts, const int32_t* __restrict__ counts,
                                                 int pts_stride, float* __restrict__ next_out,
                                                 uint8_t* __restrict__ status_out, float* __restrict__ err_out) {
    const int pair = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int pi = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int n = counts[pair];
    if (pi >= n) return;
    const int ia = pairs[2 * pair], ib = pairs[2 * pair + 1];
    const int64_t po = (int64_t)pair * pts_stride + pi;
    const int win = P.win, npix = win * win;
    const float halfw = (float)((win - 1) * 0.5f);
    const float px0 = pts[2 * po], py0 = pts[2 * po + 1];
    float nxo = 0.f, nyo = 0.f;  // nextPts[ptidx]
    uint8_t status = 1;
    float err = 0.f;
    const float FLT_SCALE = 1.f / (1 << 20);
    for (int level = P.levels; level >= 0; --level) {
        const int Wl = P.w[level], Hl = P.h[level];
        const uint8_t* I = level == 0 ? P.img0 + (int64_t)ia * P.pitch0 : P.pyr + (int64_t)ia * P.pyr_pitch + P.off[level];
        const uint8_t* J = level == 0 ? P.img0 + (int64_t)ib * P.pitch0 : P.pyr + (int64_t)ib * P.pyr_pitch + P.off[level];
        const int sI = level == 0 ? P.stride0 : Wl;
        const int16_t* D = P.der + (int64_t)ia * P.der_pitch + P.der_off[level];
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
        // this lane's window pixels: I value and derivatives (IWinBuf / derivIWinBuf)
        int iv[kMaxPix], ixv[kMaxPix], iyv[kMaxPix];
        float a11 = 0.0f, a12 = 0.0f, a22 = 0.0f;
        // the whole bilinear footprint inside the level image (wave-uniform): no border logic per sample
        const bool inI = ipx >= 0 && ipy >= 0 && ipx + win < Wl && ipy + win < Hl;
#pragma unroll
        for (int k = 0; k < kMaxPix; ++k) {
            const int p = lane + 64 * k;
            iv[k] = ixv[k] = iyv[k] = 0;
            if (p < npix) {
                const int y = p / win, x = p - y * win;
                const int yy = ipy + y, xx = ipx + x;
                const int r0 = inI ? yy : refl(yy, Hl), r1 = inI ? yy + 1 : refl(yy + 1, Hl);
                const int c0 = inI ? xx : refl(xx, Wl), c1 = inI ? xx + 1 : refl(xx + 1, Wl);
                const uint8_t* i0 = I + r0 * sI;
                const uint8_t* i1 = I + r1 * sI;
                iv[k] = descale(i0[c0] * iw[0] + i0[c1] * iw[1] + i1[c0] * iw[2] + i1[c1] * iw[3], kWBits - 5);
                // derivative image: zero outside [0, Hl) x [0, Wl)
                int dxs[4], dys[4];
                if (inI) {
                    const int16_t* d0 = D + (yy * Wl + xx) * 2;
                    const int16_t* d1 = d0 + Wl * 2;
                    dxs[0] = d0[0]; dys[0] = d0[1]; dxs[1] = d0[2]; dys[1] = d0[3];
                    dxs[2] = d1[0]; dys[2] = d1[1]; dxs[3] = d1[2]; dys[3] = d1[3];
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int ry = yy + (q >> 1), rx = xx + (q & 1);
                        const bool in = ry >= 0 && ry < Hl && rx >= 0 && rx < Wl;
                        const int16_t* dp = D + ((in ? ry : 0) * Wl + (in ? rx : 0)) * 2;
                        dxs[q] = in ? dp[0] : 0;
                        dys[q] = in ? dp[1] : 0;
                    }
                }
                ixv[k] = descale(dxs[0] * iw[0] + dxs[1] * iw[1] + dxs[2] * iw[2] + dxs[3] * iw[3], kWBits);
                iyv[k] = descale(dys[0] * iw[0] + dys[1] * iw[1] + dys[2] * iw[2] + dys[3] * iw[3], kWBits);
                a11 = a11 + (float)(ixv[k] * ixv[k]);
                a12 = a12 + (float)(ixv[k] * iyv[k]);
                a22 = a22 + (float)(iyv[k] * iyv[k]);
            }
        }
        const float A11 = wave_sum(a11) * FLT_SCALE;
        const float A12 = wave_sum(a12) * FLT_SCALE;
        const float A22 = wave_sum(a22) * FLT_SCALE;
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
        for (int j = 0; j < P.max_count; ++j) {
            const int inx = (int)floorf(nx), iny = (int)floorf(ny);
            if (inx < -win || inx >= Wl || iny < -win || iny >= Hl) {
                if (level == 0) status = 0;
                break;
            }
            weights(nx - (float)inx, ny - (float)iny, iw);
            const bool inJ = inx >= 0 && iny >= 0 && inx + win < Wl && iny + win < Hl;
            float b1 = 0.0f, b2 = 0.0f;
#pragma unroll
            for (int k = 0; k < kMaxPix; ++k) {
                const int p = lane + 64 * k;
                if (p < npix) {
                    const int y = p / win, x = p - y * win;
                    const int yy = iny + y, xx = inx + x;
                    const int r0 = inJ ? yy : refl(yy, Hl), r1 = inJ ? yy + 1 : refl(yy + 1, Hl);
                    const int c0 = inJ ? xx : refl(xx, Wl), c1 = inJ ? xx + 1 : refl(xx + 1, Wl);
                    const uint8_t* j0 = J + r0 * sI;
                    const uint8_t* j1 = J + r1 * sI;
                    const int diff = descale(j0[c0] * iw[0] + j0[c1] * iw[1] + j1[c0] * iw[2] + j1[c1] * iw[3],
                                             kWBits - 5) - iv[k];
                    b1 = b1 + (float)(diff * ixv[k]);
                    b2 = b2 + (float)(diff * iyv[k]);
                }
            }
            const float B1 = wave_sum(b1) * FLT_SCALE;
            const float B2 = wave_sum(b2) * FLT_SCALE;
            const float dx = (float)((A12 * B2 - A22 * B1) * Dd);
            const float dy = (float)((A12 * B1 - A11 * B2) * Dd);
            nx += dx;
            ny += dy;
            nxo = nx + halfw;
            nyo = ny + halfw;
            if ((double)dx * dx + (double)dy * dy <= P.eps2) break;
            if (j > 0 && fabsf(dx + pdx) < 0.01 && fabsf(dy + pdy) < 0.01) {
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
                float e = 0.0f;
#pragma unroll
                for (int k = 0; k < kMaxPix; ++k) {
                    const int p = lane + 64 * k;
                    if (p < npix) {
                        const int y = p / win, x = p - y * win;
                        const int yy = iny + y, xx = inx + x;
                        const int r0 = refl(yy, Hl), r1 = refl(yy + 1, Hl), c0 = refl(xx, Wl), c1 = refl(xx + 1, Wl);
                        const int diff = descale(J[(int64_t)r0 * sI + c0] * iw[0] + J[(int64_t)r0 * sI + c1] * iw[1] +
                                                     J[(int64_t)r1 * sI + c0] * iw[2] + J[(int64_t)r1 * sI + c1] * iw[3],
                                                 kWBits - 5) - iv[k];
                        e = e + fabsf((float)diff);
                    }
                }
                err = wave_sum(e) * 1.f / (float)(32 * win * win);
            }
        }
    }
    if (lane == 0) {
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
    dim3 grid((max_pts + 3) / 4, n_pairs);
    const int npix = P.win * P.win;
    if (npix <= 128)
        hipLaunchKernelGGL(lk::lk_kernel<2>, grid, dim3(256), 0, s, P, pairs, pts, counts, pts_stride, next_pts, status, err);
    else if (npix <= 256)
        hipLaunchKernelGGL(lk::lk_kernel<4>, grid, dim3(256), 0, s, P, pairs, pts, counts, pts_stride, next_pts, status, err);
    else
        hipLaunchKernelGGL(lk::lk_kernel<8>, grid, dim3(256), 0, s, P, pairs, pts, counts, pts_stride, next_pts, status, err);
}

}  // namespace yavo
