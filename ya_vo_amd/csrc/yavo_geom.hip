// yavo_geom.hip -- gfx950 kernels for the geometry rows of the hot path.
//
//   f_ransac_kernel      _3DHandler::getFRANSAC / getFundamentalMatrix   src/3DHandler.cc:17-195
//                        (cv::SVD = OpenCV JacobiSVDImpl_<double>), one workgroup per match list, one
//                        hypothesis per lane, the match list staged in LDS for the inlier counts
//   triangulate_kernel   LoopHandler::triangulation + pixel2camera        src/LoopHandler.cc:658-726, 867-915
//                        (Eigen JacobiSVD on the 4x4 DLT system), one lane per match, all in registers
//   world2camera_kernel  Frame::world2Camera                              src/Frame.cc:16-28
//   pose_lm_kernel       LoopHandler::optimizePoseOnly + the g2o edge     src/LoopHandler.cc:730-861,
//                        include/Optimizer.hpp:40-135; one workgroup per pose problem: edge terms
//                        (residual, 2x6 Jacobian, Huber weight) per lane, J^T W J / J^T W e / chi2 as
//                        fixed-order tree reductions in LDS, the 6x6 LDLT + LM control on lane 0
//   pose_gn_kernel       bundleAdjustmentGaussNewton                      src/test.cc:172-244
//
// Every floating-point expression is written in the reference's operation order and the file is built
// with -ffp-contract=off, so each kernel matches oracle/yavo_oracle_geom.c bit for bit (sums over edges
// in the oracle's sum_mode 1 = this file's tree order).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>

#include "yavo_internal.h"
#include "yavo_cvsvd.h"
#include "yavo_se3.h"
#include "yavo_xlane.h"

namespace yavo {
namespace geom {

using cv::cv_hypot;
using cv::cv_rng_next;
using cv::cv_jacobi_svd;
using cv::cv_jacobi_svd_mn;
using se3::k_cos;
using se3::k_sin;
using se3::mm3;
using se3::quat_mul;
using se3::quat_rotate;
using se3::quat_to_R;
using se3::se3_act;
using se3::se3_exp;
using se3::se3_mul;

constexpr int kNT = 256;          // threads per workgroup of the reduction kernels

// YAVO_LM_PROFILE builds (tools/lm_profile.py) time the pose-LM phases with the shader clock on lane 0
#ifdef YAVO_LM_PROFILE
__device__ unsigned long long g_lm_prof[1024][10];
#define LMP_DECL unsigned long long lmp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long lmp_t = __builtin_readcyclecounter();
#define LMP_MARK(slot) do { const unsigned long long t_ = __builtin_readcyclecounter(); lmp_acc[slot] += t_ - lmp_t; lmp_t = t_; } while (0)
#define LMP_STORE() do { if (threadIdx.x == 0) for (int q_ = 0; q_ < 10; ++q_) g_lm_prof[blockIdx.x & 1023][q_] = lmp_acc[q_]; } while (0)
#else
#define LMP_DECL
#define LMP_MARK(slot) do {} while (0)
#define LMP_STORE() do {} while (0)
#endif
constexpr int kMaxEdges = 4096;   // edges per pose problem held in LDS

// exclusive scan over an NT-thread block; s_tmp >= NT/64 ints
template <int NT = kNT>
__device__ int block_excl_scan_geom(int v, int* s_tmp, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
    }
    if (lane == 63) s_tmp[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < NT / 64; ++w) {
        if (w < wave) base += s_tmp[w];
        tot += s_tmp[w];
    }
    __syncthreads();
    if (total) *total = tot;
    return base + incl - v;
}

// OpenCV JacobiSVDImpl_<double>, cv::RNG, hypot: yavo_cvsvd.h

// a wave-uniform double (the value of lane 0) in SGPRs
__device__ __forceinline__ double uni_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}


// OpenCV JacobiSVDImpl_<double>(At 9x9, W, Vt) (yavo_cvsvd.h cv_jacobi_svd_mn<9, 9, 9>, operation for operation) as
// getFundamentalMatrix uses it: only the row of Vt that OpenCV's descending sort of W leaves last is read
// (src/3DHandler.cc:104-106, F0 = V row 8), so U's normalisation, its FULL_UV completion (both write At only) and the
// sorted W itself are not formed.  The sort's swap sequence is replayed on the row indices, ties and NaNs included,
// so the row picked is the one OpenCV's swaps leave at position 8.  At, Vt and W are lane-private rows in LDS laid out
// [element][lane] (s[e * 64 + lane]): every access of a wave is one conflict-free ds_*_b64, and the rotation loops
// stay rolled (a 9 x 9 SVD unrolled into registers is ~10k instructions, more than the instruction cache).
__device__ void cv_svd9_last_v(double* sA, double* sV, double* sW, double out[9]) {
    constexpr int L = 64;  // lane stride of one element
    const double eps = DBL_EPSILON * 10;
    for (int i = 0; i < 9; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            const double t = sA[(i * 9 + k) * L];
            sd += t * t;
        }
        sW[i * L] = sd;
#pragma unroll
        for (int k = 0; k < 9; k++) sV[(i * 9 + k) * L] = i == k ? 1.0 : 0.0;
    }
    for (int iter = 0; iter < 30; iter++) {  // max_iter = max(m, 30)
        bool changed = false;
        for (int i = 0; i < 8; i++) {
            double* Ai = sA + i * 9 * L;
            double* Vi = sV + i * 9 * L;
            for (int j = i + 1; j < 9; j++) {
                double* Aj = sA + j * 9 * L;
                double ai[9], aj[9];
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    ai[k] = Ai[k * L];
                    aj[k] = Aj[k * L];
                }
                double a = sW[i * L], p = 0, b = sW[j * L];
#pragma unroll
                for (int k = 0; k < 9; k++) p += ai[k] * aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double c, s;
                const double beta = a - b, gamma = cv_hypot(p, beta);
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    const double t0 = c * ai[k] + s * aj[k];
                    const double t1 = -s * ai[k] + c * aj[k];
                    Ai[k * L] = t0;
                    Aj[k * L] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                sW[i * L] = a;
                sW[j * L] = b;
                changed = true;
                double* Vj = sV + j * 9 * L;
                double vi[9], vj[9];
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    vi[k] = Vi[k * L];
                    vj[k] = Vj[k * L];
                }
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    Vi[k * L] = c * vi[k] + s * vj[k];
                    Vj[k * L] = -s * vi[k] + c * vj[k];
                }
            }
        }
        if (!changed) break;
    }
    // W[i] = |row i of At|, then OpenCV's selection sort (descending, first maximum) on (W, row index)
    double w[9];
    int idx[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            const double t = sA[(i * 9 + k) * L];
            sd += t * t;
        }
        w[i] = sqrt(sd);
        idx[i] = i;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        int j = i;
        double wj = w[i];
        int xj = idx[i];
#pragma unroll
        for (int k = i + 1; k < 9; k++)
            if (wj < w[k]) {
                j = k;
                wj = w[k];
                xj = idx[k];
            }
        // swap positions i and j (a no-op when j == i)
        const double wi = w[i];
        const int xi = idx[i];
#pragma unroll
        for (int k = i + 1; k < 9; k++)
            if (k == j) {
                w[k] = wi;
                idx[k] = xi;
            }
        w[i] = wj;
        idx[i] = xj;
    }
    const double* Vr = sV + idx[8] * 9 * L;
#pragma unroll
    for (int k = 0; k < 9; k++) out[k] = Vr[k * L];
}

// getFundamentalMatrix (src/3DHandler.cc:50-142) on 8 correspondences pts[8][4] = (x1, y1, x2, y2); sA / sV / sW:
// this lane's LDS rows of cv_svd9_last_v
__device__ void fundamental_8pt(const double* pts, double* F, double* sA, double* sV, double* sW) {
    constexpr int L = 64;
    const int n = 8;
    double xs[4][8];
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) xs[q][i] = pts[4 * i + q];
    double N[2][9];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        const double* x = xs[2 * v];
        const double* y = xs[2 * v + 1];
        double mx = 0.0, my = 0.0;
        for (int i = 0; i < n; ++i) mx += x[i];
        mx /= n;
        for (int i = 0; i < n; ++i) my += y[i];
        my /= n;
        double scaleDenom = 0.0;
        for (int i = 0; i < n; i++) {
            double xh = x[i] - mx, yh = y[i] - my;
            scaleDenom += sqrt(xh * xh + yh * yh);
        }
        double scale = sqrt(2.0) / (scaleDenom / n);
        double* M = N[v];
        M[0] = scale; M[1] = 0; M[2] = -scale * mx;
        M[3] = 0; M[4] = scale; M[5] = -scale * my;
        M[6] = 0; M[7] = 0; M[8] = 1;
    }
    double A[8][9];
#pragma unroll
    for (int i = 0; i < n; i++) {
        const double* N1 = N[0];
        const double* N2 = N[1];
        double nx1 = N1[0] * xs[0][i] + N1[1] * xs[1][i] + N1[2] * 1.0;
        double ny1 = N1[3] * xs[0][i] + N1[4] * xs[1][i] + N1[5] * 1.0;
        double nx2 = N2[0] * xs[2][i] + N2[1] * xs[3][i] + N2[2] * 1.0;
        double ny2 = N2[3] * xs[2][i] + N2[4] * xs[3][i] + N2[5] * 1.0;
        A[i][0] = nx1 * nx2; A[i][1] = nx1 * ny2; A[i][2] = nx1;
        A[i][3] = ny1 * nx2; A[i][4] = ny1 * ny2; A[i][5] = ny1;
        A[i][6] = nx2; A[i][7] = ny2; A[i][8] = 1;
    }
    // AtA = A^T A (symmetric); _SVDcompute transposes it into temp_a
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < n; ++k) s += A[k][i] * A[k][j];
            sA[(j * 9 + i) * L] = s;
        }
    double F0[9], A3[9], V3[9], w3[3];
    cv_svd9_last_v(sA, sV, sW, F0);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A3[i * 3 + j] = F0[j * 3 + i];
    cv_jacobi_svd<3>(A3, w3, V3);
    double U[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) U[i * 3 + j] = A3[j * 3 + i];
    w3[2] = 0;
    double D[9] = {w3[0], 0, 0, 0, w3[1], 0, 0, 0, w3[2]};
    double T[9];
    mm3(U, D, T);
    mm3(T, V3, F0);
    const double* N1 = N[0];
    const double* N2 = N[1];
    double N2t[9] = {N2[0], N2[3], N2[6], N2[1], N2[4], N2[7], N2[2], N2[5], N2[8]};
    mm3(N2t, F0, T);
    mm3(T, N1, F0);
    double inv = 1. / F0[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) F[i] = F0[i] * inv + 0.0;
}

__device__ __forceinline__ double epipolar_error(const double* F, double x1, double y1, double x2, double y2) {
    double r0 = x2 * F[0] + y2 * F[3] + 1.0 * F[6];
    double r1 = x2 * F[1] + y2 * F[4] + 1.0 * F[7];
    double r2 = x2 * F[2] + y2 * F[5] + 1.0 * F[8];
    return r0 * x1 + r1 * y1 + r2 * 1.0;
}

// getFRANSAC (src/3DHandler.cc:145-195) in three launches, so a list's 400 hypotheses spread over the chip instead of
// one workgroup (round 3: 5.1 ms per 1,935-match list, the 9 x 9 SVDs in scratch):
//   f_hyp_kernel    one lane per hypothesis, 64 per workgroup: its 8 sampled matches -> F (getFundamentalMatrix)
//   f_count_kernel  one wave per hypothesis, lanes over the matches: inliers |p2^T F p1| < thr (exact integer counts,
//                   so the order of the partial counts does not matter)
//   f_select_kernel one wave per list: the most inliers, then the first hypothesis (the reference's strict '>' in
//                   hypothesis order), its F, the count and `found`
constexpr int kFHypWG = 64;
constexpr int kFCountWaves = 4;

__global__ __launch_bounds__(kFHypWG) void f_hyp_kernel(const yv_match* __restrict__ matches, int64_t list_stride,
                                                        const int32_t* __restrict__ counts,
                                                        const int32_t* __restrict__ samples, int64_t sample_stride,
                                                        int iters, double* __restrict__ ws_F) {
    __shared__ double s_A[81 * kFHypWG], s_V[81 * kFHypWG], s_W[9 * kFHypWG];
    const int list = blockIdx.y, lane = threadIdx.x;
    const int h = blockIdx.x * kFHypWG + lane;
    int n = counts[list];
    if (n > kMaxKp) n = kMaxKp;
    if (n < 8 || h >= iters) return;  // no barriers below: lanes leave independently
    const yv_match* m = matches + (int64_t)list * list_stride;
    const int32_t* smp = samples + (int64_t)list * sample_stride + 8 * (int64_t)h;
    double pts8[32];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        int idx = smp[j];
        idx = idx < 0 ? 0 : (idx >= n ? n - 1 : idx);
        pts8[4 * j + 0] = (double)m[idx].pt1.x;
        pts8[4 * j + 1] = (double)m[idx].pt1.y;
        pts8[4 * j + 2] = (double)m[idx].pt2.x;
        pts8[4 * j + 3] = (double)m[idx].pt2.y;
    }
    double Fh[9];
    fundamental_8pt(pts8, Fh, s_A + lane, s_V + lane, s_W + lane);
    double* o = ws_F + ((int64_t)list * iters + h) * 9;
#pragma unroll
    for (int q = 0; q < 9; ++q) o[q] = Fh[q];
}

__global__ __launch_bounds__(64 * kFCountWaves) void f_count_kernel(const yv_match* __restrict__ matches,
                                                                    int64_t list_stride,
                                                                    const int32_t* __restrict__ counts, int iters,
                                                                    double thr, const double* __restrict__ ws_F,
                                                                    int32_t* __restrict__ ws_cnt) {
    const int list = blockIdx.y, lane = threadIdx.x & 63;
    const int h = blockIdx.x * kFCountWaves + (threadIdx.x >> 6);
    int n = counts[list];
    if (n > kMaxKp) n = kMaxKp;
    if (n < 8 || h >= iters) return;
    const double* Fp = ws_F + ((int64_t)list * iters + h) * 9;
    double F[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) F[q] = uni_f64(Fp[q]);  // wave-uniform: the hypothesis' F in SGPRs
    const yv_match* m = matches + (int64_t)list * list_stride;
    int cnt = 0;
    for (int k = lane; k < n; k += 64) {
        const yv_match& mk = m[k];
        const double e = epipolar_error(F, (double)mk.pt1.x, (double)mk.pt1.y, (double)mk.pt2.x, (double)mk.pt2.y);
        cnt += __popcll(__ballot(fabs(e) < thr));
    }
    if (lane == 0) ws_cnt[(int64_t)list * iters + h] = cnt;
}

__global__ __launch_bounds__(64) void f_select_kernel(const int32_t* __restrict__ counts, int iters,
                                                      const double* __restrict__ ws_F,
                                                      const int32_t* __restrict__ ws_cnt, double* __restrict__ F_out,
                                                      int32_t* __restrict__ max_inliers, int32_t* __restrict__ found) {
    const int list = blockIdx.x, lane = threadIdx.x;
    int n = counts[list];
    if (n > kMaxKp) n = kMaxKp;
    if (n < 8) {  // "Not enough matches": return false, F untouched
        if (lane == 0) found[list] = 0;
        return;
    }
    // (count, -h) lexicographic maximum: hypotheses in order, strict '>' keeps the first best
    int bc = INT32_MIN, bh = 0x7fffffff;
    for (int h = lane; h < iters; h += 64) {
        const int c = ws_cnt[(int64_t)list * iters + h];
        if (c > bc) {  // h increases within a lane
            bc = c;
            bh = h;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int oc = __shfl_xor(bc, off, 64), oh = __shfl_xor(bh, off, 64);
        if (oc > bc || (oc == bc && oh < bh)) {
            bc = oc;
            bh = oh;
        }
    }
    if (lane == 0) {
        max_inliers[list] = bc;
        found[list] = 1;
    }
    if (iters > 0 && lane < 9) F_out[(int64_t)list * 9 + lane] = ws_F[((int64_t)list * iters + bh) * 9 + lane];
}

// Sophus SE3 (pose = {qx, qy, qz, qw, tx, ty, tz}): yavo_se3.h

// ------------------------------------------------------------------------------------------------
// triangulation (Eigen JacobiSVD 4x4, registers) and world2Camera
// ------------------------------------------------------------------------------------------------
struct JRot {
    double c, s;
};

__device__ __forceinline__ JRot make_jacobi(double x, double y, double z) {
    JRot r;
    double deno = 2 * fabs(y);
    if (deno < DBL_MIN) {
        r.c = 1; r.s = 0;
        return r;
    }
    double tau = (x - z) / deno;
    double w = sqrt(tau * tau + 1);
    double t = tau > 0 ? 1 / (tau + w) : 1 / (tau - w);
    double sign_t = t > 0 ? 1 : -1;
    double nn = 1 / sqrt(t * t + 1);
    // Eigen's y / |y|: exactly +-1 here (2|y| >= DBL_MIN, and the inputs are finite and scaled to <= 1), so the
    // sign is taken instead of an FP64 division (one of the seven per rotation); the products are unchanged
    r.s = -sign_t * copysign(1.0, y) * fabs(t) * nn;
    r.c = nn;
    return r;
}

// JacobiSVD<MatrixXd>(A 4x4 column-major): sv descending, V column-major.  false on non-finite input.
__device__ bool eigen_jacobi_svd4(const double (&Ain)[16], double (&sv)[4], double (&V)[16]) {
    constexpr int n = 4;
    double Wk[16];
    double scale = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        double a = fabs(Ain[i]);
        if (a != a) return false;
        if (a > scale) scale = a;
    }
    if (!isfinite(scale)) return false;
    if (scale == 0) scale = 1;
#pragma unroll
    for (int i = 0; i < 16; ++i) Wk[i] = Ain[i] / scale;
#pragma unroll
    for (int i = 0; i < 16; ++i) V[i] = (i % 5 == 0) ? 1.0 : 0.0;
    const double considerAsZero = DBL_MIN, precision = 2 * DBL_EPSILON;
    double maxDiag = 0;
#pragma unroll
    for (int i = 0; i < n; ++i) {
        double a = fabs(Wk[i + i * n]);
        if (a > maxDiag) maxDiag = a;
    }
    bool finished = false;
    int guard = 0;
    while (!finished && guard < 10000) {
        finished = true;
        ++guard;
#pragma unroll
        for (int p = 1; p < n; ++p)
#pragma unroll
            for (int q = 0; q < p; ++q) {
                double threshold = considerAsZero > precision * maxDiag ? considerAsZero : precision * maxDiag;
                if (fabs(Wk[p + q * n]) > threshold || fabs(Wk[q + p * n]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd
                    double m00 = Wk[p + p * n], m01 = Wk[p + q * n], m10 = Wk[q + p * n], m11 = Wk[q + q * n];
                    JRot rot1;
                    double t = m00 + m11;
                    double d = m10 - m01;
                    if (fabs(d) < DBL_MIN) {
                        rot1.s = 0; rot1.c = 1;
                    } else {
                        double u = t / d;
                        double tmp = sqrt(1 + u * u);
                        rot1.s = 1 / tmp;
                        rot1.c = u / tmp;
                    }
                    if (!(rot1.c == 1 && rot1.s == 0)) {
                        double a0 = m00, b0 = m10, a1 = m01, b1 = m11;
                        m00 = rot1.c * a0 + rot1.s * b0;
                        m10 = -rot1.s * a0 + rot1.c * b0;
                        m01 = rot1.c * a1 + rot1.s * b1;
                        m11 = -rot1.s * a1 + rot1.c * b1;
                    }
                    JRot jr = make_jacobi(m00, m01, m11);
                    JRot jl;
                    {
                        const double jtc = jr.c, jts = -jr.s;
                        jl.c = rot1.c * jtc - rot1.s * jts;
                        jl.s = rot1.c * jts + rot1.s * jtc;
                    }
                    // work.applyOnTheLeft(p, q, jl): rows p, q
                    if (!(jl.c == 1 && jl.s == 0)) {
#pragma unroll
                        for (int i = 0; i < n; ++i) {
                            double xi = Wk[p + i * n], yi = Wk[q + i * n];
                            Wk[p + i * n] = jl.c * xi + jl.s * yi;
                            Wk[q + i * n] = -jl.s * xi + jl.c * yi;
                        }
                    }
                    // work.applyOnTheRight(p, q, jr) and V.applyOnTheRight(p, q, jr): rotation by jr^T
                    const double tc = jr.c, ts = -jr.s;
                    if (!(tc == 1 && ts == 0)) {
#pragma unroll
                        for (int i = 0; i < n; ++i) {
                            double xi = Wk[i + p * n], yi = Wk[i + q * n];
                            Wk[i + p * n] = tc * xi + ts * yi;
                            Wk[i + q * n] = -ts * xi + tc * yi;
                        }
#pragma unroll
                        for (int i = 0; i < n; ++i) {
                            double xi = V[i + p * n], yi = V[i + q * n];
                            V[i + p * n] = tc * xi + ts * yi;
                            V[i + q * n] = -ts * xi + tc * yi;
                        }
                    }
                    double aa = fabs(Wk[p + p * n]), bb = fabs(Wk[q + q * n]);
                    double mx = aa > bb ? aa : bb;
                    if (mx > maxDiag) maxDiag = mx;
                }
            }
    }
#pragma unroll
    for (int i = 0; i < n; ++i) sv[i] = fabs(Wk[i + i * n]) * scale;
#pragma unroll
    for (int i = 0; i < n; ++i) {
        int pos = i;
        double mx = sv[i];
#pragma unroll
        for (int k = i + 1; k < n; ++k)
            if (sv[k] > mx) { mx = sv[k]; pos = k; }
        if (mx == 0) break;
        if (pos != i) {
            // swap sv[i] <-> sv[pos] and V columns, static indices only
#pragma unroll
            for (int k = i + 1; k < n; ++k)
                if (k == pos) {
                    double t = sv[i]; sv[i] = sv[k]; sv[k] = t;
#pragma unroll
                    for (int r = 0; r < n; ++r) { t = V[r + k * n]; V[r + k * n] = V[r + i * n]; V[r + i * n] = t; }
                }
        }
    }
    return true;
}

// LoopHandler::triangulation of one match (pixel2camera of both integer pixels, DLT rows, Eigen JacobiSVD);
// returns success (s4/s3 < 1e-2) && Z > 0, the triangulate2View acceptance test (src/LoopHandler.cc:676)
__device__ bool triangulate_px(int x1, int y1, int x2, int y2, const double* Ta, const double* Tb,
                               const double* K, double* Xo) {
    const double K0 = K[0], K2 = K[2], K4 = K[4], K5 = K[5];
    const double pa[2] = {((double)x1 - K2) * 1.0 / K0, ((double)y1 - K5) * 1.0 / K4};
    const double pb[2] = {((double)x2 - K2) * 1.0 / K0, ((double)y2 - K5) * 1.0 / K4};
    double A[16];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        const double* T = v == 0 ? Ta : Tb;
        const double* pp = v == 0 ? pa : pb;
        double R[9];
        quat_to_R(T, R);
        double mm[12];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            mm[4 * r] = R[3 * r]; mm[4 * r + 1] = R[3 * r + 1]; mm[4 * r + 2] = R[3 * r + 2]; mm[4 * r + 3] = T[4 + r];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            A[(2 * v) + 4 * j] = pp[0] * mm[8 + j] - mm[j];
            A[(2 * v + 1) + 4 * j] = pp[1] * mm[8 + j] - mm[4 + j];
        }
    }
    double sv[4], V[16];
    double X0 = NAN, X1 = NAN, X2 = NAN;
    bool s = false;
    if (eigen_jacobi_svd4(A, sv, V)) {
        X0 = V[0 + 12] / V[3 + 12];
        X1 = V[1 + 12] / V[3 + 12];
        X2 = V[2 + 12] / V[3 + 12];
        s = sv[3] / sv[2] < 1e-2;
    }
    Xo[0] = X0;
    Xo[1] = X1;
    Xo[2] = X2;
    return s && X2 > 0;
}

__global__ __launch_bounds__(256) void triangulate_kernel(const yv_match* __restrict__ m, int n, const double* __restrict__ poses /*[2][7]*/,
                                   const double* __restrict__ K, double* __restrict__ Xw, uint8_t* __restrict__ ok,
                                   int32_t* __restrict__ n_ok) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool good = false;
    if (i < n) {
        good = triangulate_px(m[i].pt1.x, m[i].pt1.y, m[i].pt2.x, m[i].pt2.y, poses, poses + 7, K, Xw + 3 * i);
        ok[i] = good ? 1 : 0;
    }
    if (!n_ok) return;  // the host counts ok[] (yv_triangulate)
    const uint64_t bal = __ballot(good);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(n_ok, (int32_t)__popcll(bal));
}

__global__ void world2camera_kernel(const double* __restrict__ X, int n, const double* __restrict__ T,
                                    const double* __restrict__ K, double* __restrict__ out) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    double R[9], M[12], KM[12];
    quat_to_R(T, R);
    for (int i = 0; i < 3; ++i) {
        M[4 * i] = R[3 * i]; M[4 * i + 1] = R[3 * i + 1]; M[4 * i + 2] = R[3 * i + 2]; M[4 * i + 3] = T[4 + i];
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) KM[4 * i + j] = K[3 * i] * M[j] + K[3 * i + 1] * M[4 + j] + K[3 * i + 2] * M[8 + j];
    for (int i = 0; i < 3; ++i)
        out[3 * k + i] = KM[4 * i] * X[3 * k] + KM[4 * i + 1] * X[3 * k + 1] + KM[4 * i + 2] * X[3 * k + 2] + KM[4 * i + 3] * 1.0;
}

// ------------------------------------------------------------------------------------------------
// Eigen LDLT 6x6 (lane 0)
// ------------------------------------------------------------------------------------------------
// Eigen::LDLT<Matrix6d> (diagonal pivoting, Eigen's ldlt_inplace + solve) -- variant 0 subtracts the
// GEMV update term by term (the dynamic-size path g2o's LinearSolverDense takes), variant 1 forms the dot
// first (fixed-size path, test.cc's GN).  Fully unrolled: every index is a compile-time constant and the
// pivot swaps are predicated swaps, so the 6x6 factor lives in registers (a runtime-indexed private array
// would go to scratch memory, one dependent round trip per access).

template <int variant>
__device__ bool ldlt6_solve(const double* Hin, const double* b, double* x) {
    double m[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) m[i] = Hin[i];
    constexpr int n = 6;
    int tr[6];
    int sign = 0;
    int found_zero_pivot = 0;
    bool stop = false;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        if (!stop) {
            int big = k;
            double bv = fabs(m[k * 7]);
#pragma unroll
            for (int i = k + 1; i < n; ++i)
                if (fabs(m[i * 7]) > bv) {
                    bv = fabs(m[i * 7]);
                    big = i;
                }
            tr[k] = big;
#pragma unroll
            for (int c = k + 1; c < n; ++c) {
                if (c == big) {
                    // rows/cols k <-> c of the lower triangle (Eigen's ldlt_inplace swap sequence)
#pragma unroll
                    for (int j = 0; j < k; ++j) {
                        const double t = m[k * 6 + j]; m[k * 6 + j] = m[c * 6 + j]; m[c * 6 + j] = t;
                    }
#pragma unroll
                    for (int j = 0; j < n - c - 1; ++j) {
                        const double t = m[(c + 1 + j) * 6 + k]; m[(c + 1 + j) * 6 + k] = m[(c + 1 + j) * 6 + c];
                        m[(c + 1 + j) * 6 + c] = t;
                    }
                    { const double t = m[k * 7]; m[k * 7] = m[c * 7]; m[c * 7] = t; }
#pragma unroll
                    for (int i = k + 1; i < c; ++i) {
                        const double t = m[i * 6 + k]; m[i * 6 + k] = m[c * 6 + i]; m[c * 6 + i] = t;
                    }
                }
            }
            if (k > 0) {
                double temp[6];
#pragma unroll
                for (int j = 0; j < k; ++j) temp[j] = m[j * 7] * m[k * 6 + j];
                double dot = m[k * 6 + 0] * temp[0];
#pragma unroll
                for (int j = 1; j < k; ++j) dot = dot + m[k * 6 + j] * temp[j];
                m[k * 7] -= dot;
#pragma unroll
                for (int i = k + 1; i < n; ++i) {
                    if (variant == 0) {
                        double acc = m[i * 6 + k];
#pragma unroll
                        for (int j = 0; j < k; ++j) acc = acc - m[i * 6 + j] * temp[j];
                        m[i * 6 + k] = acc;
                    } else {
                        double d = m[i * 6 + 0] * temp[0];
#pragma unroll
                        for (int j = 1; j < k; ++j) d = d + m[i * 6 + j] * temp[j];
                        m[i * 6 + k] = m[i * 6 + k] - d;
                    }
                }
            }
            const double akk = m[k * 7];
            const int valid = fabs(akk) > 0;
            if (k == 0 && !valid) {
                sign = 0;
#pragma unroll
                for (int j = 0; j < n; ++j) tr[j] = j;
                stop = true;
            } else {
                if (k + 1 < n && valid) {
#pragma unroll
                    for (int i = k + 1; i < n; ++i) m[i * 6 + k] /= akk;
                }
                if (!(found_zero_pivot && valid) && !valid) found_zero_pivot = 1;
                if (sign == 1) { if (akk < 0) sign = 3; }
                else if (sign == 2) { if (akk > 0) sign = 3; }
                else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
            }
        } else {
            tr[k] = k;
        }
    }
    const bool positive = (sign == 1 || sign == 0);
    double v[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = b[i];
    // v = P b: transpositions applied in order, swap(v[k], v[tr[k]]) with tr[k] >= k
#pragma unroll
    for (int k = 0; k < n; ++k) {
#pragma unroll
        for (int c = k + 1; c < n; ++c)
            if (tr[k] == c) { const double t = v[k]; v[k] = v[c]; v[c] = t; }
    }
#pragma unroll
    for (int j = 0; j < n; ++j)
#pragma unroll
        for (int i = j + 1; i < n; ++i) v[i] = v[i] - m[i * 6 + j] * v[j];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        if (fabs(m[i * 7]) > DBL_MIN) v[i] /= m[i * 7];
        else v[i] = 0;
    }
#pragma unroll
    for (int j = n - 1; j >= 0; --j)
#pragma unroll
        for (int i = 0; i < j; ++i) v[i] = v[i] - m[j * 6 + i] * v[j];
#pragma unroll
    for (int k = n - 1; k >= 0; --k) {
#pragma unroll
        for (int c = k + 1; c < n; ++c)
            if (tr[k] == c) { const double t = v[k]; v[k] = v[c]; v[c] = t; }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = v[i];
    return positive;
}

// The same Eigen LDLT for a symmetric system held in LDS (H + lambda I, the LM trial's damped matrix).
// Eigen's pivot at step k is the largest |diagonal| among rows k..5, and those diagonal entries are still
// the original ones (a row's diagonal is only updated at its own step), so the whole transposition
// sequence follows from the six diagonal values alone.  Pivoted LDLT then performs exactly the arithmetic
// of unpivoted LDLT on P H P^T: the permutation is resolved first, P H P^T's lower triangle is gathered
// from LDS, and the factorization runs straight-line in registers.
// Hf the full symmetric 6x6 (row-major), bs the right-hand side, xs the solution (all LDS); P b and P^T v are indexed
// LDS accesses.
template <int variant>
__device__ bool ldlt6_solve_lds(const double* Hf, double lambda, const double* bs, double* xs) {
    constexpr int n = 6;
    double dg[6];
    int id[6];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        dg[i] = Hf[i * 7] + lambda;
        id[i] = i;
    }
#pragma unroll
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = fabs(dg[k]);
#pragma unroll
        for (int i = k + 1; i < n; ++i)
            if (fabs(dg[i]) > bv) {
                bv = fabs(dg[i]);
                big = i;
            }
        const double dk = dg[k];
        const int ik = id[k];
#pragma unroll
        for (int c = k + 1; c < n; ++c) {
            const bool sw = c == big;
            dg[k] = sw ? dg[c] : dg[k];
            id[k] = sw ? id[c] : id[k];
            dg[c] = sw ? dk : dg[c];
            id[c] = sw ? ik : id[c];
        }
    }
    const bool zero0 = !(fabs(dg[0]) > 0);  // Eigen's k == 0 early exit: no transposition, no factorization
    if (zero0) {
#pragma unroll
        for (int i = 0; i < n; ++i) {
            id[i] = i;
            dg[i] = Hf[i * 7] + lambda;
        }
    }
    double m[36];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        const double* row = Hf + id[i] * 6;
#pragma unroll
        for (int j = 0; j < i; ++j) m[i * 6 + j] = row[id[j]];
        m[i * 7] = dg[i];
    }
    int sign = 0;
    int found_zero_pivot = 0;
    if (!zero0) {
#pragma unroll
        for (int k = 0; k < n; ++k) {
            if (k > 0) {
                double temp[6];
#pragma unroll
                for (int j = 0; j < k; ++j) temp[j] = m[j * 7] * m[k * 6 + j];
                double dot = m[k * 6 + 0] * temp[0];
#pragma unroll
                for (int j = 1; j < k; ++j) dot = dot + m[k * 6 + j] * temp[j];
                m[k * 7] -= dot;
#pragma unroll
                for (int i = k + 1; i < n; ++i) {
                    if (variant == 0) {
                        double acc = m[i * 6 + k];
#pragma unroll
                        for (int j = 0; j < k; ++j) acc = acc - m[i * 6 + j] * temp[j];
                        m[i * 6 + k] = acc;
                    } else {
                        double d = m[i * 6 + 0] * temp[0];
#pragma unroll
                        for (int j = 1; j < k; ++j) d = d + m[i * 6 + j] * temp[j];
                        m[i * 6 + k] = m[i * 6 + k] - d;
                    }
                }
            }
            const double akk = m[k * 7];
            const int valid = fabs(akk) > 0;
            if (k + 1 < n && valid) {
#pragma unroll
                for (int i = k + 1; i < n; ++i) m[i * 6 + k] /= akk;
            }
            if (!(found_zero_pivot && valid) && !valid) found_zero_pivot = 1;
            if (sign == 1) { if (akk < 0) sign = 3; }
            else if (sign == 2) { if (akk > 0) sign = 3; }
            else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
        }
    }
    const bool positive = (sign == 1 || sign == 0);
    double v[6];
#pragma unroll
    for (int i = 0; i < n; ++i) v[i] = bs[id[i]];  // v = P b
#pragma unroll
    for (int j = 0; j < n; ++j)
#pragma unroll
        for (int i = j + 1; i < n; ++i) v[i] = v[i] - m[i * 6 + j] * v[j];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        if (fabs(m[i * 7]) > DBL_MIN) v[i] /= m[i * 7];
        else v[i] = 0;
    }
#pragma unroll
    for (int j = n - 1; j >= 0; --j)
#pragma unroll
        for (int i = 0; i < j; ++i) v[i] = v[i] - m[j * 6 + i] * v[j];
#pragma unroll
    for (int i = 0; i < n; ++i) xs[id[i]] = v[i];  // x = P^T v
    return positive;
}

// ------------------------------------------------------------------------------------------------
// pose-only LM (g2o semantics) and GN, one workgroup per problem
// ------------------------------------------------------------------------------------------------
// the edge's error from its camera-frame point pc = T X (computeError: K pc, projected)
__device__ __forceinline__ void edge_error_pc(const double* pc, const double* K, const double* meas, double* e) {
    double u0 = K[0] * pc[0] + K[1] * pc[1] + K[2] * pc[2];
    double u1 = K[3] * pc[0] + K[4] * pc[1] + K[5] * pc[2];
    double u2 = K[6] * pc[0] + K[7] * pc[1] + K[8] * pc[2];
    e[0] = meas[0] - u0 / u2;
    e[1] = meas[1] - u1 / u2;
}

__device__ __forceinline__ void edge_error(const double* T, const double* K, const double* X, const double* meas,
                                           double* e) {
    double pc[3];
    se3_act(T, X, pc);
    edge_error_pc(pc, K, meas, e);
}

// linearizeOplus's 2 x 6 Jacobian from the same pc (computeError and linearizeOplus both form T X at one estimate:
// one evaluation serves both, the same operations)
__device__ __forceinline__ void edge_jacobian_pc(const double* pc, const double* K, double* J) {
    double fx = K[0], fy = K[4];
    double x = pc[0], y = pc[1], z = pc[2];
    double zinv = 1.0 / (z + 1e-18);
    double zinv2 = zinv * zinv;
    J[0] = -fx * zinv; J[1] = 0; J[2] = fx * x * zinv2; J[3] = fx * x * y * zinv2;
    J[4] = -fx - fx * x * x * zinv2; J[5] = fx * y * zinv;
    J[6] = 0; J[7] = -fy * zinv; J[8] = fy * y * zinv2; J[9] = fy + fy * y * y * zinv2;
    J[10] = -fy * x * y * zinv2; J[11] = -fy * x * zinv;
}

__device__ __forceinline__ double huber_rho(double e2, double* rho1) {
    const double delta = 1.0, dsqr = delta * delta;
    if (e2 <= dsqr) {
        *rho1 = 1.;
        return e2;
    }
    double sqrte = sqrt(e2);
    *rho1 = delta / sqrte;
    return 2 * sqrte * delta - dsqr;
}

// Tree sum of per-thread partials in the oracle's order (sum_mode log2(NT) - 7): p[t] += p[t + off] for
// off = NT/2 .. 64 (across waves, through LDS), then 32 .. 1 inside wave 0 (shuffles).  part[] holds this
// thread's nv partials; totals land in out[0..nv) (LDS), visible after the trailing barrier.
// red: >= nv * NT/2 doubles of LDS.
template <int NV, int NT = kNT>
__device__ void tree_reduce(double (&part)[NV], double* red, double* out, unsigned long long* t_sync = nullptr) {
    const int tid = threadIdx.x;
    __syncthreads();
#ifdef YAVO_LM_PROFILE
    if (t_sync) *t_sync = __builtin_readcyclecounter();
#endif
#pragma unroll
    for (int off = NT / 2; off >= 128; off >>= 1) {
        if (tid >= off && tid < 2 * off) {
#pragma unroll
            for (int v = 0; v < NV; ++v) red[v * (NT / 2) + (tid - off)] = part[v];
        }
        __syncthreads();
        if (tid < off) {
#pragma unroll
            for (int v = 0; v < NV; ++v) part[v] = part[v] + red[v * (NT / 2) + tid];
        }
        __syncthreads();
    }
    if (tid >= 64 && tid < 128) {
#pragma unroll
        for (int v = 0; v < NV; ++v) red[v * (NT / 2) + (tid - 64)] = part[v];
    }
    __syncthreads();
    if (tid < 64) {
        // wave 0: the NV independent shuffle trees advance together (all NV shuffles of a level are issued
        // before the adds), so one LDS-permute latency is paid per level instead of per value and level
        double x[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) x[v] = part[v] + red[v * (NT / 2) + tid];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            double y[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) y[v] = __shfl_down(x[v], off, 64);
#pragma unroll
            for (int v = 0; v < NV; ++v) x[v] = x[v] + y[v];
        }
        if (tid == 0) {
#pragma unroll
            for (int v = 0; v < NV; ++v) out[v] = x[v];
        }
    }
    __syncthreads();
}

// The pose LM's reduction of NV per-thread partials over NT = 64 W threads (oracle sum_mode 4 + log2(W)): the
// halving tree p[l] += p[l + off], off = 32 .. 1, inside each wave, then the W wave totals left to right.
// Inside the wave it runs as a reduce-scatter: at the level with offset off the two lanes l, l ^ off split their
// n live values, each keeping ceil(n / 2) of them (the lane with bit off clear the lower half) and adding its
// partner's copy of those -- one shuffle per kept value instead of one per value, 29 instead of 168 exchanges for
// 28 values. Each value's partials still meet in the tree's pairs and order (the kept sum is own + partner, and
// IEEE addition commutes, so the lane with bit off set computes the lower lane's bits). After the six levels the
// lane pair (l, l ^ 1) holds value v(l) = 14 b5 + 7 b4 + 4 b3 + 2 b2 + b1 (28 values: v < 28 is real, the rest
// are padding slots).
// The exchanges run on the VALU side (yavo_xlane.h): permlane swaps at offsets 32 / 16, DPP below.
template <int N, int OFF>
__device__ __forceinline__ void rs_level(const double* in, double* out, int lane, int& v) {
    constexpr int h = (N + 1) / 2;
    const bool up = (lane & OFF) != 0;
#pragma unroll
    for (int j = 0; j < h; ++j) {
        double lo = in[j];
        double hi = (h + j < N) ? in[h + j] : 0.0;
        if constexpr (OFF >= 16) {
            xl::swap_halves_f64<OFF>(lo, hi);  // {own kept, partner's} in some order: the sum commutes
            out[j] = lo + hi;
        } else {
            const double keep = up ? hi : lo;
            out[j] = keep + xl::xor_row_f64<OFF>(up ? lo : hi);
        }
    }
    if (up) v += h;
}

// flag (optional): read by every thread after the reduction's first barrier and returned (the pass's literal-form
// flag rides on the reduction's barriers instead of a barrier of its own); thread 0 clears it after the last one.
template <int NV, int NT>
__device__ int lm_reduce(double (&part)[NV], double* red /* >= NV * NT / 64 */, double* out,
                         unsigned long long* t_sync = nullptr, int* flag = nullptr) {
    static_assert(NV == 28, "the reduce-scatter schedule is written for 28 values");
    constexpr int W = NT / 64;
    static_assert(W >= 2, "the flag hand-off needs the two barriers of the multi-wave form");
#ifdef YAVO_LM_PROFILE
    if (t_sync) *t_sync = __builtin_readcyclecounter();
#endif
    const int tid = threadIdx.x, lane = tid & 63;
    int v = 0;
    double a14[14], a7[7], a4[4], a2[2], a1[1];
    rs_level<28, 32>(part, a14, lane, v);
    rs_level<14, 16>(a14, a7, lane, v);
    rs_level<7, 8>(a7, a4, lane, v);
    rs_level<4, 4>(a4, a2, lane, v);
    rs_level<2, 2>(a2, a1, lane, v);
    const double tot = a1[0] + xl::xor_row_f64<1>(a1[0]);
    const bool owner = v < NV && (lane & 1) == 0;
    if (owner) red[(tid >> 6) * NV + v] = tot;
    __syncthreads();
    const int f = flag ? *flag : 0;
    if (tid < NV) {
        double q = red[tid];
#pragma unroll
        for (int w = 1; w < W; ++w) q = q + red[w * NV + tid];
        out[tid] = q;
    }
    __syncthreads();
    if (flag && tid == 0 && f) *flag = 0;  // every thread read it before the barrier above; set again next pass
    return f;
}

struct LMShared {
    double T[7], Tbak[7], Tlast[7], K[9];
    double sys[28], x[6], vals[32];  // sys: {H lower packed (21), b (6), chi2} of the current iteration
    double Hf[36];                     // the same H, full symmetric (the LDLT's gather source)
    double lambda, ni, currentChi, tempChi, rho;
    int flag;  // control broadcast from lane 0
    int hub;   // a Huber weight (c2 > delta^2 on a robust edge) was applied in some pass of the current round
    int lit;   // some edge of the current pass had a non-finite operand (lm_pass: the pass is redone literally)
};

constexpr int kLMVals = 28;  // 21 lower-triangle H entries + 6 b + 1 chi2

// The exact short form of one edge's J^T W J lower triangle and -J^T W e (see lm_pass), added to the partials.
__device__ __forceinline__ void lm_accumulate_short(double (&part)[28], const double* J, double w, const double* e) {
    double a[6], b[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        a[r] = J[r] * w;
        b[r] = J[6 + r] * w;
    }
    part[0] = part[0] + a[0] * J[0];
    part[2] = part[2] + b[1] * J[7];
#pragma unroll
    for (int r = 2; r < 6; ++r) {
        part[r * (r + 1) / 2 + 0] = part[r * (r + 1) / 2 + 0] + a[r] * J[0];
        part[r * (r + 1) / 2 + 1] = part[r * (r + 1) / 2 + 1] + b[r] * J[7];
#pragma unroll
        for (int c = 2; c <= r; ++c)
            part[r * (r + 1) / 2 + c] = part[r * (r + 1) / 2 + c] + (a[r] * J[c] + b[r] * J[6 + c]);
    }
    part[21] = part[21] + (-(a[0] * e[0]));
    part[22] = part[22] + (-(b[1] * e[1]));
#pragma unroll
    for (int r = 2; r < 6; ++r) part[21 + r] = part[21 + r] + (-(a[r] * e[0] + b[r] * e[1]));
}

// The literal form of one edge's contributions (rho' Omega with Omega = I spelt out: every product with the literal
// 0.0 / 1.0), added to partials held in a stack array: only the rare pass that meets a non-finite operand runs it
// (lm_pass), so its temporaries do not count against the hot loop's registers.
__device__ __noinline__ void lm_accumulate_literal(double* part, const double* J, double w, const double* e) {
#pragma unroll 1
    for (int r = 0; r < 6; ++r) {
        const double t0 = J[r] * w + J[6 + r] * 0.0;
        const double t1 = J[r] * 0.0 + J[6 + r] * w;
#pragma unroll 1
        for (int c = 0; c <= r; ++c) part[r * (r + 1) / 2 + c] = part[r * (r + 1) / 2 + c] + (t0 * J[c] + t1 * J[6 + c]);
        const double s0 = (w * J[r]) * 1.0 + (w * J[6 + r]) * 0.0;
        const double s1 = (w * J[r]) * 0.0 + (w * J[6 + r]) * 1.0;
        part[21 + r] = part[21 + r] + (-(s0 * e[0] + s1 * e[1]));
    }
}

// One edge at T: its error, robust chi2 and weight, and J.  Returns c2 > delta^2 on a robust edge (a Huber weight).
__device__ __forceinline__ void lm_edge(const double* T, const double* K, const double* xi, const double* mi, int rob,
                                        double* e, double& chi, double& w, double* J, bool& hub) {
    double pc[3];
    se3_act(T, xi, pc);
    edge_error_pc(pc, K, mi, e);
    const double c2 = e[0] * e[0] + e[1] * e[1];
    w = 1.0;
    chi = c2;
    // Huber only past delta: skipped by the whole wave when no lane needs it (a per-lane branch is if-converted
    // into an unconditional sqrt + division)
    hub = rob && c2 > 1.0;
    if (__any(hub)) {
        if (rob) chi = huber_rho(c2, &w);
    }
    edge_jacobian_pc(pc, K, J);
}

// One pass over the active edges at S.T: computeActiveErrors + activeRobustChi2 + buildSystem of g2o's
// BlockSolver (Huber-weighted J^T J lower triangle, -J^T W e, robust chi2), summed in the oracle's tree
// order into S.vals[0..28).  Also records S.Tlast (the estimate the active edges' errors refer to).
//
// g2o forms J^T (rho' Omega) J and -J^T (rho' Omega) e with Omega = I, i.e. products with the literal 0.0 / 1.0 of
// Omega, and J[1] = J[6] = 0 structurally.  With finite operands those products only contribute signed zeros, which
// cannot change a partial sum (a partial that starts at +0.0 never becomes -0.0, and p + (+-0) = p for p != 0), so the
// short form gives bit-identical sums.  A pass in which some edge has a non-finite operand is run again by the whole
// workgroup in the literal form (for every edge: bit-identical to the short form on the finite ones), with the
// partials on the stack; the hot loop carries only the short form (the literal form inside it raised the kernel's
// register demand by ~50 VGPRs).
template <int NT, typename UV>
__device__ __forceinline__ void lm_pass(LMShared& S, const int16_t* s_active, int na, const uint8_t* s_robust,
                                        const double* X, const UV* uv, double* s_red,
                                        unsigned long long* lmp = nullptr) {
    const int tid = threadIdx.x;
    __syncthreads();  // S.T written by lane 0
#ifdef YAVO_LM_PROFILE
    const unsigned long long p0 = __builtin_readcyclecounter();
#endif
    // the estimate and K are wave-uniform: held in SGPRs (16 doubles = 32 VGPRs fewer through the edge loop)
    double T[7], K[9];
#pragma unroll
    for (int q = 0; q < 7; ++q) T[q] = uni_f64(S.T[q]);
#pragma unroll
    for (int q = 0; q < 9; ++q) K[q] = uni_f64(S.K[q]);
    if (tid < 7) S.Tlast[tid] = S.T[tid];
    double part[kLMVals];
#pragma unroll
    for (int v = 0; v < kLMVals; ++v) part[v] = 0.0;
    bool literal = false;
    // the next edge's point / measurement / robust flag are loaded while this one is evaluated (the gathers
    // hit L2: their latency would otherwise be paid once per edge)
    double nx[5] = {0, 0, 0, 0, 0};
    int nrob = 0;
    if (tid < na) {
        const int i = s_active[tid];
        nx[0] = X[3 * i]; nx[1] = X[3 * i + 1]; nx[2] = X[3 * i + 2]; nx[3] = (double)uv[2 * i]; nx[4] = (double)uv[2 * i + 1];
        nrob = s_robust[i];
    }
    for (int a = tid; a < na; a += NT) {
        const double xi[3] = {nx[0], nx[1], nx[2]}, mi[2] = {nx[3], nx[4]};
        const int rob = nrob;
        if (a + NT < na) {
            const int i = s_active[a + NT];
            nx[0] = X[3 * i]; nx[1] = X[3 * i + 1]; nx[2] = X[3 * i + 2]; nx[3] = (double)uv[2 * i]; nx[4] = (double)uv[2 * i + 1];
            nrob = s_robust[i];
        }
        double e[2], J[12], chi, w;
        bool hub;
        lm_edge(T, K, xi, mi, rob, e, chi, w, J, hub);
        if (__any(hub) && (tid & 63) == 0) S.hub = 1;
        part[27] = part[27] + chi;
        const double fin = J[0] + J[2] + J[3] + J[4] + J[5] + J[7] + J[8] + J[9] + J[10] + J[11] + w + e[0] + e[1];
        literal |= !isfinite(fin);
        lm_accumulate_short(part, J, w, e);
    }
    if (literal) S.lit = 1;
#ifdef YAVO_LM_PROFILE
    const unsigned long long p1 = __builtin_readcyclecounter();
    unsigned long long ps = 0;
    const int lit = lm_reduce<kLMVals, NT>(part, s_red, S.vals, &ps, &S.lit);
    if (lmp) {
        const unsigned long long p2 = __builtin_readcyclecounter();
        lmp[0] += p1 - p0;
        lmp[1] += p2 - ps;  // the reduction proper
        lmp[8] += ps - p1;  // waiting at the first barrier for the other waves' edges
        lmp[9] += 1;        // passes (error + system evaluations)
    }
#else
    const int lit = lm_reduce<kLMVals, NT>(part, s_red, S.vals, nullptr, &S.lit);
#endif
    if (lit) {
        // the rare pass: every edge again in the literal form, partials on the stack, in the same order
        double lp[kLMVals];
        for (int v = 0; v < kLMVals; ++v) lp[v] = 0.0;
        for (int a = tid; a < na; a += NT) {
            const int i = s_active[a];
            const double xi[3] = {X[3 * i], X[3 * i + 1], X[3 * i + 2]}, mi[2] = {(double)uv[2 * i], (double)uv[2 * i + 1]};
            double e[2], J[12], chi, w;
            bool hub;
            lm_edge(T, K, xi, mi, s_robust[i], e, chi, w, J, hub);
            lp[27] = lp[27] + chi;
            lm_accumulate_literal(lp, J, w, e);
        }
#pragma unroll
        for (int v = 0; v < kLMVals; ++v) part[v] = lp[v];
        lm_reduce<kLMVals, NT>(part, s_red, S.vals);
    }
}

// Problem p owns edges [offsets[p], offsets[p+1]) (CSR) or, with counts != nullptr, [p*stride, p*stride +
// counts[p]) (the batch's fixed-stride track layout).  The prior is read from priors[p] and the estimate
// written to poses[p] (the two may alias).
// Register budget of the LM.  The 256-thread form (the batch of a step's 2048 tracks, beside top-K and BRIEF): 3 waves
// per SIMD = 168 VGPRs.  With the literal J^T Omega J form out of the edge loop (lm_pass) the hot loop fits without
// spills (the stack partials and the call of the rare literal pass are the kernel's only scratch), and two LM waves
// leave a SIMD 176 registers for BRIEF / top-K beside them instead of 48: 230.1 k -> 233.7 k frames/s, the LM itself
// 2.29 -> 2.12 ms per launch in the step (profiles/r06/c19).  The 512-thread form (one problem of the LoopHandler, the
// sequence's 20-track batches) keeps 2 waves per SIMD = 256: at 168 its single-problem latency rose ~9% (the pose LM
// 54 -> 60 ms of a 200-frame LoopHandler run, profiles/r06/c27).
template <int NT>
struct LMWaves {
    static constexpr int value = NT >= 512 ? 2 : 3;
};
#ifdef YAVO_LM_WPE
#define YAVO_LM_ATTR __attribute__((amdgpu_waves_per_eu(YAVO_LM_WPE)))
#else
#define YAVO_LM_ATTR __attribute__((amdgpu_waves_per_eu(LMWaves<NT>::value)))
#endif
template <int NT>
__device__ __forceinline__ void pose_lm_body(const int32_t* __restrict__ offsets, const int32_t* __restrict__ counts,
                                                      int stride, const double* __restrict__ Xall,
                                                      const double* __restrict__ uvall, const double* __restrict__ Kall,
                                                      const double* priors, double* poses,
                                                      uint8_t* __restrict__ outlier_all, int32_t* __restrict__ inliers,
                                                      int n_prob) {
    constexpr int CAP = kMaxEdges;
    __shared__ uint8_t s_level[CAP], s_out[CAP], s_robust[CAP];
    __shared__ int16_t s_active[CAP];
    __shared__ double s_red[NT > 64 ? kLMVals * (NT / 64) : 1];
    __shared__ LMShared S;
    __shared__ int s_tmp[40];
    LMP_DECL
    // problems blockIdx.x, blockIdx.x + gridDim.x, ...: a grid smaller than the problem count keeps the LM on fewer
    // CUs (launch_lm), every problem is solved exactly as with one workgroup each
    for (int prob = blockIdx.x; prob < n_prob; prob += gridDim.x) {
    const int tid = threadIdx.x;
    const int64_t e0 = counts ? (int64_t)prob * stride : (int64_t)offsets[prob];
    int n = counts ? counts[prob] : (int)(offsets[prob + 1] - e0);
    if (n > CAP) n = CAP;
    const double* X = Xall + 3 * e0;
    const double* uv = uvall + 2 * e0;
    if (tid < 9) S.K[tid] = Kall[9 * prob + tid];
    if (tid < 7) S.T[tid] = priors[7 * prob + tid];
    if (tid == 0) S.lit = 0;
    for (int i = tid; i < n; i += NT) {
        s_level[i] = 0;
        s_out[i] = 0;
        s_robust[i] = 1;
    }
    __syncthreads();
    double prior[7];
    for (int q = 0; q < 7; ++q) prior[q] = S.T[q];
    const double chi2th = 5.991;
    const double tau = 1e-5, goodLower = 1.0 / 3.0, goodUpper = 2.0 / 3.0;
    int outlierCount = 0;
    // Round memoization (exact): every round restarts from the same prior with a fresh LM (src/LoopHandler.cc:817-
    // 819: setEstimate(currentFrame->pose), initializeOptimization(), optimize(10)), so a round whose active edge set
    // and robust kernels equal those of the last executed round replays it operation for operation: its estimate,
    // its edges' errors and hence its classification are the last round's, and it is skipped.  The active set is
    // unchanged iff the last classification moved no edge between levels.  Dropping the Huber kernel after round 2
    // changes nothing either when no pass of the replayed round applied a Huber weight: below delta^2 the kernel's
    // rho = e2 and rho' = 1.0, and every product with 1.0 is exact.
    bool replay = false;
    int hub = 0;

    for (int round = 0; round < 4; ++round) {
        int changed = 0;
        if (!replay) {
            if (tid == 0) S.hub = 0;  // the first pass starts with a barrier: no wave writes S.hub before this store
            if (tid < 7) S.T[tid] = prior[tid];
            // initializeOptimization(): active = level-0 edges in insertion order (block compaction)
            int na = 0;
            for (int base = 0; base < n; base += NT) {
                const int i = base + tid;
                const int f = (i < n && s_level[i] == 0) ? 1 : 0;
                int tot = 0;
                const int off = block_excl_scan_geom<NT>(f, s_tmp, &tot);
                if (f) s_active[na + off] = (int16_t)i;
                na += tot;
            }
            __syncthreads();
            if (na > 0) {
                double lambda = 0, ni = 2;
                // S.vals holds {H, b, chi2} at S.T when `have` (the last trial was accepted: g2o's next
                // computeActiveErrors + buildSystem happen at exactly that estimate, so the trial pass builds the
                // system along with its chi2 and the rebuild is skipped)
                bool have = false;
                for (int it = 0; it < 10; ++it) {
    #ifdef YAVO_LM_PROFILE
                    LMP_MARK(5);
                    if (!have) lm_pass<NT>(S, s_active, na, s_robust, X, uv, s_red, lmp_acc);
                    lmp_t = __builtin_readcyclecounter();
    #else
                    if (!have) lm_pass<NT>(S, s_active, na, s_robust, X, uv, s_red);
    #endif
                    if (tid == 0) {
                        double sys[28];
    #pragma unroll
                        for (int v = 0; v < 28; ++v) sys[v] = S.vals[v];
    #pragma unroll
                        for (int v = 0; v < 28; ++v) S.sys[v] = sys[v];
    #pragma unroll
                        for (int r = 0; r < 6; ++r)
    #pragma unroll
                            for (int c = 0; c <= r; ++c) {
                                S.Hf[r * 6 + c] = sys[r * (r + 1) / 2 + c];
                                S.Hf[c * 6 + r] = sys[r * (r + 1) / 2 + c];
                            }
                        S.currentChi = sys[27];
                        if (it == 0) {
                            double maxDiag = 0;
    #pragma unroll
                            for (int j = 0; j < 6; ++j) {
                                const double d = fabs(sys[j * (j + 1) / 2 + j]);
                                maxDiag = d > maxDiag ? d : maxDiag;
                            }
                            lambda = tau * maxDiag;
                            ni = 2;
                        }
                    }
                    LMP_MARK(7);
                    // trial loop (do ... while (rho < 0 && qmax < 10))
                    int qmax = 0;
                    int f = 0;
                    while (true) {
                        if (tid == 0) {
                            double Tc[7], xs[6];
    #pragma unroll
                            for (int q = 0; q < 7; ++q) Tc[q] = S.T[q];
    #pragma unroll
                            for (int q = 0; q < 7; ++q) S.Tbak[q] = Tc[q];
                            const int ok2 = ldlt6_solve_lds<0>(S.Hf, lambda, S.sys + 21, S.x) ? 1 : 0;
    #pragma unroll
                            for (int q = 0; q < 6; ++q) xs[q] = S.x[q];
                            LMP_MARK(6);
                            double Tn[7], Tnew[7];
                            se3_exp(xs, Tn);
                            se3_mul(Tn, Tc, Tnew);
    #pragma unroll
                            for (int q = 0; q < 7; ++q) S.T[q] = Tnew[q];
                            S.flag = ok2;
                        }
                        LMP_MARK(2);
    #ifdef YAVO_LM_PROFILE
                        lm_pass<NT>(S, s_active, na, s_robust, X, uv, s_red, lmp_acc);
                        lmp_t = __builtin_readcyclecounter();
    #else
                        lm_pass<NT>(S, s_active, na, s_robust, X, uv, s_red);  // errors + system at the trial estimate
    #endif
                        if (tid == 0) {
                            const int ok2 = S.flag;
                            double tempChi = S.vals[27];
                            if (!ok2) tempChi = DBL_MAX;
                            double rho = S.currentChi - tempChi;
                            double scale = 1;
                            if (ok2) {
                                double sc = 0;
                                for (int j = 0; j < 6; ++j) sc += S.x[j] * (lambda * S.x[j] + S.sys[21 + j]);
                                scale = sc + 1e-3;
                            }
                            rho /= scale;
                            int brk = 0, accepted = 0;
                            if (rho > 0 && isfinite(tempChi) && ok2) {
                                double t = 2 * rho - 1;
                                double alpha = 1. - cube_cr(t);  // pow(t, 3), correctly rounded
                                alpha = alpha < goodUpper ? alpha : goodUpper;
                                double sf = goodLower > alpha ? goodLower : alpha;
                                lambda *= sf;
                                ni = 2;
                                S.currentChi = tempChi;
                                accepted = 1;
                            } else {
                                lambda *= ni;
                                ni *= 2;
                                for (int q = 0; q < 7; ++q) S.T[q] = S.Tbak[q];
                                if (!isfinite(lambda)) brk = 1;
                            }
                            qmax++;
                            const bool again = !brk && rho < 0 && qmax < 10;
                            int fl = again ? 1 : 0;
                            if (!again) fl = (qmax == 10 || rho == 0 || !isfinite(lambda)) ? 2 : 0;
                            S.flag = fl | (accepted << 2);
                        }
                        __syncthreads();
                        f = S.flag;
                        __syncthreads();
                        LMP_MARK(3);
                        if ((f & 3) == 1) continue;
                        break;
                    }
                    if ((f & 3) == 2) break;
                    have = (f & 4) != 0;
                }
            }
            __syncthreads();
            // classify: previous outliers are recomputed at the final estimate (e->computeError()); the
            // active edges keep the error of the last computeActiveErrors, i.e. at the last TRIAL estimate
            // Tlast (possibly a rejected one) -- recomputed here from Tlast, bit-identical to the stored value
            double T[7], Tl[7], K[9];
            for (int q = 0; q < 7; ++q) T[q] = uni_f64(S.T[q]);
            for (int q = 0; q < 7; ++q) Tl[q] = uni_f64(S.Tlast[q]);
            for (int q = 0; q < 9; ++q) K[q] = uni_f64(S.K[q]);
            int cnt = 0, chg = 0;
            for (int i = tid; i < n; i += NT) {
                double ee[2];
                const double mi[2] = {(double)uv[2 * i], (double)uv[2 * i + 1]};
                edge_error(s_out[i] ? T : Tl, K, X + 3 * i, mi, ee);
                const double c2 = ee[0] * ee[0] + ee[1] * ee[1];
                const uint8_t lev = c2 > chi2th ? 1 : 0;
                chg |= lev != s_level[i];
                s_out[i] = lev;
                s_level[i] = lev;
                cnt += lev;
                if (round == 2) s_robust[i] = 0;
            }
            int tot = 0;
            block_excl_scan_geom<NT>(cnt, s_tmp, &tot);
            outlierCount = tot;
            hub = S.hub;  // read before the barrier: the next executed round's lane 0 clears S.hub right after it
            changed = __syncthreads_or(chg);
            LMP_MARK(4);
        } else if (round == 2) {  // a replayed round 2 still drops the Huber kernels
            for (int i = tid; i < n; i += NT) s_robust[i] = 0;
            __syncthreads();
        }
        // round + 1 replays the last executed round iff no edge changed level and, across the Huber drop after round 2,
        // no pass of that round applied a Huber weight (`hub` is that round's: replayed rounds run no pass).  Every
        // wave takes the same decision: `changed` comes from the barrier vote and `hub` from a read every wave made
        // before that barrier.
        replay = !changed && (round != 2 || hub == 0);
    }
    if (tid < 7) poses[7 * prob + tid] = S.T[tid];
    for (int i = tid; i < n; i += NT) outlier_all[e0 + i] = s_out[i];
    if (tid == 0) inliers[prob] = n - outlierCount;
    __syncthreads();  // the next problem reinitialises the shared state
    }
    LMP_STORE();
}

template <int NT>
__global__ __launch_bounds__(NT) YAVO_LM_ATTR void pose_lm_kernel(const int32_t* __restrict__ offsets, const int32_t* __restrict__ counts,
                                                      int stride, const double* __restrict__ Xall,
                                                      const double* __restrict__ uvall, const double* __restrict__ Kall,
                                                      const double* priors, double* poses,
                                                      uint8_t* __restrict__ outlier_all, int32_t* __restrict__ inliers,
                                                      int n_prob) {
    pose_lm_body<NT>(offsets, counts, stride, Xall, uvall, Kall, priors, poses, outlier_all, inliers, n_prob);
}

// Track edges of the batched frontend: track t = {stereo pair sp, temporal pair tp} with
// pairs[sp].query == pairs[tp].train (frame k's left image).  For temporal query i (frame k-1 keypoint)
// kept by removeOutliers with best train keypoint j of frame k, and j's stereo match kept with right-image
// keypoint r: X = triangulate(kp_k[j], kp_right[r]) with the left camera as world (pose identity) and the
// right camera at T_right; accepted iff triangulation succeeds and Z > 0 (triangulate2View,
// src/LoopHandler.cc:658-726).  uv = (kp_{k-1}[i].x, kp_{k-1}[i].y) (the reference's measurement,
// src/LoopHandler.cc:786).  Edges keep temporal query order.  One workgroup per track.
template <int NT>
__global__ __launch_bounds__(NT) void track_build_kernel(
    const int32_t* __restrict__ tracks, const int32_t* __restrict__ pairs, const yv_keypoint* __restrict__ keypoints,
    const int32_t* __restrict__ kp_count, const int2* __restrict__ match_dj, const int32_t* __restrict__ match_lim,
    int max_kp, const double* __restrict__ Kall, const double* __restrict__ T_right, double* __restrict__ edge_X,
    double* __restrict__ edge_uv, int32_t* __restrict__ edge_query, int32_t* __restrict__ edge_count) {
    __shared__ int s_tmp[40];
    __shared__ double s_K[9], s_Ta[7], s_Tb[7];
    const int t = blockIdx.x, tid = threadIdx.x;
    const int sp = tracks[2 * t], tp = tracks[2 * t + 1];
    const int qs = pairs[2 * sp], rs = pairs[2 * sp + 1];  // frame k left, frame k right
    const int qt = pairs[2 * tp];                          // frame k-1 left
    if (tid < 9) s_K[tid] = Kall[9 * t + tid];
    if (tid < 7) {
        s_Ta[tid] = tid == 3 ? 1.0 : 0.0;
        s_Tb[tid] = T_right[tid];
    }
    __syncthreads();
    const int nq = kp_count[qt];
    const int lim_t = match_lim[tp], lim_s = match_lim[sp];
    const int2* dj_t = match_dj + (int64_t)tp * max_kp;
    const int2* dj_s = match_dj + (int64_t)sp * max_kp;
    const yv_keypoint* kq = keypoints + (int64_t)qt * max_kp;
    const yv_keypoint* kl = keypoints + (int64_t)qs * max_kp;
    const yv_keypoint* kr = keypoints + (int64_t)rs * max_kp;
    double* Xo = edge_X + 3 * (int64_t)t * max_kp;
    double* uvo = edge_uv + 2 * (int64_t)t * max_kp;
    int32_t* qo = edge_query + (int64_t)t * max_kp;
    int ne = 0;
    for (int base = 0; base < nq; base += NT) {
        const int i = base + tid;
        bool good = false;
        double X[3];
        if (i < nq) {
            const int2 a = dj_t[i];
            if (a.x < lim_t && a.y >= 0) {
                const int2 b = dj_s[a.y];
                if (b.x < lim_s && b.y >= 0)
                    good = triangulate_px(kl[a.y].x, kl[a.y].y, kr[b.y].x, kr[b.y].y, s_Ta, s_Tb, s_K, X);
            }
        }
        int tot = 0;
        const int off = block_excl_scan_geom<NT>(good ? 1 : 0, s_tmp, &tot);
        if (good) {
            const int e = ne + off;
            Xo[3 * e] = X[0];
            Xo[3 * e + 1] = X[1];
            Xo[3 * e + 2] = X[2];
            uvo[2 * e] = (double)kq[i].x;
            uvo[2 * e + 1] = (double)kq[i].y;
            qo[e] = i;
        }
        ne += tot;
    }
    if (tid == 0) edge_count[t] = ne;
}

// LK tracking mode (the reference's trackLastFrame, src/LoopHandler.cc:298-454).  Map points of frame k-1: its
// left keypoints whose stereo match (pair sp) survives removeOutliers and triangulates (left camera = world).
// Compacted in keypoint order: X, the LK start point (x = column, y = row as cv::Point2f, :344) and the
// keypoint index.  One workgroup per track.
template <int NT>
__global__ __launch_bounds__(NT) void stereo_points_kernel(
    const int32_t* __restrict__ stereo_pairs, const int32_t* __restrict__ pairs,
    const yv_keypoint* __restrict__ keypoints, const int32_t* __restrict__ kp_count, const int2* __restrict__ match_dj,
    const int32_t* __restrict__ match_lim, int max_kp, const double* __restrict__ Kall,
    const double* __restrict__ T_right, double* __restrict__ pX, float* __restrict__ pts, int32_t* __restrict__ pq,
    int32_t* __restrict__ pcount) {
    __shared__ int s_tmp[40];
    __shared__ double s_K[9], s_Ta[7], s_Tb[7];
    const int t = blockIdx.x, tid = threadIdx.x;
    const int sp = stereo_pairs[t];
    const int qs = pairs[2 * sp], rs = pairs[2 * sp + 1];
    if (tid < 9) s_K[tid] = Kall[9 * t + tid];
    if (tid < 7) {
        s_Ta[tid] = tid == 3 ? 1.0 : 0.0;
        s_Tb[tid] = T_right[tid];
    }
    __syncthreads();
    const int nq = kp_count[qs];
    const int lim = match_lim[sp];
    const int2* dj = match_dj + (int64_t)sp * max_kp;
    const yv_keypoint* kl = keypoints + (int64_t)qs * max_kp;
    const yv_keypoint* kr = keypoints + (int64_t)rs * max_kp;
    double* Xo = pX + 3 * (int64_t)t * max_kp;
    float* po = pts + 2 * (int64_t)t * max_kp;
    int32_t* qo = pq + (int64_t)t * max_kp;
    int ne = 0;
    for (int base = 0; base < nq; base += NT) {
        const int j = base + tid;
        bool good = false;
        double X[3];
        if (j < nq) {
            const int2 a = dj[j];
            if (a.x < lim && a.y >= 0) good = triangulate_px(kl[j].x, kl[j].y, kr[a.y].x, kr[a.y].y, s_Ta, s_Tb, s_K, X);
        }
        int tot = 0;
        const int off = block_excl_scan_geom<NT>(good ? 1 : 0, s_tmp, &tot);
        if (good) {
            const int e = ne + off;
            Xo[3 * e] = X[0];
            Xo[3 * e + 1] = X[1];
            Xo[3 * e + 2] = X[2];
            po[2 * e] = (float)kl[j].y;      // cv::Point2i(kp.y, kp.x) -> Point2f: x = column
            po[2 * e + 1] = (float)kl[j].x;  // y = row
            qo[e] = j;
        }
        ne += tot;
    }
    if (tid == 0) pcount[t] = ne;
}

// Pose edges from the LK result: points with status 1 become features at cv::Point2i(next.y, next.x), i.e. the
// float coordinates truncated toward zero (src/LoopHandler.cc:395), measurement (kp.x, kp.y) = (row, col).
__global__ __launch_bounds__(kNT) void lk_edges_kernel(const double* __restrict__ pX, const float* __restrict__ next,
                                                       const uint8_t* __restrict__ status,
                                                       const int32_t* __restrict__ pq,
                                                       const int32_t* __restrict__ pcount, int max_kp,
                                                       double* __restrict__ edge_X, double* __restrict__ edge_uv,
                                                       int32_t* __restrict__ edge_query,
                                                       int32_t* __restrict__ edge_count) {
    __shared__ int s_tmp[40];
    const int t = blockIdx.x, tid = threadIdx.x;
    const int n = pcount[t];
    const int64_t b = (int64_t)t * max_kp;
    int ne = 0;
    for (int base = 0; base < n; base += kNT) {
        const int i = base + tid;
        const bool good = i < n && status[b + i];
        int tot = 0;
        const int off = block_excl_scan_geom(good ? 1 : 0, s_tmp, &tot);
        if (good) {
            const int64_t e = b + ne + off;
            edge_X[3 * e] = pX[3 * (b + i)];
            edge_X[3 * e + 1] = pX[3 * (b + i) + 1];
            edge_X[3 * e + 2] = pX[3 * (b + i) + 2];
            edge_uv[2 * e] = (double)(int)next[2 * (b + i) + 1];  // kp.x = (int) row
            edge_uv[2 * e + 1] = (double)(int)next[2 * (b + i)];  // kp.y = (int) column
            edge_query[e] = pq[b + i];
        }
        ne += tot;
    }
    if (tid == 0) edge_count[t] = ne;
}

__global__ __launch_bounds__(kNT) void pose_gn_kernel(const int32_t* __restrict__ offsets, const double* __restrict__ Xall,
                                                      const double* __restrict__ uvall, const double* __restrict__ Kall,
                                                      double* __restrict__ poses, int32_t* __restrict__ iters_out) {
    __shared__ double s_red[kLMVals * 128];
    __shared__ double s_vals[32];
    __shared__ double s_T[7];
    __shared__ int s_flag;
    const int prob = blockIdx.x;
    const int tid = threadIdx.x;
    const int e0 = offsets[prob];
    const int n = offsets[prob + 1] - e0;
    const double* X = Xall + 3 * (int64_t)e0;
    const double* uv = uvall + 2 * (int64_t)e0;
    double K[9];
    for (int q = 0; q < 9; ++q) K[q] = Kall[9 * prob + q];
    if (tid < 7) s_T[tid] = poses[7 * prob + tid];
    __syncthreads();
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double lastCost = 0;
    int acc = 0;
    for (int iter = 0; iter < 10; iter++) {
        double T[7];
        for (int q = 0; q < 7; ++q) T[q] = s_T[q];
        double part[kLMVals];
        for (int v = 0; v < kLMVals; ++v) part[v] = 0.0;
        for (int i = tid; i < n; i += kNT) {
            double pc[3];
            se3_act(T, X + 3 * i, pc);
            double inv_z = 1.0 / pc[2];
            double inv_z2 = inv_z * inv_z;
            double proj0 = fx * pc[0] / pc[2] + cx, proj1 = fy * pc[1] / pc[2] + cy;
            double ee0 = uv[2 * i] - proj0, ee1 = uv[2 * i + 1] - proj1;
            part[27] = part[27] + (ee0 * ee0 + ee1 * ee1);
            double J[12] = {-fx * inv_z, 0, fx * pc[0] * inv_z2, fx * pc[0] * pc[1] * inv_z2,
                            -fx - fx * pc[0] * pc[0] * inv_z2, fx * pc[1] * inv_z,
                            0, -fy * inv_z, fy * pc[1] * inv_z2, fy + fy * pc[1] * pc[1] * inv_z2,
                            -fy * pc[0] * pc[1] * inv_z2, -fy * pc[0] * inv_z};
            int v = 0;
            for (int r = 0; r < 6; ++r) {
                for (int c = 0; c <= r; ++c) {
                    part[v] = part[v] + (J[r] * J[c] + J[6 + r] * J[6 + c]);
                    ++v;
                }
                part[21 + r] = part[21 + r] + ((-J[r]) * ee0 + (-J[6 + r]) * ee1);
            }
        }
        tree_reduce<kLMVals>(part, s_red, s_vals);
        if (tid == 0) {
            double H[36], b[6], dx[6];
            int v = 0;
            for (int r = 0; r < 6; ++r)
                for (int c = 0; c <= r; ++c) {
                    H[r * 6 + c] = s_vals[v];
                    H[c * 6 + r] = s_vals[v];
                    ++v;
                }
            for (int r = 0; r < 6; ++r) b[r] = s_vals[21 + r];
            const double cost = s_vals[27];
            ldlt6_solve<1>(H, b, dx);
            int stop = 0;
            if (isnan(dx[0])) stop = 1;
            else if (iter > 0 && cost >= lastCost) stop = 1;
            else {
                double Tn[7], Tnew[7], Tc[7];
                for (int q = 0; q < 7; ++q) Tc[q] = s_T[q];
                se3_exp(dx, Tn);
                se3_mul(Tn, Tc, Tnew);
                for (int q = 0; q < 7; ++q) s_T[q] = Tnew[q];
                lastCost = cost;
                acc++;
                double q0 = dx[0] * dx[0] + (dx[2] * dx[2] + dx[4] * dx[4]);
                double q1 = dx[1] * dx[1] + (dx[3] * dx[3] + dx[5] * dx[5]);
                if (sqrt(q0 + q1) < 1e-6) stop = 1;
            }
            s_flag = stop;
        }
        __syncthreads();
        const int stop = s_flag;
        __syncthreads();
        if (stop) break;
    }
    if (tid < 7) poses[7 * prob + tid] = s_T[tid];
    if (tid == 0) iters_out[prob] = acc;
}

// Threads per pose-LM workgroup: 256, one wave per SIMD (the LM is latency-bound: 64 / 128 threads measured 2.1 /
// 1.5 ms against 1.0 ms per 256-frame batch).  The summation order follows (yv_lm_sum_mode 6).  Measured and not kept
// (DESIGN.md 4.3, 10): fewer workgroups looping over the problems, LDS padding to one workgroup per CU, and a form
// holding each problem's edges in LDS.
constexpr int kLMThreads = 256;
// A few problems (the host-pointer yv_pose_lm of the LoopHandler, small yv_pose_lm_batch calls, the tracks of a small
// batch such as the sequence front end's 20-frame chunks) leave most CUs idle, so their latency is what counts: 512
// threads, two waves per SIMD of the problem's own CU, halve each thread's edge share (sum order 7,
// yv_pose_lm_sum_mode / yv_track_lm_sum_mode).  Larger batches keep 256 (two problems per CU interleave there).
constexpr int kLMThreadsWide = 512;
constexpr int kLMWideMaxProblems = 256;

template <int NT = kLMThreads, typename... A>
void launch_lm(int n, hipStream_t s, A... args) {
    hipLaunchKernelGGL(pose_lm_kernel<NT>, dim3(n), dim3(NT), 0, s, args..., n);
}

constexpr int lm_mode_of(int nt) { return nt == 512 ? 7 : nt == 256 ? 6 : nt == 128 ? 5 : 4; }

}  // namespace geom

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
size_t f_ransac_ws_bytes(int n_lists, int iters) {
    const size_t h = (size_t)std::max(n_lists, 1) * (size_t)std::max(iters, 1);
    return ((h * 9 * sizeof(double) + 255) & ~(size_t)255) + h * sizeof(int32_t);
}

void launch_f_ransac(const yv_match* matches, int64_t list_stride, const int32_t* counts, int n_lists,
                     const int32_t* samples, int64_t sample_stride, int iters, double thr, double* F_out,
                     int32_t* max_inliers, int32_t* found, void* ws, hipStream_t s) {
    if (n_lists <= 0) return;
    const size_t h = (size_t)n_lists * (size_t)std::max(iters, 1);
    double* ws_F = static_cast<double*>(ws);
    int32_t* ws_cnt = reinterpret_cast<int32_t*>(static_cast<char*>(ws) + ((h * 9 * sizeof(double) + 255) & ~(size_t)255));
    if (iters > 0) {
        hipLaunchKernelGGL(geom::f_hyp_kernel, dim3((iters + geom::kFHypWG - 1) / geom::kFHypWG, n_lists),
                           dim3(geom::kFHypWG), 0, s, matches, list_stride, counts, samples, sample_stride, iters, ws_F);
        hipLaunchKernelGGL(geom::f_count_kernel, dim3((iters + geom::kFCountWaves - 1) / geom::kFCountWaves, n_lists),
                           dim3(64 * geom::kFCountWaves), 0, s, matches, list_stride, counts, iters, thr, ws_F, ws_cnt);
    }
    hipLaunchKernelGGL(geom::f_select_kernel, dim3(n_lists), dim3(64), 0, s, counts, iters, ws_F, ws_cnt, F_out,
                       max_inliers, found);
}

void launch_triangulate(const yv_match* m, int n, const double* poses2, const double* K, double* Xw, uint8_t* ok,
                        int32_t* n_ok, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(geom::triangulate_kernel, dim3((n + 255) / 256), dim3(256), 0, s, m, n, poses2, K, Xw, ok, n_ok);
}

void launch_world2camera(const double* X, int n, const double* T, const double* K, double* out, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(geom::world2camera_kernel, dim3((n + 255) / 256), dim3(256), 0, s, X, n, T, K, out);
}

void launch_pose_lm(const int32_t* offsets, int n_problems, const double* X, const double* uv, const double* K,
                    double* poses, uint8_t* outlier, int32_t* inliers, hipStream_t s) {
    if (n_problems <= geom::kLMWideMaxProblems)
        geom::launch_lm<geom::kLMThreadsWide>(n_problems, s, offsets, static_cast<const int32_t*>(nullptr), 0, X, uv, K,
                                              static_cast<const double*>(poses), poses, outlier, inliers);
    else
        geom::launch_lm(n_problems, s, offsets, static_cast<const int32_t*>(nullptr), 0, X, uv, K,
                        static_cast<const double*>(poses), poses, outlier, inliers);
}

void launch_track_build(const int32_t* tracks, int n_tracks, const int32_t* pairs, const yv_keypoint* keypoints,
                        const int32_t* kp_count, const int2* match_dj, const int32_t* match_lim, int max_kp,
                        const double* K, const double* T_right, double* edge_X, double* edge_uv, int32_t* edge_query,
                        int32_t* edge_count, hipStream_t s) {
    if (n_tracks <= 0) return;
    // 1024 threads: about one query keypoint per thread (the FP64 triangulations are latency-bound; 256 / 512 were
    // measured)
    hipLaunchKernelGGL(geom::track_build_kernel<1024>, dim3(n_tracks), dim3(1024), 0, s, tracks, pairs, keypoints,
                       kp_count, match_dj, match_lim, max_kp, K, T_right, edge_X, edge_uv, edge_query, edge_count);
}

void launch_stereo_points(const int32_t* stereo_pairs, int n_tracks, const int32_t* pairs,
                          const yv_keypoint* keypoints, const int32_t* kp_count, const int2* match_dj,
                          const int32_t* match_lim, int max_kp, const double* K, const double* T_right, double* pX,
                          float* pts, int32_t* pq, int32_t* pcount, hipStream_t s) {
    if (n_tracks <= 0) return;
    // 1024 threads: about one keypoint per thread (FP64 triangulations, latency-bound)
    hipLaunchKernelGGL(geom::stereo_points_kernel<1024>, dim3(n_tracks), dim3(1024), 0, s, stereo_pairs, pairs,
                       keypoints, kp_count, match_dj, match_lim, max_kp, K, T_right, pX, pts, pq, pcount);
}

void launch_lk_edges(int n_tracks, const double* pX, const float* next, const uint8_t* status, const int32_t* pq,
                     const int32_t* pcount, int max_kp, double* edge_X, double* edge_uv, int32_t* edge_query,
                     int32_t* edge_count, hipStream_t s) {
    if (n_tracks <= 0) return;
    hipLaunchKernelGGL(geom::lk_edges_kernel, dim3(n_tracks), dim3(geom::kNT), 0, s, pX, next, status, pq, pcount,
                       max_kp, edge_X, edge_uv, edge_query, edge_count);
}

void launch_track_pose(int n_tracks, const int32_t* edge_count, int stride, const double* edge_X,
                       const double* edge_uv, const double* K, const double* priors, double* poses,
                       uint8_t* edge_outlier, int32_t* inliers, hipStream_t s) {
    if (n_tracks <= 0) return;
    if (n_tracks <= geom::kLMWideMaxProblems)
        geom::launch_lm<geom::kLMThreadsWide>(n_tracks, s, static_cast<const int32_t*>(nullptr), edge_count, stride,
                                              edge_X, edge_uv, K, priors, poses, edge_outlier, inliers);
    else
        geom::launch_lm(n_tracks, s, static_cast<const int32_t*>(nullptr), edge_count, stride, edge_X, edge_uv, K,
                        priors, poses, edge_outlier, inliers);
}

void launch_pose_gn(const int32_t* offsets, int n_problems, const double* X, const double* uv, const double* K,
                    double* poses, int32_t* iters, hipStream_t s) {
    hipLaunchKernelGGL(geom::pose_gn_kernel, dim3(n_problems), dim3(geom::kNT), 0, s, offsets, X, uv, K, poses, iters);
}

}  // namespace yavo

extern "C" int yv_lm_sum_mode(void) { return yavo::geom::lm_mode_of(yavo::geom::kLMThreads); }

extern "C" int yv_track_lm_sum_mode(int n_tracks) {
    return yavo::geom::lm_mode_of(n_tracks <= yavo::geom::kLMWideMaxProblems ? yavo::geom::kLMThreadsWide
                                                                             : yavo::geom::kLMThreads);
}

extern "C" int yv_pose_lm_sum_mode(int n_problems) {
    return yavo::geom::lm_mode_of(n_problems <= yavo::geom::kLMWideMaxProblems ? yavo::geom::kLMThreadsWide
                                                                               : yavo::geom::kLMThreads);
}

#ifdef YAVO_LM_PROFILE
// profiling builds only (lib/libyavo_prof.so): per-workgroup pose-LM phase cycle counts of the last launch
extern "C" int yv_debug_lm_prof(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(yavo::geom::g_lm_prof), sizeof(unsigned long long) * 1024 * 10) ==
                   hipSuccess ? 0 : -2;
}
#endif

