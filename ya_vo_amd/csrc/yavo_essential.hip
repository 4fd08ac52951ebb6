// yavo_essential.hip -- gfx950 kernels for cv::findEssentialMat (RANSAC) + cv::recoverPose as the reference calls
// them at (re)initialisation (src/LoopHandler.cc:239,256,581,598).  Restates the classic OpenCV
// 4.x path like oracle/yavo_oracle_essential.c, expression for expression (built with -ffp-contract=off):
//
//   ess_prepare_kernel   (p - c) / f per point as OpenCV's MatExpr evaluates it, float -> double
//   ess_subsets_kernel   getSubset's cv::RNG((uint64)-1) draws of a round (64 iterations; 1024 for <= 8 lists) (one lane
//                        per list; the draws never depend on the models, so a round's subsets are drawn before its models)
//   ess_models_kernel    EMEstimatorCallback::runKernel, one RANSAC iteration per lane (64-lane workgroups) or, for
//                        <= 8 lists, per 10-lane group (six per workgroup):
//                        JacobiSVD null space, the cubic-constraint matrix, LU inverse, det B(z), Durand-Kerner,
//                        solveZ, up to 10 models
//   ess_score_kernel     one workgroup per iteration: float Sampson errors of its models over the whole list
//   ess_select_kernel    one lane per list: RANSACPointSetRegistrator::run's sequential best / niters update over
//                        the round; later rounds are skipped once niters is reached
//   rp_*                 recoverPose: decomposeEssentialMat per list, one lane per (point, candidate) triangulating
//                        (4 x 4 JacobiSVD), counts by ballot + one atomic per candidate and wave, the selection
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "yavo_internal.h"
#include "yavo_cvsvd.h"
#include "yavo_xlane.h"

namespace yavo {
namespace ess {

// YAVO_LM_PROFILE builds (tools/ess_profile.py): the five-point solver's phase cycles per lane of the first 256
// iterations of list 0 (SVD, coefficient matrix, LU inverse + product, det B(z), Durand-Kerner, solveZ), and the
// Durand-Kerner sweep count
#ifdef YAVO_LM_PROFILE
__device__ unsigned long long g_ess_prof[256][8];
#define EP_DECL unsigned long long ep_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long ep_t = __builtin_readcyclecounter();
#define EP_MARK(slot) do { const unsigned long long t_ = __builtin_readcyclecounter(); ep_acc[slot] += t_ - ep_t; ep_t = t_; } while (0)
#define EP_SET(slot, v) (ep_acc[slot] = (v))
#define EP_STORE(k) do { if ((k) < 256) for (int q_ = 0; q_ < 8; ++q_) g_ess_prof[(k)][q_] = ep_acc[q_]; } while (0)
#else
#define EP_DECL
#define EP_MARK(slot) do {} while (0)
#define EP_SET(slot, v) do {} while (0)
#define EP_STORE(k) do {} while (0)
#endif

using cv::cv_jacobi_svd;
using cv::cv_jacobi_svd_mn;
using cv::cv_rng_next;

// ------------------------------------------------------------------------------------------------
// polynomial term orders (oracle: kLinExp / kQuadExp / kCubExp)
// ------------------------------------------------------------------------------------------------
struct Exp3 {
    int a, b, c;
};
constexpr Exp3 kLin[4] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
constexpr Exp3 kQuad[10] = {{2, 0, 0}, {1, 1, 0}, {1, 0, 1}, {1, 0, 0}, {0, 2, 0},
                            {0, 1, 1}, {0, 1, 0}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
constexpr Exp3 kCub[20] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                           {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                           {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
constexpr int quad_index(int a, int b, int c) {
    for (int i = 0; i < 10; ++i)
        if (kQuad[i].a == a && kQuad[i].b == b && kQuad[i].c == c) return i;
    return -1;
}
constexpr int cub_index(int a, int b, int c) {
    for (int i = 0; i < 20; ++i)
        if (kCub[i].a == a && kCub[i].b == b && kCub[i].c == c) return i;
    return -1;
}
struct LLTab {
    int t[4][4];
};
struct QLTab {
    int t[10][4];
};
constexpr LLTab make_ll() {
    LLTab r{};
    for (int p = 0; p < 4; ++p)
        for (int q = 0; q < 4; ++q) r.t[p][q] = quad_index(kLin[p].a + kLin[q].a, kLin[p].b + kLin[q].b, kLin[p].c + kLin[q].c);
    return r;
}
constexpr QLTab make_ql() {
    QLTab r{};
    for (int p = 0; p < 10; ++p)
        for (int q = 0; q < 4; ++q)
            r.t[p][q] = cub_index(kQuad[p].a + kLin[q].a, kQuad[p].b + kLin[q].b, kQuad[p].c + kLin[q].c);
    return r;
}
constexpr LLTab kLL = make_ll();
constexpr QLTab kQL = make_ql();

__device__ __forceinline__ void mul_lin_lin(const double* P, const double* Q, double* R) {
#pragma unroll
    for (int i = 0; i < 10; ++i) R[i] = 0.0;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) R[kLL.t[p][q]] += P[p] * Q[q];
}
__device__ __forceinline__ void mul_quad_lin(const double* P, const double* Q, double* R) {
#pragma unroll
    for (int i = 0; i < 20; ++i) R[i] = 0.0;
#pragma unroll
    for (int p = 0; p < 10; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) R[kQL.t[p][q]] += P[p] * Q[q];
}

// getCoeffMat (oracle or_em_coeff_mat): rows 0..8 = 2 (E E^T E)_ij - tr(E E^T) E_ij, row 9 = det E
__device__ void em_coeff_mat(const double* EE, double* A) {
    double e[9][4];
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int v = 0; v < 4; ++v) e[k][v] = EE[v * 9 + k];
    double S[9][10];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double t[10];
            mul_lin_lin(e[i * 3 + 0], e[j * 3 + 0], S[i * 3 + j]);
#pragma unroll
            for (int k = 1; k < 3; ++k) {
                mul_lin_lin(e[i * 3 + k], e[j * 3 + k], t);
#pragma unroll
                for (int q = 0; q < 10; ++q) S[i * 3 + j][q] = S[i * 3 + j][q] + t[q];
            }
        }
    double tr[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) tr[q] = S[0][q] + S[4][q] + S[8][q];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc[20], t[20];
            mul_quad_lin(S[i * 3 + 0], e[0 * 3 + j], acc);
#pragma unroll
            for (int k = 1; k < 3; ++k) {
                mul_quad_lin(S[i * 3 + k], e[k * 3 + j], t);
#pragma unroll
                for (int q = 0; q < 20; ++q) acc[q] = acc[q] + t[q];
            }
            mul_quad_lin(tr, e[i * 3 + j], t);
            double* row = A + (i * 3 + j) * 20;
#pragma unroll
            for (int q = 0; q < 20; ++q) row[q] = 2.0 * acc[q] - t[q];
        }
    double m1[10], m2[10], d[10], c0[20], c1[20], c2[20];
    mul_lin_lin(e[4], e[8], m1);
    mul_lin_lin(e[5], e[7], m2);
#pragma unroll
    for (int q = 0; q < 10; ++q) d[q] = m1[q] - m2[q];
    mul_quad_lin(d, e[0], c0);
    mul_lin_lin(e[3], e[8], m1);
    mul_lin_lin(e[5], e[6], m2);
#pragma unroll
    for (int q = 0; q < 10; ++q) d[q] = m1[q] - m2[q];
    mul_quad_lin(d, e[1], c1);
    mul_lin_lin(e[3], e[7], m1);
    mul_lin_lin(e[4], e[6], m2);
#pragma unroll
    for (int q = 0; q < 10; ++q) d[q] = m1[q] - m2[q];
    mul_quad_lin(d, e[2], c2);
    double* row = A + 9 * 20;
#pragma unroll
    for (int q = 0; q < 20; ++q) row[q] = c0[q] - c1[q] + c2[q];
}

// every lane gets lane j's v in out[j] (j < N) of its 16-lane row
template <int N, int J = 0>
__device__ __forceinline__ void bcast_col(double v, double* out) {
    if constexpr (J < N) {
        out[J] = xl::row_bcast_f64<J>(v);
        bcast_col<N, J + 1>(v, out);
    }
}
// every lane gets lane `from`'s row[0 .. N) (from: a loop counter the compiler unrolls)
template <int N, int J = 0>
__device__ __forceinline__ void bcast_row_from(int from, const double* row, double* out) {
    if constexpr (J < N) {
        if (from == J) {
#pragma unroll
            for (int q = 0; q < N; ++q) out[q] = xl::row_bcast_f64<J>(row[q]);
        } else {
            bcast_row_from<N, J + 1>(from, row, out);
        }
    }
}

// cv::invert(DECOMP_LU), n = 10: LUImpl<double> with b = I, eps = 100 DBL_EPSILON, zeros when singular.
// A: 10 rows of stride 20 (the first 10 columns are inverted).  Only rows first .. 9 of the inverse are formed (the
// back substitution of row i reads rows > i alone; runKernel uses rows 4 .. 9); the others are left as they are.
__device__ void lu_inverse10(const double* A, double* inv, int first = 0) {
    constexpr int n = 10;
    double a[100], b[100];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            a[i * n + j] = A[i * 20 + j];
            b[i * n + j] = i == j ? 1.0 : 0.0;
        }
    const double eps = DBL_EPSILON * 100;
    for (int i = 0; i < n; i++) {
        int k = i;
        for (int j = i + 1; j < n; j++)
            if (fabs(a[j * n + i]) > fabs(a[k * n + i])) k = j;
        if (fabs(a[k * n + i]) < eps) {
            for (int q = 0; q < n * n; ++q) inv[q] = 0.0;
            return;
        }
        if (k != i) {
            for (int j = i; j < n; j++) { const double t = a[i * n + j]; a[i * n + j] = a[k * n + j]; a[k * n + j] = t; }
            for (int j = 0; j < n; j++) { const double t = b[i * n + j]; b[i * n + j] = b[k * n + j]; b[k * n + j] = t; }
        }
        const double d = -1 / a[i * n + i];
        for (int j = i + 1; j < n; j++) {
            const double alpha = a[j * n + i] * d;
            for (int q = i + 1; q < n; q++) a[j * n + q] += alpha * a[i * n + q];
            for (int q = 0; q < n; q++) b[j * n + q] += alpha * b[i * n + q];
        }
    }
    for (int i = n - 1; i >= first; i--)
        for (int j = 0; j < n; j++) {
            double s = b[i * n + j];
            for (int q = i + 1; q < n; q++) s -= a[i * n + q] * b[q * n + j];
            b[i * n + j] = s / a[i * n + i];
        }
    for (int q = first * n; q < n * n; ++q) inv[q] = b[q];
}

// The same LU inverse on a 10-lane group, lane r holding row r of a and b in registers: the pivot search is the
// sequential scan over the column broadcast to every lane, row swaps exchange two lanes' rows, the pivot row is
// broadcast (DPP) and every lower lane eliminates its own row -- each row's operations are the sequential code's, in
// its order.  The back substitution forms rows 9 .. 4 (lane i, rows q > i broadcast as they become final).  Then lane
// r's M row (r >= 4) = inv row r x A's right block; M4 gets rows 4 .. 9 in every lane.
__device__ void lu_m_group(const double* A, int r, int base, double* M4 /* [6][10] */) {
    constexpr int n = 10;
    const int rr = r < n ? r : 0;
    double a[n], b[n];
#pragma unroll
    for (int q = 0; q < n; ++q) {
        a[q] = A[rr * 20 + q];
        b[q] = q == r ? 1.0 : 0.0;
    }
    const double eps = DBL_EPSILON * 100;
    bool singular = false;
#pragma unroll
    for (int i = 0; i < n; i++) {
        if (singular) break;  // group-uniform
        double col[n];
        bcast_col<n>(a[i], col);
        int k = i;
        double vk = fabs(col[i]);
#pragma unroll
        for (int j = i + 1; j < n; j++)
            if (fabs(col[j]) > vk) {
                k = j;
                vk = fabs(col[j]);
            }
        if (vk < eps) {
            singular = true;
            break;
        }
        if (k != i) {  // group-uniform: rows i and k trade lanes (columns i .. 9 of a, all of b)
            const int src = base + (r == i ? k : (r == k ? i : r));
#pragma unroll
            for (int q = i; q < n; ++q) a[q] = __shfl(a[q], src, 64);
#pragma unroll
            for (int q = 0; q < n; ++q) b[q] = __shfl(b[q], src, 64);
        }
        double pa[n], pb[n];
        bcast_row_from<n>(i, a, pa);
        bcast_row_from<n>(i, b, pb);
        const double d = -1 / pa[i];
        if (r > i) {
            const double alpha = a[i] * d;
#pragma unroll
            for (int q = i + 1; q < n; q++) a[q] += alpha * pa[q];
#pragma unroll
            for (int q = 0; q < n; q++) b[q] += alpha * pb[q];
        }
    }
    if (singular) {
#pragma unroll
        for (int q = 0; q < n; ++q) b[q] = 0.0;
    } else {
#pragma unroll
        for (int i = n - 1; i >= 4; i--) {
            double sv[n];
#pragma unroll
            for (int j = 0; j < n; j++) sv[j] = b[j];
#pragma unroll
            for (int q = i + 1; q < n; q++) {
                double bq[n];
                bcast_row_from<n>(q, b, bq);
#pragma unroll
                for (int j = 0; j < n; j++) sv[j] -= a[q] * bq[j];
            }
            if (r == i) {
#pragma unroll
                for (int j = 0; j < n; j++) b[j] = sv[j] / a[i];
            }
        }
    }
    // M row r (r >= 4): sum over k of inv[r][k] * A[k][10 + j], k in order
    double m[n];
#pragma unroll
    for (int j = 0; j < n; ++j) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < n; ++k) s += b[k] * A[k * 20 + 10 + j];
        m[j] = s;
    }
#pragma unroll
    for (int q = 4; q < n; ++q) {
        double mq[n];
        bcast_row_from<n>(q, m, mq);
#pragma unroll
        for (int j = 0; j < n; ++j) M4[(q - 4) * n + j] = mq[j];
    }
}

template <int NP, int NQ>
__device__ __forceinline__ void pmul(const double* P, const double* Q, double* R) {
#pragma unroll
    for (int i = 0; i < NP + NQ - 1; ++i) R[i] = 0.0;
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int q = 0; q < NQ; ++q) R[p + q] += P[p] * Q[q];
}

// det B(z) (oracle or_em_det_poly)
__device__ void em_det_poly(const double* B, double* c) {
    double px[3][4], py[3][4], p1[3][5];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double* br = B + 13 * i;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            px[i][k] = br[3 - k];
            py[i][k] = br[7 - k];
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) p1[i][k] = br[12 - k];
    }
    double u[8], v[8], d[8], t0[11], t1[11], t2[11];
    pmul<4, 5>(py[1], p1[2], u);
    pmul<5, 4>(p1[1], py[2], v);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = u[k] - v[k];
    pmul<4, 8>(px[0], d, t0);
    pmul<4, 5>(px[1], p1[2], u);
    pmul<5, 4>(p1[1], px[2], v);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = u[k] - v[k];
    pmul<4, 8>(py[0], d, t1);
    double w[7], x[7], d2[7];
    pmul<4, 4>(px[1], py[2], w);
    pmul<4, 4>(py[1], px[2], x);
#pragma unroll
    for (int k = 0; k < 7; ++k) d2[k] = w[k] - x[k];
    pmul<5, 7>(p1[0], d2, t2);
#pragma unroll
    for (int k = 0; k < 11; ++k) c[k] = t0[k] - t1[k] + t2[k];
}

// cv::solvePoly (Durand-Kerner) of degree NN (the coefficients above NN were trimmed) on one lane; rre / rim [10].
// Every loop is unrolled (NN is a template constant), so j != i is resolved at compile time and a coincident root
// (OpenCV skips its factor) is a select, not a branch.  OpenCV stops when the largest |update| is 0; |q| > 0 exactly
// when qr^2 + qi^2 > 0 (NaN compares false either way), so the squared magnitude decides without the square root; a
// sweep that moved no root is a fixed point (every later sweep repeats it).  Returns the sweeps run.
// One sweep of dk_solve.  kSel: solvePoly's skip of a coincident root's factor, as a select; otherwise every factor is
// multiplied and `hit` reports a coincidence (the sweep is then run again from the same roots with the skip).
template <int NN, bool kSel>
__device__ __forceinline__ void dk_solve_sweep(const double* cr, double* xr, double* xi, bool& moved, double& maxDiff2,
                                               bool& hit) {
    maxDiff2 = 0;
    moved = false;
    hit = false;
#pragma unroll
    for (int i = 0; i < NN; i++) {
        const double pr = xr[i], pi = xi[i];
        double nr = cr[NN], ni = 0.0, dr = cr[NN], di = 0.0;
#pragma unroll
        for (int j = 0; j < NN; j++) {
            const double tr = nr * pr - ni * pi, ti = nr * pi + ni * pr;
            nr = tr + cr[NN - j - 1];
            ni = ti + 0.0;
            if (j != i) {
                const bool same = pr == xr[j] && pi == xi[j];
                const double sr = pr - xr[j], si = pi - xi[j];
                const double ur = dr * sr - di * si, ui = dr * si + di * sr;
                if (kSel) {
                    dr = same ? dr : ur;
                    di = same ? di : ui;
                } else {
                    hit |= same;
                    dr = ur;
                    di = ui;
                }
            }
        }
        const double t = 1. / (dr * dr + di * di);
        const double qr = (nr * dr + ni * di) * t, qi = (-nr * di + ni * dr) * t;
        xr[i] = pr - qr;
        xi[i] = pi - qi;
        moved |= __double_as_longlong(xr[i]) != __double_as_longlong(pr) ||
                 __double_as_longlong(xi[i]) != __double_as_longlong(pi);
        const double an2 = qr * qr + qi * qi;
        maxDiff2 = maxDiff2 < an2 ? an2 : maxDiff2;
    }
}

// cv::solvePoly (Durand-Kerner) of degree NN (the coefficients above NN were trimmed) on one lane; rre / rim [10].
// Every loop is unrolled (NN is a template constant), so j != i is resolved at compile time and a coincident root
// (OpenCV skips its factor) is a select, not a branch.  (The group form's replay-on-coincidence does not pay here:
// with 64 independent lanes a wave replays whenever any lane meets a coincidence -- 256 lists 2.75 -> 3.03 ms.)
// OpenCV stops when the largest |update| is 0; |q| > 0 exactly when qr^2 + qi^2 > 0 (NaN compares false either way),
// so the squared magnitude decides without the square root; a sweep that moved no root is a fixed point (every later
// sweep repeats it).  Returns the sweeps run.
template <int NN>
__device__ int dk_solve(const double* c, double* rre, double* rim) {
    double cr[NN + 1], xr[NN], xi[NN];
#pragma unroll
    for (int i = 0; i <= NN; ++i) cr[i] = c[i];
    {
        double pr = 1, pi = 0;
        const double qr = 1, qi = 1;
#pragma unroll
        for (int i = 0; i < NN; i++) {
            xr[i] = pr;
            xi[i] = pi;
            const double tr = pr * qr - pi * qi, ti = pr * qi + pi * qr;
            pr = tr;
            pi = ti;
        }
    }
    int sweeps = 0;
    for (int iter = 0; iter < 300; iter++) {
        ++sweeps;
        bool moved, hit;
        double maxDiff2;
        dk_solve_sweep<NN, true>(cr, xr, xi, moved, maxDiff2, hit);
        if (maxDiff2 <= 0 || !moved) break;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        if (i < NN) {
            rre[i] = xr[i];
            rim[i] = fabs(xi[i]) < 1e-100 ? 0.0 : xi[i];
        } else {
            rre[i] = 0.0;
            rim[i] = 0.0;
        }
    }
    return sweeps;
}

// cv::solvePoly's Durand-Kerner sweep with one root per lane of a group: lanes 0 .. 9 of a 16-lane row (lane r owns
// root r; all ten active whenever this runs), the roots exchanged by DPP row broadcasts.  The same operations in the same order as solvePoly: OpenCV's
// sweep is Gauss-Seidel -- root i's denominator prod_{j != i} (x_i - x_j) takes the roots j < i already updated in
// this sweep and j > i as they were -- so per sweep every lane first gathers the group's old roots and evaluates its
// Horner value (independent of the other roots), then for k = 0 .. NN-1: lane k multiplies its denominator by its
// suffix terms j > k (old values, in order), divides and updates; its new root is broadcast and every lane r > k
// multiplies its running denominator by (x_r - x_k^new): solvePoly's left-to-right product, factor by factor.
// A wave issues ~650 instead of ~1750 FP64 instructions per sweep (the ten roots' Horner chains and the tail of the
// products run side by side), and six hypotheses share a wave.  rre / rim: this lane's root (0 past NN).  Returns
// the sweeps run.
// the row's roots 0 .. N-1 into ox / oy, and root k (a loop counter the compiler unrolls) into kr / ki
template <int N, int J = 0>
__device__ __forceinline__ void bcast_all(double xr, double xi, double* ox, double* oy) {
    if constexpr (J < N) {
        ox[J] = xl::row_bcast_f64<J>(xr);
        oy[J] = xl::row_bcast_f64<J>(xi);
        bcast_all<N, J + 1>(xr, xi, ox, oy);
    }
}
template <int N, int J = 0>
__device__ __forceinline__ void bcast_one(int k, double xr, double xi, double& kr, double& ki) {
    if constexpr (J < N) {
        if (k == J) {
            kr = xl::row_bcast_f64<J>(xr);
            ki = xl::row_bcast_f64<J>(xi);
        } else {
            bcast_one<N, J + 1>(k, xr, xi, kr, ki);
        }
    }
}

// One Gauss-Seidel sweep of the group (see dk_group).  kSel: solvePoly's skip of a factor whose roots coincide, as a
// select; otherwise every factor is multiplied and `hit` reports whether a coincidence occurred in this lane.
template <int NN, bool kSel>
__device__ __forceinline__ void dk_sweep(const double* cr, int r, bool own, double& xr, double& xi, bool& moved,
                                         double& an2, bool& hit) {
    double ox[NN], oy[NN];
    bcast_all<NN>(xr, xi, ox, oy);
    const double pr = xr, pi = xi;
    double nr = cr[NN], ni = 0.0, dr = cr[NN], di = 0.0;
#pragma unroll
    for (int j = 0; j < NN; j++) {
        const double tr = nr * pr - ni * pi, ti = nr * pi + ni * pr;
        nr = tr + cr[NN - j - 1];
        ni = ti + 0.0;
    }
    moved = false;
    an2 = 0;
    hit = false;
    auto factor = [&](double xj, double yj) {
        const bool same = pr == xj && pi == yj;
        const double sr = pr - xj, si = pi - yj;
        const double ur = dr * sr - di * si, ui = dr * si + di * sr;
        if (kSel) {
            dr = same ? dr : ur;
            di = same ? di : ui;
        } else {
            hit |= same;
            dr = ur;
            di = ui;
        }
    };
#pragma unroll
    for (int k = 0; k < NN; ++k) {
        if (r == k) {
#pragma unroll
            for (int j = k + 1; j < NN; ++j) factor(ox[j], oy[j]);
            const double t = 1. / (dr * dr + di * di);
            const double qr = (nr * dr + ni * di) * t, qi = (-nr * di + ni * dr) * t;
            xr = pr - qr;
            xi = pi - qi;
            moved = __double_as_longlong(xr) != __double_as_longlong(pr) ||
                    __double_as_longlong(xi) != __double_as_longlong(pi);
            an2 = qr * qr + qi * qi;
        }
        double kr, ki;
        bcast_one<NN>(k, xr, xi, kr, ki);
        if (r > k && own) factor(kr, ki);
    }
}

template <int NN>
__device__ int dk_group(const double* c, int r, int base, uint64_t gmask, double& rre, double& rim) {
    double cr[NN + 1];
#pragma unroll
    for (int i = 0; i <= NN; ++i) cr[i] = c[i];
    // initial roots (1 + i)^r, the same products as solvePoly's sequence
    double xr = 1, xi = 0;
    {
        double pr = 1, pi = 0;
        const double qr = 1, qi = 1;
#pragma unroll
        for (int i = 0; i < NN; i++) {
            if (i == r) {
                xr = pr;
                xi = pi;
            }
            const double tr = pr * qr - pi * qi, ti = pr * qi + pi * qr;
            pr = tr;
            pi = ti;
        }
    }
    const bool own = r < NN;
    int sweeps = 0;
    for (int iter = 0; iter < 300; iter++) {
        ++sweeps;
        // the sweep without solvePoly's coincident-root skip (a select per factor); a coincidence anywhere in the group
        // is seen by its first occurrence, before which both forms computed the same values, and the sweep then runs
        // again from the same roots with the skip
        const double xr0 = xr, xi0 = xi;
        bool moved = false, hit = false;
        double an2 = 0;
        dk_sweep<NN, false>(cr, r, own, xr, xi, moved, an2, hit);
        if (__ballot(own && hit) & gmask) {
            xr = xr0;
            xi = xi0;
            dk_sweep<NN, true>(cr, r, own, xr, xi, moved, an2, hit);
        }
        // OpenCV stops when the largest |update| is 0 (an2 > 0 iff |q| > 0; NaN compares false); a sweep that moved no
        // root is a fixed point (every later sweep repeats it), so stopping there gives the 300-sweep roots too
        const uint64_t any_moved = __ballot(own && moved) & gmask, any_pos = __ballot(own && an2 > 0) & gmask;
        if (!any_moved || !any_pos) break;
    }
    rre = own ? xr : 0.0;
    rim = own ? (fabs(xi) < 1e-100 ? 0.0 : xi) : 0.0;
    return sweeps;
}

// solveZ of root (re, im) and its model: the body of runKernel's loop over the roots; false when the root is complex
// (|Im| > 1e-10) or solveZ degenerate
__device__ __forceinline__ bool em_root_model(const double* B, const double* EE, double re, double im, double* ev) {
    if (fabs(im) > 1e-10) return false;
    const double z1 = re, z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
    double bz[9];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const double* br = B + j * 13;
        bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
        bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
        bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
    }
    // SVD::solveZ: the square SVD transposes into At; the answer is the last row of Vt
    double A3[9], V3[9], w3[3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) A3[a * 3 + b] = bz[b * 3 + a];
    cv_jacobi_svd<3>(A3, w3, V3);
    const double* xy1 = V3 + 6;
    if (fabs(xy1[2]) < 1e-10) return false;
    const double xs = xy1[0] / xy1[2], ys = xy1[1] / xy1[2], zs = z1;
#pragma unroll
    for (int k = 0; k < 9; ++k) ev[k] = ((EE[0 * 9 + k] * xs + EE[1 * 9 + k] * ys) + EE[2 * 9 + k] * zs) + EE[3 * 9 + k];
    double s2 = 0;
    s2 += ev[0] * ev[0] + ev[1] * ev[1] + ev[2] * ev[2] + ev[3] * ev[3];
    s2 += ev[4] * ev[4] + ev[5] * ev[5] + ev[6] * ev[6] + ev[7] * ev[7];
    s2 += ev[8] * ev[8];
    const double sc = 1. / sqrt(s2);
#pragma unroll
    for (int k = 0; k < 9; ++k) ev[k] = ev[k] * sc;
    return true;
}

// EMEstimatorCallback::runKernel (oracle or_em_kernel); models [10][9]; returns the count.  kGroup: on a 10-lane
// group (lane r of the group at base, mask gmask) every lane forms the null space, the constraint matrix, its LU
// inverse and det B(z) redundantly, the Durand-Kerner roots are one per lane (dk_group) and lane r runs the loop's
// iteration i = r (solveZ and the model), the models landing in root order by a ballot prefix -- the latency form
// (1.5 vs 2.5 ms for one list).  Otherwise one lane per iteration (dk_solve and the loop over the ten roots) -- the
// throughput form (a whole 64-lane wave of iterations).
template <bool kGroup>
__device__ int em_models(const double* q1, const double* q2, double* models, int r, int base, uint64_t gmask,
                         int prof_k = 1 << 30) {
    EP_DECL
    double At[81], Vt5[25], W[5];
#pragma unroll
    for (int i = 0; i < 81; ++i) At[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        double* r = At + 9 * i;
        r[0] = x1 * x2; r[1] = y1 * x2; r[2] = x2 * 1.0;
        r[3] = x1 * y2; r[4] = y1 * y2; r[5] = y2 * 1.0;
        r[6] = x1 * 1.0; r[7] = y1 * 1.0; r[8] = 1.0;
    }
    cv_jacobi_svd_mn<9, 5, 9>(At, W, Vt5);
    EP_MARK(0);
    const double* EE = At + 5 * 9;
    double A[200];
    em_coeff_mat(EE, A);
    EP_MARK(1);
    // runKernel reads rows 4 .. 9 of M = inv(A[:, :10]) A[:, 10:] only (B below)
    double M4[60];
    if constexpr (kGroup) {
        lu_m_group(A, r, base, M4);
    } else {
        double inv[100];
        lu_inverse10(A, inv, 4);
        for (int i = 4; i < 10; ++i)
            for (int j = 0; j < 10; ++j) {
                double s = 0;
                for (int k = 0; k < 10; ++k) s += inv[i * 10 + k] * A[k * 20 + 10 + j];
                M4[(i - 4) * 10 + j] = s;
            }
    }
    double B[39];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const double* a1 = M4 + (i * 2) * 10;
        const double* a2 = M4 + (i * 2 + 1) * 10;
        double r1[13], r2[13];
#pragma unroll
        for (int k = 0; k < 13; ++k) r1[k] = r2[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) { r1[1 + k] = a1[k]; r1[5 + k] = a1[3 + k]; }
#pragma unroll
        for (int k = 0; k < 4; ++k) r1[9 + k] = a1[6 + k];
#pragma unroll
        for (int k = 0; k < 3; ++k) { r2[0 + k] = a2[k]; r2[4 + k] = a2[3 + k]; }
#pragma unroll
        for (int k = 0; k < 4; ++k) r2[8 + k] = a2[6 + k];
#pragma unroll
        for (int k = 0; k < 13; ++k) B[i * 13 + k] = r1[k] - r2[k];
    }
    EP_MARK(2);
    double c[11];
    em_det_poly(B, c);
    EP_MARK(3);
    int nn = 10;
    for (; nn > 1; nn--)
        if (fabs(c[nn]) + fabs(0.0) > DBL_EPSILON) break;  // solvePoly trims the vanishing leading coefficients
    int sweeps = 0, count = 0;
    if constexpr (kGroup) {
        double rre = 0, rim = 0;
        switch (nn) {  // group-uniform
            case 10: sweeps = dk_group<10>(c, r, base, gmask, rre, rim); break;
            case 9: sweeps = dk_group<9>(c, r, base, gmask, rre, rim); break;
            case 8: sweeps = dk_group<8>(c, r, base, gmask, rre, rim); break;
            case 7: sweeps = dk_group<7>(c, r, base, gmask, rre, rim); break;
            case 6: sweeps = dk_group<6>(c, r, base, gmask, rre, rim); break;
            case 5: sweeps = dk_group<5>(c, r, base, gmask, rre, rim); break;
            case 4: sweeps = dk_group<4>(c, r, base, gmask, rre, rim); break;
            case 3: sweeps = dk_group<3>(c, r, base, gmask, rre, rim); break;
            case 2: sweeps = dk_group<2>(c, r, base, gmask, rre, rim); break;
            default: sweeps = dk_group<1>(c, r, base, gmask, rre, rim); break;
        }
        EP_MARK(4);
        double ev[9];
        const bool valid = em_root_model(B, EE, rre, rim, ev);
        const uint64_t vb = __ballot(valid) & gmask;
        const int lane = (int)(threadIdx.x & 63);
        const int pos = __popcll(vb & ((1ull << lane) - 1ull));
        if (valid) {
#pragma unroll
            for (int k = 0; k < 9; ++k) models[pos * 9 + k] = ev[k];
        }
        count = __popcll(vb);
    } else {
        double rre[10], rim[10];
        switch (nn) {
            case 10: sweeps = dk_solve<10>(c, rre, rim); break;
            case 9: sweeps = dk_solve<9>(c, rre, rim); break;
            case 8: sweeps = dk_solve<8>(c, rre, rim); break;
            case 7: sweeps = dk_solve<7>(c, rre, rim); break;
            case 6: sweeps = dk_solve<6>(c, rre, rim); break;
            case 5: sweeps = dk_solve<5>(c, rre, rim); break;
            case 4: sweeps = dk_solve<4>(c, rre, rim); break;
            case 3: sweeps = dk_solve<3>(c, rre, rim); break;
            case 2: sweeps = dk_solve<2>(c, rre, rim); break;
            default: sweeps = dk_solve<1>(c, rre, rim); break;
        }
        EP_MARK(4);
        for (int i = 0; i < 10; i++) {
            double ev[9];
            if (!em_root_model(B, EE, rre[i], rim[i], ev)) continue;
#pragma unroll
            for (int k = 0; k < 9; ++k) models[count * 9 + k] = ev[k];
            count++;
        }
    }
    EP_SET(7, sweeps);
    (void)sweeps;
    EP_MARK(5);
    if (r == 0) EP_STORE(prof_k);
    (void)prof_k;
    return count;
}

// Sampson error (EMEstimatorCallback::computeError) <= t
__device__ __forceinline__ bool em_inlier(const double* E, double x1x, double x1y, double x2x, double x2y, float t) {
    const double x1[3] = {x1x, x1y, 1.}, x2[3] = {x2x, x2y, 1.};
    double Ex1[3], Etx2[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        Ex1[r] = E[r * 3 + 0] * x1[0] + E[r * 3 + 1] * x1[1] + E[r * 3 + 2] * x1[2];
        Etx2[r] = E[0 * 3 + r] * x2[0] + E[1 * 3 + r] * x2[1] + E[2 * 3 + r] * x2[2];
    }
    const double x2tEx1 = x2[0] * Ex1[0] + x2[1] * Ex1[1] + x2[2] * Ex1[2];
    const double a = Ex1[0] * Ex1[0], b = Ex1[1] * Ex1[1], c = Etx2[0] * Etx2[0], d = Etx2[1] * Etx2[1];
    const float err = (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
    return err <= t;
}

// RANSACUpdateNumIters (log / pow from the device math library: a 1-ulp difference from the host libm can only move
// cvRound at an exact .5 of num / denom)
__device__ int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - pow(1. - ep, (double)model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

// state[8] per list: 0 niters, 1 max_good, 2 iterations run, 3 models scored, 4 found, 5 n
__global__ __launch_bounds__(256) void ess_prepare_kernel(const float* __restrict__ pts1, const float* __restrict__ pts2,
                                                          const int32_t* __restrict__ counts, int pts_stride,
                                                          EssParams P, double fx, double fy, double cx, double cy,
                                                          int max_iters) {
    const int pair = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = max(min(counts[pair], pts_stride), 0);
    if (i == 0) {
        int32_t* st = P.state + 8 * pair;
        st[0] = max_iters > 1 ? max_iters : 1;
        st[1] = 0;
        st[2] = 0;
        st[3] = 0;
        st[4] = 0;
        st[5] = n;
    }
    if (i >= n) return;
    const double ax = 1. / fx, ay = 1. / fy, sx = -cx * ax, sy = -cy * ay;
    const float* a = pts1 + 2 * ((int64_t)pair * pts_stride + i);
    const float* b = pts2 + 2 * ((int64_t)pair * pts_stride + i);
    double* m1 = P.m1 + 2 * ((int64_t)pair * P.max_points + i);
    double* m2 = P.m2 + 2 * ((int64_t)pair * P.max_points + i);
    m1[0] = (double)a[0] * ax + sx;
    m1[1] = (double)a[1] * ay + sy;
    m2[0] = (double)b[0] * ax + sx;
    m2[1] = (double)b[1] * ay + sy;
}

// the draws of iterations [chunk0, chunk0 + P.chunk) of a still-running list; the RNG state carries over in
// state[6..7] (cv::RNG((uint64)-1) at chunk 0)
__global__ void ess_subsets_kernel(int n_pairs, EssParams P, int chunk0, int iters) {
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= n_pairs) return;
    int32_t* st = P.state + 8 * pair;
    const int count = st[5];
    if (count <= 5 || chunk0 >= st[0]) return;
    int32_t* idx = P.idx + (int64_t)pair * P.max_iters * 5;
    uint64_t rng = chunk0 == 0 ? (uint64_t)-1 : ((uint64_t)(uint32_t)st[7] << 32) | (uint32_t)st[6];
    const int end = min(chunk0 + P.chunk, iters);
    for (int it = chunk0; it < end; ++it) {
        int d[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            int v;
            bool dup;
            do {
                v = (int)(cv_rng_next(&rng) % (uint32_t)count + 0u);
                dup = false;
#pragma unroll
                for (int j = 0; j < i; ++j) dup |= d[j] == v;
            } while (dup);
            d[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) idx[5 * it + i] = d[i];
    }
    st[6] = (int32_t)(uint32_t)rng;
    st[7] = (int32_t)(uint32_t)(rng >> 32);
}

// Round 0 of a wide round (<= 8 lists, the whole iteration budget in one round) drawn in parallel.  The sequential
// draw stream is list-independent (cv::RNG((uint64)-1), P.rng_tab holds its states), and an iteration without a
// duplicate consumes exactly five draws, so iteration it's draws are the five from offset 5 it as long as no earlier
// iteration re-drew.  One workgroup per list: every thread takes iterations at those offsets, the first iteration f
// with a duplicate is found by a block minimum, thread 0 replays f with getSubset's re-draws, every later offset
// shifts by its extra draws, and the pass repeats from f + 1 (one pass per re-drawing iteration: ~0.5% of the
// iterations for a 2000-point list).  Lists under 64 points (frequent re-draws) and draw counts past the table run
// the sequential loop.  The RNG state after the round goes to state[6..7] as in ess_subsets_kernel.
__device__ void subsets_sequential(EssParams& P, int32_t* st, int32_t* idx, int count, uint64_t rng, int it0, int end) {
    for (int it = it0; it < end; ++it) {
        int d[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            int v;
            bool dup;
            do {
                v = (int)(cv_rng_next(&rng) % (uint32_t)count + 0u);
                dup = false;
#pragma unroll
                for (int j = 0; j < i; ++j) dup |= d[j] == v;
            } while (dup);
            d[i] = v;
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) idx[5 * it + i] = d[i];
    }
    st[6] = (int32_t)(uint32_t)rng;
    st[7] = (int32_t)(uint32_t)(rng >> 32);
}

__global__ __launch_bounds__(256) void ess_subsets_par_kernel(EssParams P, int iters) {
    __shared__ int s_red[4];
    __shared__ int s_base_it, s_base_off, s_bad;
    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int32_t* st = P.state + 8 * pair;
    const int count = st[5];
    if (count <= 5 || 0 >= st[0]) return;
    int32_t* idx = P.idx + (int64_t)pair * P.max_iters * 5;
    const int end = min(P.chunk, iters);
    const uint64_t* tab = P.rng_tab;
    const int len = P.rng_len;
    if (count < 64) {
        if (tid == 0) subsets_sequential(P, st, idx, count, ~0ull, 0, end);
        return;
    }
    int base_it = 0, base_off = 0;  // iterations < base_it are final; base_it's draws start at table offset base_off
    while (true) {
        int first = end;  // this thread's first iteration with a duplicate
        bool over = false;
        for (int it = base_it + tid; it < end; it += 256) {
            const int off = base_off + 5 * (it - base_it);
            if (off + 5 > len) {
                over = true;
                break;
            }
            int d[5];
            bool dup = false;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                d[i] = (int)((uint32_t)tab[off + i] % (uint32_t)count);
#pragma unroll
                for (int j = 0; j < i; ++j) dup |= d[j] == d[i];
            }
            if (dup) {
                first = it;
                break;  // later iterations of this thread are past it
            }
#pragma unroll
            for (int i = 0; i < 5; ++i) idx[5 * it + i] = d[i];
        }
        // block minimum of the first duplicate, and any table overflow
        int m = first;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o, 64));
        const bool any_over = __syncthreads_or(over);
        if (lane == 0) s_red[wave] = m;
        __syncthreads();
        const int f = min(min(s_red[0], s_red[1]), min(s_red[2], s_red[3]));
        if (any_over) {  // a pathological re-draw count: the sequential stream from the start
            if (tid == 0) subsets_sequential(P, st, idx, count, ~0ull, 0, end);
            return;
        }
        if (f >= end) {  // every iteration from base_it on is final
            if (tid == 0) {
                const int off_end = base_off + 5 * (end - base_it);
                const uint64_t rng = off_end > 0 ? tab[off_end - 1] : ~0ull;
                st[6] = (int32_t)(uint32_t)rng;
                st[7] = (int32_t)(uint32_t)(rng >> 32);
            }
            return;
        }
        if (tid == 0) {  // iteration f with getSubset's re-draws
            int off = base_off + 5 * (f - base_it);
            int d[5];
            bool bad = false;
            for (int i = 0; i < 5 && !bad; ++i) {
                int v;
                bool dup;
                do {
                    if (off >= len) {
                        bad = true;
                        break;
                    }
                    v = (int)((uint32_t)tab[off++] % (uint32_t)count);
                    dup = false;
                    for (int j = 0; j < i; ++j) dup |= d[j] == v;
                } while (dup);
                d[i] = v;
            }
            if (!bad)
                for (int i = 0; i < 5; ++i) idx[5 * f + i] = d[i];
            s_bad = bad ? 1 : 0;
            s_base_it = f + 1;
            s_base_off = off;
        }
        __syncthreads();
        if (s_bad) {
            if (tid == 0) subsets_sequential(P, st, idx, count, ~0ull, 0, end);
            return;
        }
        base_it = s_base_it;
        base_off = s_base_off;
        __syncthreads();  // s_red / s_base_* are rewritten by the next pass
    }
}

// The five-point models of a round.  kGroup (workspaces of <= kEssWidePairs lists, latency): a 64-lane workgroup
// holds four RANSAC iterations, one per 16-lane row, whose lanes 0 .. 9 are the group (10 .. 15 idle: the row
// broadcasts of dk_group need the group inside one DPP row).  Otherwise (throughput) one iteration per lane, 64 per
// workgroup.
constexpr int kModelGroup = 10;
constexpr int kModelRow = 16;
constexpr int kModelIters = 4;  // iterations per workgroup in the group form

template <bool kGroup>
__global__ __launch_bounds__(64) void ess_models_kernel(EssParams P, int chunk0) {
    const int pair = blockIdx.y;
    const int lane = threadIdx.x;
    const int g = kGroup ? lane / kModelRow : lane;
    const int r = kGroup ? lane - g * kModelRow : 0;
    const int base = kGroup ? g * kModelRow : lane;
    const int k = blockIdx.x * (kGroup ? kModelIters : 64) + g;
    if ((kGroup && r >= kModelGroup) || k >= P.chunk) return;  // whole groups leave together
    const uint64_t gmask = kGroup ? ((1ull << kModelGroup) - 1ull) << base : 1ull << lane;
    const int it = chunk0 + k;
    const int32_t* st = P.state + 8 * pair;
    const int n = st[5];
    int32_t* nmod = P.nmod + pair * P.chunk + k;
    const bool single = n == 5;
    if (n < 5 || it >= st[0] || (single && it > 0)) {
        if (r == 0) *nmod = 0;
        return;
    }
    const double* m1 = P.m1 + 2 * (int64_t)pair * P.max_points;
    const double* m2 = P.m2 + 2 * (int64_t)pair * P.max_points;
    double q1[10], q2[10];
    const int32_t* idx = P.idx + ((int64_t)pair * P.max_iters + it) * 5;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const int j = single ? i : idx[i];
        q1[2 * i] = m1[2 * j];
        q1[2 * i + 1] = m1[2 * j + 1];
        q2[2 * i] = m2[2 * j];
        q2[2 * i + 1] = m2[2 * j + 1];
    }
    double* out = P.models + ((int64_t)pair * P.chunk + k) * 90;
    const int cnt = em_models<kGroup>(q1, q2, out, r, base, gmask, pair == 0 ? it : 1 << 30);
    if (r == 0) *nmod = cnt;
}

__global__ __launch_bounds__(256) void ess_score_kernel(EssParams P, int chunk0, float t) {
    __shared__ double s_E[90];
    __shared__ int s_cnt[10];
    const int pair = blockIdx.y;
    const int k = blockIdx.x;
    const int32_t* st = P.state + 8 * pair;
    const int n = st[5];
    const int nm = P.nmod[pair * P.chunk + k];
    if (n <= 5 || chunk0 + k >= st[0] || nm == 0) return;
    const double* src = P.models + ((int64_t)pair * P.chunk + k) * 90;
    for (int i = threadIdx.x; i < nm * 9; i += 256) s_E[i] = src[i];
    if (threadIdx.x < 10) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const double* m1 = P.m1 + 2 * (int64_t)pair * P.max_points;
    const double* m2 = P.m2 + 2 * (int64_t)pair * P.max_points;
    int cnt[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < n; i += 256) {
        const double a = m1[2 * i], b = m1[2 * i + 1], c = m2[2 * i], d = m2[2 * i + 1];
#pragma unroll
        for (int m = 0; m < 10; ++m)
            if (m < nm) cnt[m] += em_inlier(s_E + 9 * m, a, b, c, d, t) ? 1 : 0;
    }
#pragma unroll
    for (int m = 0; m < 10; ++m) {
        int v = cnt[m];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (m < nm && (threadIdx.x & 63) == 0 && v) atomicAdd(&s_cnt[m], v);
    }
    __syncthreads();
    if (threadIdx.x < nm) P.good[(pair * P.chunk + k) * 10 + threadIdx.x] = s_cnt[threadIdx.x];
}

__global__ void ess_select_kernel(EssParams P, int n_pairs, int chunk0, double prob) {
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= n_pairs) return;
    int32_t* st = P.state + 8 * pair;
    const int n = st[5];
    if (n < 5) return;
    const int32_t* nmod = P.nmod + pair * P.chunk;
    const double* models = P.models + (int64_t)pair * P.chunk * 90;
    double* best = P.best + 9 * pair;
    if (n == 5) {
        if (chunk0 == 0) {
            st[2] = 1;
            st[3] = nmod[0];
            st[1] = n;
            if (nmod[0] > 0) {
                st[4] = 1;
                for (int q = 0; q < 9; ++q) best[q] = models[q];
            }
        }
        return;
    }
    int niters = st[0], max_good = st[1], run = st[2], total = st[3];
    const int32_t* good = P.good + pair * P.chunk * 10;
    for (int k = 0; k < P.chunk; ++k) {
        const int it = chunk0 + k;
        if (it >= niters) break;
        const int nm = nmod[k];
        total += nm;
        for (int m = 0; m < nm; ++m) {
            const int g = good[k * 10 + m];
            if (g > (max_good > 4 ? max_good : 4)) {
                for (int q = 0; q < 9; ++q) best[q] = models[k * 90 + m * 9 + q];
                max_good = g;
                niters = update_num_iters(prob, (double)(n - g) / n, 5, niters);
            }
        }
        run = it + 1;
    }
    st[0] = niters;
    st[1] = max_good;
    st[2] = run;
    st[3] = total;
    st[4] = max_good > 0 ? 1 : 0;
}

__global__ __launch_bounds__(256) void ess_output_kernel(EssParams P, int pts_stride, float t, double* __restrict__ E,
                                                         uint8_t* __restrict__ mask, int32_t* __restrict__ found,
                                                         int32_t* __restrict__ stats) {
    const int pair = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int32_t* st = P.state + 8 * pair;
    const int n = st[5];
    const bool ok = st[4] != 0;
    const double* best = P.best + 9 * pair;
    if (i == 0) {
        found[pair] = ok ? 1 : 0;
        for (int q = 0; q < 9; ++q) E[9 * pair + q] = ok ? best[q] : 0.0;
        if (stats) {
            stats[3 * pair + 0] = st[2];
            stats[3 * pair + 1] = st[3];
            stats[3 * pair + 2] = st[1];
        }
    }
    if (!mask || i >= n) return;
    uint8_t f = 0;
    if (ok) {
        if (n == 5) {
            f = 1;
        } else {
            const double* m1 = P.m1 + 2 * ((int64_t)pair * P.max_points + i);
            const double* m2 = P.m2 + 2 * ((int64_t)pair * P.max_points + i);
            f = em_inlier(best, m1[0], m1[1], m2[0], m2[1], t) ? 1 : 0;
        }
    }
    mask[(int64_t)pair * pts_stride + i] = f;
}

// ------------------------------------------------------------------------------------------------
// recoverPose
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double det3(const double* a) {
    return a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
}
__device__ __forceinline__ void mm3x3(const double* A, const double* B, double* C) {
    double R[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s += A[i * 3 + k] * B[k * 3 + j];
            R[i * 3 + j] = s;
        }
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = R[i];
}

__global__ void rp_decompose_kernel(const double* __restrict__ Ein, int n_pairs, EssParams P) {
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= n_pairs) return;
    const double* E = Ein + 9 * pair;
    // SVD::compute(E, D, U, Vt): temp_a = E^T, u = transpose(temp_a), vt = temp_v
    double At[9], Vt[9], w[3], U[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) At[i * 3 + j] = E[j * 3 + i];
    cv_jacobi_svd<3>(At, w, Vt);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) U[i * 3 + j] = At[j * 3 + i];
    if (det3(U) < 0)
#pragma unroll
        for (int i = 0; i < 9; ++i) U[i] *= -1.;
    if (det3(Vt) < 0)
#pragma unroll
        for (int i = 0; i < 9; ++i) Vt[i] *= -1.;
    const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1}, Wt[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    double T[9], R1[9], R2[9];
    mm3x3(U, W, T);
    mm3x3(T, Vt, R1);
    mm3x3(U, Wt, T);
    mm3x3(T, Vt, R2);
    double* cand = P.cand + 48 * pair;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double* R = (c & 1) ? R2 : R1;
#pragma unroll
            for (int j = 0; j < 3; ++j) cand[c * 12 + i * 4 + j] = R[i * 3 + j] * 1.0;
            const double ti = U[i * 3 + 2] * 1.0;
            cand[c * 12 + i * 4 + 3] = c < 2 ? ti * 1.0 : -ti * 1.0;
        }
#pragma unroll
    for (int c = 0; c < 4; ++c) P.cgood[4 * pair + c] = 0;
}

// lane l of a wave: point blockIdx.x * 16 + l / 4, candidate l % 4
__global__ __launch_bounds__(64) void rp_count_kernel(const float* __restrict__ pts1, const float* __restrict__ pts2,
                                                      const int32_t* __restrict__ counts, int pts_stride, EssParams P,
                                                      Mat3 K) {
    __shared__ double s_P[48];
    const int pair = blockIdx.y;
    const int c = threadIdx.x & 3;
    const int i = blockIdx.x * 16 + (threadIdx.x >> 2);
    const int n = max(min(counts[pair], pts_stride), 0);
    if (blockIdx.x * 16 >= n) return;
    if (threadIdx.x < 48) s_P[threadIdx.x] = P.cand[48 * pair + threadIdx.x];
    __syncthreads();
    const double fx = K.v[0], fy = K.v[4], cx = K.v[2], cy = K.v[5], dist = 50.0;
    const double ax = 1. / fx, ay = 1. / fy, sx = -cx * ax, sy = -cy * ay;
    double a[2] = {0, 0}, b[2] = {0, 0};
    if (i < n) {
        const float* p1 = pts1 + 2 * ((int64_t)pair * pts_stride + i);
        const float* p2 = pts2 + 2 * ((int64_t)pair * pts_stride + i);
        a[0] = (double)p1[0] * ax + sx;
        a[1] = (double)p1[1] * ay + sy;
        b[0] = (double)p2[0] * ax + sx;
        b[1] = (double)p2[1] * ay + sy;
    }
    const double* Pc = s_P + 12 * c;
    // cvTriangulatePoints: rows x P[2] - P[0], y P[2] - P[1] for P0 = [I | 0] (a) and Pc (b)
    double A[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double p0r0 = k == 0 ? 1.0 : 0.0, p0r1 = k == 1 ? 1.0 : 0.0, p0r2 = k == 2 ? 1.0 : 0.0;
        A[0 * 4 + k] = a[0] * p0r2 - p0r0;
        A[1 * 4 + k] = a[1] * p0r2 - p0r1;
        A[2 * 4 + k] = b[0] * Pc[2 * 4 + k] - Pc[0 * 4 + k];
        A[3 * 4 + k] = b[1] * Pc[2 * 4 + k] - Pc[1 * 4 + k];
    }
    double At[16], V[16], w[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) At[r * 4 + q] = A[q * 4 + r];
    cv_jacobi_svd<4>(At, w, V);
    const double Q0 = V[12], Q1 = V[13], Q2 = V[14], Q3 = V[15];
    bool ok = Q2 * Q3 > 0;
    const double X[4] = {Q0 / Q3, Q1 / Q3, Q2 / Q3, Q3 / Q3};
    ok = (X[2] < dist) && ok;
    double z = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) z += Pc[2 * 4 + k] * X[k];
    ok = (z > 0) && ok;
    ok = (z < dist) && ok;
    ok = ok && i < n;
    const uint64_t bal = __ballot(ok);
    if (threadIdx.x < 4) atomicAdd(&P.cgood[4 * pair + c], (int)__popcll(bal & (0x1111111111111111ull << c)));
}

__global__ void rp_select_kernel(int n_pairs, EssParams P, double* __restrict__ R, double* __restrict__ t,
                                 int32_t* __restrict__ good_out) {
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= n_pairs) return;
    const int32_t* g = P.cgood + 4 * pair;
    int pick;
    if (g[0] >= g[1] && g[0] >= g[2] && g[0] >= g[3]) pick = 0;
    else if (g[1] >= g[0] && g[1] >= g[2] && g[1] >= g[3]) pick = 1;
    else if (g[2] >= g[0] && g[2] >= g[1] && g[2] >= g[3]) pick = 2;
    else pick = 3;
    const double* cand = P.cand + 48 * pair + 12 * pick;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) R[9 * pair + i * 3 + j] = cand[i * 4 + j];
        t[3 * pair + i] = cand[i * 4 + 3];
    }
    if (good_out) good_out[pair] = g[pick];
}

}  // namespace ess

#ifdef YAVO_LM_PROFILE
extern "C" int yv_debug_ess_prof(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(ess::g_ess_prof), sizeof(unsigned long long) * 256 * 8) == hipSuccess
               ? 0 : -2;
}
#endif

void launch_find_essential(const EssParams& P, const EssRun& r, const float* pts1, const float* pts2,
                           const int32_t* counts, int n_pairs, int pts_stride, double* E, uint8_t* mask,
                           int32_t* found, int32_t* stats, hipStream_t s) {
    if (n_pairs <= 0) return;
    const int iters = r.max_iters > 1 ? r.max_iters : 1;
    dim3 gpts((P.max_points + 255) / 256, n_pairs);
    hipLaunchKernelGGL(ess::ess_prepare_kernel, gpts, dim3(256), 0, s, pts1, pts2, counts, pts_stride, P, r.focal,
                       r.focal, r.ppx, r.ppy, iters);
    double thr = r.threshold;
    thr /= (r.focal + r.focal) / 2;
    const float t = (float)(thr * thr);
    for (int c0 = 0; c0 < iters; c0 += P.chunk) {
        if (c0 == 0 && P.rng_tab && P.chunk >= iters)  // the whole budget in one wide round: parallel draws
            hipLaunchKernelGGL(ess::ess_subsets_par_kernel, dim3(n_pairs), dim3(256), 0, s, P, iters);
        else
            hipLaunchKernelGGL(ess::ess_subsets_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, s, n_pairs, P, c0, iters);
        if (P.chunk == kEssChunkWide)  // few lists: the latency form
            hipLaunchKernelGGL(ess::ess_models_kernel<true>,
                               dim3((P.chunk + ess::kModelIters - 1) / ess::kModelIters, n_pairs), dim3(64), 0, s, P, c0);
        else
            hipLaunchKernelGGL(ess::ess_models_kernel<false>, dim3((P.chunk + 63) / 64, n_pairs), dim3(64), 0, s, P, c0);
        hipLaunchKernelGGL(ess::ess_score_kernel, dim3(P.chunk, n_pairs), dim3(256), 0, s, P, c0, t);
        hipLaunchKernelGGL(ess::ess_select_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, s, P, n_pairs, c0, r.prob);
    }
    hipLaunchKernelGGL(ess::ess_output_kernel, gpts, dim3(256), 0, s, P, pts_stride, t, E, mask, found, stats);
}

void launch_recover_pose(const EssParams& P, const double* E, const float* pts1, const float* pts2,
                         const int32_t* counts, int n_pairs, int pts_stride, const Mat3& K, double* R, double* t,
                         int32_t* good, hipStream_t s) {
    if (n_pairs <= 0) return;
    hipLaunchKernelGGL(ess::rp_decompose_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, s, E, n_pairs, P);
    hipLaunchKernelGGL(ess::rp_count_kernel, dim3((P.max_points + 15) / 16, n_pairs), dim3(64), 0, s, pts1, pts2,
                       counts, pts_stride, P, K);
    hipLaunchKernelGGL(ess::rp_select_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, s, n_pairs, P, R, t, good);
}

}  // namespace yavo
