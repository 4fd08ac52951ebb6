/*
 * yavo_oracle_essential.c -- CPU restatement of cv::findEssentialMat (RANSAC) and cv::recoverPose as the reference
 * calls them at initialisation / re-initialisation:
 *     E = cv::findEssentialMat(currFeatures, prevFeatures, 718.8560, Point2d(607.1928, 185.2157), cv::RANSAC,
 *                              0.999, 1.0, mask);                        src/LoopHandler.cc:239 and :581
 *     cv::recoverPose(E, currFramePts, lastFramePts, K, R, t);           src/LoopHandler.cc:256 and :598
 * (points are the reference's (x = row, y = col) KeyPoint coordinates, used literally with pp = (cx, cy)).
 * TEST INFRASTRUCTURE ONLY (see yavo_oracle.h).
 *
 * OpenCV is absent from this image and the reference does not pin its version (CMakeLists.txt:6), so this restates
 * the classic (non-USAC) OpenCV 4.x path from its published algorithm; parity with the reference binary is
 * unpinned (no reference fixture holds E, R or t):
 *   findEssentialMat   points normalised as MatExpr evaluates (p - c) / f: p * (1/f) + (-c * (1/f)); threshold / f
 *   RANSAC             RANSACPointSetRegistrator::run: cv::RNG((uint64)-1), getSubset (5 distinct draws, redraw on a
 *                      repeat), every model of a subset scored, best iff count > max(best, 4), niters from
 *                      RANSACUpdateNumIters(0.999, outlier ratio, 5, niters), maxIters 1000
 *   EM kernel          EMEstimatorCallback::runKernel: SVD (JacobiSVD, FULL_UV) of the 5 x 9 epipolar rows, null
 *                      space = Vt rows 5..8; the 10 x 20 cubic-constraint matrix (det E = 0, 2 E E^T E - tr(E E^T) E
 *                      = 0) over the monomials x^3 y^3 x^2y xy^2 x^2z x^2 y^2z y^2 xyz xy | xz^2 xz x yz^2 yz y z^3
 *                      z^2 z 1; inv(A[:, :10]) (LUImpl, partial pivoting) * A[:, 10:]; B = row(2i+4) - z row(2i+5)
 *                      (3 x 13); det B(z) -> degree-10 polynomial; solvePoly (Durand-Kerner from (1 + i)^k, 300
 *                      iterations or until no root moves); per real root (|im| <= 1e-10) SVD::solveZ on B(z)
 *                      -> (x, y, 1); E = x E0 + y E1 + z E2 + E3 scaled by 1 / ||E||
 *   scoring            EMEstimatorCallback::computeError: float Sampson distance, inlier iff err <= (float)thr^2
 *   recoverPose        decomposeEssentialMat (SVD, sign-fixed U / Vt, R = U W Vt, U W^T Vt, t = U col 2); for the
 *                      four (R, +-t): triangulatePoints (4 x 4 JacobiSVD per point, last row of Vt), cheirality and
 *                      distance 50 in both views; the first maximum count in the order (R1,t) (R2,t) (R1,-t) (R2,-t)
 * Where this restatement picks an order OpenCV does not expose it is stated at the function: getCoeffMat (OpenCV's
 * generated expansion) is built here by polynomial products in a fixed term order, rows 0..8 = entries of the trace
 * constraint (row-major), row 9 = det E; solvePoly's branch for exactly coincident iterates (num_same_root > 1) is
 * not restated (the plain step is taken).  The GPU path (yavo_essential.hip) follows these orders bit for bit.
 */
#include "yavo_oracle.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------------------------- */
/* cv::RNG and getSubset                                                                            */
/* ---------------------------------------------------------------------------------------------- */
static uint32_t rng_next(uint64_t* s) {
    *s = (uint64_t)(uint32_t)*s * 4164903690ULL + (uint32_t)(*s >> 32);
    return (uint32_t)*s;
}
/* RNG::uniform(int a, int b) = a == b ? a : (int)(next() % (b - a) + a) */
static int rng_uniform(uint64_t* s, int a, int b) { return a == b ? a : (int)(rng_next(s) % (uint32_t)(b - a) + (uint32_t)a); }

void or_em_subsets(int count, int iters, int32_t* idx) {
    uint64_t rng = (uint64_t)-1; /* RNG((uint64)-1) in RANSACPointSetRegistrator::run */
    for (int it = 0; it < iters; ++it) {
        int32_t* d = idx + 5 * it;
        for (int i = 0; i < 5; ++i) {
            int v, dup;
            do {
                v = rng_uniform(&rng, 0, count);
                dup = 0;
                for (int j = 0; j < i; ++j) dup |= d[j] == v;
            } while (dup);
            d[i] = v;
        }
    }
}

/* ---------------------------------------------------------------------------------------------- */
/* polynomials in (x, y, z) of degree <= 3, fixed term orders                                       */
/* ---------------------------------------------------------------------------------------------- */
/* linear terms: x y z 1 */
static const int kLinExp[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
/* quadratic terms: x^2 xy xz x y^2 yz y z^2 z 1 */
static const int kQuadExp[10][3] = {{2, 0, 0}, {1, 1, 0}, {1, 0, 1}, {1, 0, 0}, {0, 2, 0},
                                    {0, 1, 1}, {0, 1, 0}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
/* cubic terms in OpenCV's / Nister's column order */
static const int kCubExp[20][3] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                                   {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                                   {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};

static int quad_index(int a, int b, int c) {
    for (int i = 0; i < 10; ++i)
        if (kQuadExp[i][0] == a && kQuadExp[i][1] == b && kQuadExp[i][2] == c) return i;
    return -1;
}
static int cub_index(int a, int b, int c) {
    for (int i = 0; i < 20; ++i)
        if (kCubExp[i][0] == a && kCubExp[i][1] == b && kCubExp[i][2] == c) return i;
    return -1;
}
/* R = P * Q: for p (P's order) for q (Q's order): R[term(p + q)] += P[p] * Q[q], R from 0 */
static void mul_lin_lin(const double* P, const double* Q, double* R) {
    for (int i = 0; i < 10; ++i) R[i] = 0.0;
    for (int p = 0; p < 4; ++p)
        for (int q = 0; q < 4; ++q) {
            const int t = quad_index(kLinExp[p][0] + kLinExp[q][0], kLinExp[p][1] + kLinExp[q][1], kLinExp[p][2] + kLinExp[q][2]);
            R[t] += P[p] * Q[q];
        }
}
static void mul_quad_lin(const double* P, const double* Q, double* R) {
    for (int i = 0; i < 20; ++i) R[i] = 0.0;
    for (int p = 0; p < 10; ++p)
        for (int q = 0; q < 4; ++q) {
            const int t = cub_index(kQuadExp[p][0] + kLinExp[q][0], kQuadExp[p][1] + kLinExp[q][1], kQuadExp[p][2] + kLinExp[q][2]);
            R[t] += P[p] * Q[q];
        }
}

/* getCoeffMat: A (10 x 20, row-major) from the null-space basis EE[4][9] (E(x, y, z) = x E0 + y E1 + z E2 + E3) */
void or_em_coeff_mat(const double* EE, double* A) {
    double e[9][4]; /* entry k of E as a linear polynomial (x, y, z, 1) */
    for (int k = 0; k < 9; ++k)
        for (int v = 0; v < 4; ++v) e[k][v] = EE[v * 9 + k];
    /* S = E E^T (quadratic): S_ij = sum_k e_ik e_jk, k ascending, termwise */
    double S[9][10];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double t[10];
            mul_lin_lin(e[i * 3 + 0], e[j * 3 + 0], S[i * 3 + j]);
            for (int k = 1; k < 3; ++k) {
                mul_lin_lin(e[i * 3 + k], e[j * 3 + k], t);
                for (int q = 0; q < 10; ++q) S[i * 3 + j][q] = S[i * 3 + j][q] + t[q];
            }
        }
    double tr[10];
    for (int q = 0; q < 10; ++q) tr[q] = S[0][q] + S[4][q] + S[8][q];
    /* rows 0..8: 2 (E E^T E)_ij - tr(E E^T) E_ij */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc[20], t[20];
            mul_quad_lin(S[i * 3 + 0], e[0 * 3 + j], acc);
            for (int k = 1; k < 3; ++k) {
                mul_quad_lin(S[i * 3 + k], e[k * 3 + j], t);
                for (int q = 0; q < 20; ++q) acc[q] = acc[q] + t[q];
            }
            mul_quad_lin(tr, e[i * 3 + j], t);
            double* row = A + (i * 3 + j) * 20;
            for (int q = 0; q < 20; ++q) row[q] = 2.0 * acc[q] - t[q];
        }
    /* row 9: det E = e0 (e4 e8 - e5 e7) - e1 (e3 e8 - e5 e6) + e2 (e3 e7 - e4 e6) */
    {
        double m1[10], m2[10], d[10], c0[20], c1[20], c2[20];
        mul_lin_lin(e[4], e[8], m1);
        mul_lin_lin(e[5], e[7], m2);
        for (int q = 0; q < 10; ++q) d[q] = m1[q] - m2[q];
        mul_quad_lin(d, e[0], c0);
        mul_lin_lin(e[3], e[8], m1);
        mul_lin_lin(e[5], e[6], m2);
        for (int q = 0; q < 10; ++q) d[q] = m1[q] - m2[q];
        mul_quad_lin(d, e[1], c1);
        mul_lin_lin(e[3], e[7], m1);
        mul_lin_lin(e[4], e[6], m2);
        for (int q = 0; q < 10; ++q) d[q] = m1[q] - m2[q];
        mul_quad_lin(d, e[2], c2);
        double* row = A + 9 * 20;
        for (int q = 0; q < 20; ++q) row[q] = c0[q] - c1[q] + c2[q];
    }
}

/* cv::invert(DECOMP_LU) of an n x n (n > 3): LUImpl<double> on a copy with b = I, eps = 100 DBL_EPSILON; on a
 * singular pivot the result is all zeros.  A is read with row stride lda. */
static int lu_inverse(const double* A, int lda, int n, double* inv) {
    double a[100], b[100];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            a[i * n + j] = A[i * lda + j];
            b[i * n + j] = i == j ? 1.0 : 0.0;
        }
    const double eps = DBL_EPSILON * 100;
    int ok = 1;
    for (int i = 0; i < n && ok; i++) {
        int k = i;
        for (int j = i + 1; j < n; j++)
            if (fabs(a[j * n + i]) > fabs(a[k * n + i])) k = j;
        if (fabs(a[k * n + i]) < eps) {
            ok = 0;
            break;
        }
        if (k != i) {
            for (int j = i; j < n; j++) { double t = a[i * n + j]; a[i * n + j] = a[k * n + j]; a[k * n + j] = t; }
            for (int j = 0; j < n; j++) { double t = b[i * n + j]; b[i * n + j] = b[k * n + j]; b[k * n + j] = t; }
        }
        const double d = -1 / a[i * n + i];
        for (int j = i + 1; j < n; j++) {
            const double alpha = a[j * n + i] * d;
            for (int q = i + 1; q < n; q++) a[j * n + q] += alpha * a[i * n + q];
            for (int q = 0; q < n; q++) b[j * n + q] += alpha * b[i * n + q];
        }
    }
    if (!ok) {
        for (int i = 0; i < n * n; ++i) inv[i] = 0.0;
        return 0;
    }
    for (int i = n - 1; i >= 0; i--)
        for (int j = 0; j < n; j++) {
            double s = b[i * n + j];
            for (int q = i + 1; q < n; q++) s -= a[i * n + q] * b[q * n + j];
            b[i * n + j] = s / a[i * n + i];
        }
    for (int i = 0; i < n * n; ++i) inv[i] = b[i];
    return 1;
}

/* ascending-coefficient polynomial product, R from 0, p outer q inner */
static void pmul(const double* P, int np, const double* Q, int nq, double* R) {
    for (int i = 0; i < np + nq - 1; ++i) R[i] = 0.0;
    for (int p = 0; p < np; ++p)
        for (int q = 0; q < nq; ++q) R[p + q] += P[p] * Q[q];
}

/* B (3 x 13, OpenCV layout: x part z^3 z^2 z 1, y part z^3 .. 1, constant part z^4 .. 1) -> det B(z), ascending
 * c[0 .. 10]: det = bx0 (by1 b12 - b11 by2) - by0 (bx1 b12 - b11 bx2) + b10 (bx1 by2 - by1 bx2) */
void or_em_det_poly(const double* B, double* c) {
    double px[3][4], py[3][4], p1[3][5];
    for (int i = 0; i < 3; ++i) {
        const double* br = B + 13 * i;
        for (int k = 0; k < 4; ++k) {
            px[i][k] = br[3 - k];
            py[i][k] = br[7 - k];
        }
        for (int k = 0; k < 5; ++k) p1[i][k] = br[12 - k];
    }
    double u[8], v[8], d[8], t0[11], t1[11], t2[11];
    pmul(py[1], 4, p1[2], 5, u);
    pmul(p1[1], 5, py[2], 4, v);
    for (int k = 0; k < 8; ++k) d[k] = u[k] - v[k];
    pmul(px[0], 4, d, 8, t0);
    pmul(px[1], 4, p1[2], 5, u);
    pmul(p1[1], 5, px[2], 4, v);
    for (int k = 0; k < 8; ++k) d[k] = u[k] - v[k];
    pmul(py[0], 4, d, 8, t1);
    double w[7], x[7], d2[7];
    pmul(px[1], 4, py[2], 4, w);
    pmul(py[1], 4, px[2], 4, x);
    for (int k = 0; k < 7; ++k) d2[k] = w[k] - x[k];
    pmul(p1[0], 5, d2, 7, t2);
    for (int k = 0; k < 11; ++k) c[k] = t0[k] - t1[k] + t2[k];
}

/* cv::solvePoly (Durand-Kerner), real coefficients c[0..n0] ascending, maxIters 300.  roots: re/im pairs. */
typedef struct { double re, im; } cplx;
static cplx cmul(cplx a, cplx b) { cplx r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; return r; }
static cplx cadd(cplx a, cplx b) { cplx r = {a.re + b.re, a.im + b.im}; return r; }
static cplx csub(cplx a, cplx b) { cplx r = {a.re - b.re, a.im - b.im}; return r; }
static cplx cdiv(cplx a, cplx b) {
    const double t = 1. / (b.re * b.re + b.im * b.im);
    cplx r = {(a.re * b.re + a.im * b.im) * t, (-a.re * b.im + a.im * b.re) * t};
    return r;
}
int or_solve_poly(const double* c, int n0, int max_iters, double* roots_out) {
    cplx coeffs[16], roots[16];
    for (int i = 0; i <= n0; ++i) { coeffs[i].re = c[i]; coeffs[i].im = 0.0; }
    int n = n0;
    for (; n > 1; n--) {
        if (fabs(coeffs[n].re) + fabs(coeffs[n].im) > DBL_EPSILON) break;
        roots[n - 1].re = roots[n - 1].im = 0.0;
    }
    cplx p = {1, 0}, r = {1, 1};
    for (int i = 0; i < n; i++) {
        roots[i] = p;
        p = cmul(p, r);
    }
    int iter;
    for (iter = 0; iter < max_iters; iter++) {
        double maxDiff = 0;
        for (int i = 0; i < n; i++) {
            p = roots[i];
            cplx num = coeffs[n], denom = coeffs[n];
            for (int j = 0; j < n; j++) {
                num = cadd(cmul(num, p), coeffs[n - j - 1]);
                if (j != i && (p.re != roots[j].re || p.im != roots[j].im)) denom = cmul(denom, csub(p, roots[j]));
            }
            num = cdiv(num, denom);
            roots[i] = csub(p, num);
            const double an = sqrt(num.re * num.re + num.im * num.im);
            maxDiff = maxDiff < an ? an : maxDiff; /* std::max */
        }
        if (maxDiff <= 0) break;
    }
    for (int i = 0; i < n; i++)
        if (fabs(roots[i].im) < 1e-100) roots[i].im = 0;
    for (int i = 0; i < n0; ++i) {
        roots_out[2 * i] = roots[i].re;
        roots_out[2 * i + 1] = roots[i].im;
    }
    return iter;
}

/* EMEstimatorCallback::runKernel on 5 normalised correspondences q1[5][2], q2[5][2] -> up to 10 models [10][9] */
int or_em_kernel(const double* q1, const double* q2, double* models) {
    /* SVD::compute(Q 5 x 9, FULL_UV): m < n -> temp_a = Q (5 rows of 9), JacobiSVD(m = 9, n = 5, n1 = 9); vt = At */
    double At[81], Vt5[25], W[5];
    memset(At, 0, sizeof At);
    for (int i = 0; i < 5; ++i) {
        const double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        double* r = At + 9 * i;
        r[0] = x1 * x2; r[1] = y1 * x2; r[2] = x2 * 1.0;
        r[3] = x1 * y2; r[4] = y1 * y2; r[5] = y2 * 1.0;
        r[6] = x1 * 1.0; r[7] = y1 * 1.0; r[8] = 1.0;
    }
    or_cv_jacobi_svd(At, 9, W, Vt5, 5, 9, 5, 9);
    const double* EE = At + 5 * 9; /* Vt rows 5..8 = E0, E1, E2, E3 */
    double A[200];
    or_em_coeff_mat(EE, A);
    double inv[100], M[100];
    lu_inverse(A, 20, 10, inv);
    for (int i = 0; i < 10; ++i)
        for (int j = 0; j < 10; ++j) {
            double s = 0;
            for (int k = 0; k < 10; ++k) s += inv[i * 10 + k] * A[k * 20 + 10 + j];
            M[i * 10 + j] = s;
        }
    double B[39];
    for (int i = 0; i < 3; i++) {
        const double* a1 = M + (i * 2 + 4) * 10;
        const double* a2 = M + (i * 2 + 5) * 10;
        double r1[13], r2[13];
        for (int k = 0; k < 13; ++k) r1[k] = r2[k] = 0.0;
        for (int k = 0; k < 3; ++k) { r1[1 + k] = a1[k]; r1[5 + k] = a1[3 + k]; }
        for (int k = 0; k < 4; ++k) r1[9 + k] = a1[6 + k];
        for (int k = 0; k < 3; ++k) { r2[0 + k] = a2[k]; r2[4 + k] = a2[3 + k]; }
        for (int k = 0; k < 4; ++k) r2[8 + k] = a2[6 + k];
        for (int k = 0; k < 13; ++k) B[i * 13 + k] = r1[k] - r2[k];
    }
    double c[11], roots[20];
    or_em_det_poly(B, c);
    or_solve_poly(c, 10, 300, roots);
    int count = 0;
    for (int i = 0; i < 10; i++) {
        if (fabs(roots[2 * i + 1]) > 1e-10) continue;
        const double z1 = roots[2 * i], z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
        double bz[9];
        for (int j = 0; j < 3; j++) {
            const double* br = B + j * 13;
            bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
            bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
            bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
        }
        double w3[3], vt3[9];
        or_cv_svd(bz, 3, w3, NULL, vt3); /* SVD::solveZ: last row of vt */
        const double* xy1 = vt3 + 6;
        if (fabs(xy1[2]) < 1e-10) continue;
        const double xs = xy1[0] / xy1[2], ys = xy1[1] / xy1[2], zs = z1;
        double ev[9];
        for (int k = 0; k < 9; ++k) ev[k] = ((EE[0 * 9 + k] * xs + EE[1 * 9 + k] * ys) + EE[2 * 9 + k] * zs) + EE[3 * 9 + k];
        /* cv::norm (normL2Sqr, 4-way unrolled), then Evec /= norm as a scale by 1 / norm */
        double s2 = 0;
        int k = 0;
        for (; k <= 9 - 4; k += 4) s2 += ev[k] * ev[k] + ev[k + 1] * ev[k + 1] + ev[k + 2] * ev[k + 2] + ev[k + 3] * ev[k + 3];
        for (; k < 9; ++k) s2 += ev[k] * ev[k];
        const double sc = 1. / sqrt(s2);
        for (k = 0; k < 9; ++k) models[count * 9 + k] = ev[k] * sc;
        count++;
    }
    return count;
}

/* EMEstimatorCallback::computeError + findInliers; returns the inlier count */
static int em_inliers(const double* m1, const double* m2, int n, const double* E, float t, uint8_t* mask) {
    int nz = 0;
    for (int i = 0; i < n; i++) {
        const double x1[3] = {m1[2 * i], m1[2 * i + 1], 1.};
        const double x2[3] = {m2[2 * i], m2[2 * i + 1], 1.};
        double Ex1[3], Etx2[3];
        for (int r = 0; r < 3; ++r) {
            Ex1[r] = E[r * 3 + 0] * x1[0] + E[r * 3 + 1] * x1[1] + E[r * 3 + 2] * x1[2];
            Etx2[r] = E[0 * 3 + r] * x2[0] + E[1 * 3 + r] * x2[1] + E[2 * 3 + r] * x2[2];
        }
        const double x2tEx1 = x2[0] * Ex1[0] + x2[1] * Ex1[1] + x2[2] * Ex1[2];
        const double a = Ex1[0] * Ex1[0], b = Ex1[1] * Ex1[1], c = Etx2[0] * Etx2[0], d = Etx2[1] * Etx2[1];
        const float err = (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
        const int f = err <= t;
        if (mask) mask[i] = (uint8_t)f;
        nz += f;
    }
    return nz;
}

/* RANSACUpdateNumIters */
static int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - pow(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)lrint(num / denom);
}

/* normalise (p - c) / f as MatExpr evaluates it: p * (1 / f) + (-c) * (1 / f) */
void or_normalize_points(const double* pts, int n, double fx, double fy, double cx, double cy, double* out) {
    const double ax = 1. / fx, ay = 1. / fy, sx = -cx * ax, sy = -cy * ay;
    for (int i = 0; i < n; ++i) {
        out[2 * i] = pts[2 * i] * ax + sx;
        out[2 * i + 1] = pts[2 * i + 1] * ay + sy;
    }
}

int or_find_essential(const double* pts1, const double* pts2, int n, double focal, double ppx, double ppy, double prob,
                      double threshold, int max_iters, double E[9], uint8_t* mask, int* stats) {
    if (n < 5) return 0;
    double* m1 = (double*)malloc(sizeof(double) * 4 * (size_t)n);
    double* m2 = m1 + 2 * n;
    or_normalize_points(pts1, n, focal, focal, ppx, ppy, m1);
    or_normalize_points(pts2, n, focal, focal, ppx, ppy, m2);
    threshold /= (focal + focal) / 2;
    const float t = (float)(threshold * threshold);
    double models[90], best[9];
    int ok = 0, max_good = 0, niters = max_iters > 1 ? max_iters : 1, iter = 0, n_models_total = 0;
    if (n == 5) {
        const int nm = or_em_kernel(m1, m2, models);
        if (nm > 0) {
            memcpy(E, models, sizeof(double) * 9);
            if (mask) memset(mask, 1, (size_t)n);
            ok = 1;
        }
        if (stats) { stats[0] = 1; stats[1] = nm; stats[2] = n; }
        free(m1);
        return ok;
    }
    uint8_t* cur = (uint8_t*)malloc((size_t)n * 2);
    uint8_t* bestm = cur + n;
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * 5 * (size_t)niters);
    or_em_subsets(n, niters, idx);
    for (iter = 0; iter < niters; iter++) {
        double q1[10], q2[10];
        for (int i = 0; i < 5; ++i) {
            const int k = idx[5 * iter + i];
            q1[2 * i] = m1[2 * k]; q1[2 * i + 1] = m1[2 * k + 1];
            q2[2 * i] = m2[2 * k]; q2[2 * i + 1] = m2[2 * k + 1];
        }
        const int nm = or_em_kernel(q1, q2, models);
        n_models_total += nm;
        for (int i = 0; i < nm; i++) {
            const int good = em_inliers(m1, m2, n, models + 9 * i, t, cur);
            if (good > (max_good > 4 ? max_good : 4)) {
                memcpy(bestm, cur, (size_t)n);
                memcpy(best, models + 9 * i, sizeof best);
                max_good = good;
                niters = update_num_iters(prob, (double)(n - good) / n, 5, niters);
            }
        }
    }
    if (max_good > 0) {
        memcpy(E, best, sizeof best);
        if (mask) memcpy(mask, bestm, (size_t)n);
        ok = 1;
    }
    if (stats) { stats[0] = iter; stats[1] = n_models_total; stats[2] = max_good; }
    free(idx);
    free(cur);
    free(m1);
    return ok;
}

/* ---------------------------------------------------------------------------------------------- */
/* recoverPose                                                                                      */
/* ---------------------------------------------------------------------------------------------- */
static double det3(const double* a) {
    return a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
}
static void mm3x3(const double* A, const double* B, double* C) {
    double R[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += A[i * 3 + k] * B[k * 3 + j];
            R[i * 3 + j] = s;
        }
    memcpy(C, R, sizeof R);
}

void or_decompose_essential(const double E[9], double R1[9], double R2[9], double t[3]) {
    double w[3], U[9], Vt[9];
    or_cv_svd(E, 3, w, U, Vt);
    if (det3(U) < 0)
        for (int i = 0; i < 9; ++i) U[i] *= -1.;
    if (det3(Vt) < 0)
        for (int i = 0; i < 9; ++i) Vt[i] *= -1.;
    static const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1}, Wt[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    double T[9];
    mm3x3(U, W, T);
    mm3x3(T, Vt, R1);
    mm3x3(U, Wt, T);
    mm3x3(T, Vt, R2);
    for (int i = 0; i < 3; ++i) t[i] = U[i * 3 + 2] * 1.0;
}

/* cvTriangulatePoints for one point: A rows x P[2] - P[0], y P[2] - P[1] per view; X = last row of V^T */
static void triangulate_one(const double* P0, const double* P1, const double* a, const double* b, double* X) {
    double A[16];
    const double* P[2] = {P0, P1};
    const double* q[2] = {a, b};
    for (int j = 0; j < 2; ++j)
        for (int k = 0; k < 4; ++k) {
            A[(j * 2 + 0) * 4 + k] = q[j][0] * P[j][2 * 4 + k] - P[j][0 * 4 + k];
            A[(j * 2 + 1) * 4 + k] = q[j][1] * P[j][2 * 4 + k] - P[j][1 * 4 + k];
        }
    double w[4], vt[16];
    or_cv_svd(A, 4, w, NULL, vt);
    for (int k = 0; k < 4; ++k) X[k] = vt[12 + k];
}

int or_recover_pose(const double E[9], const double* pts1, const double* pts2, int n, const double K[9], double R[9],
                    double t[3], int good_out[4]) {
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5], dist = 50.0;
    double* m1 = (double*)malloc(sizeof(double) * 4 * (size_t)(n > 0 ? n : 1));
    double* m2 = m1 + 2 * n;
    or_normalize_points(pts1, n, fx, fy, cx, cy, m1);
    or_normalize_points(pts2, n, fx, fy, cx, cy, m2);
    double R1[9], R2[9], tt[3];
    or_decompose_essential(E, R1, R2, tt);
    double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0}, P[4][12];
    const double* Rs[4] = {R1, R2, R1, R2};
    for (int c = 0; c < 4; ++c)
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) P[c][i * 4 + j] = Rs[c][i * 3 + j] * 1.0;
            P[c][i * 4 + 3] = c < 2 ? tt[i] * 1.0 : -tt[i] * 1.0;
        }
    int good[4] = {0, 0, 0, 0};
    for (int c = 0; c < 4; ++c)
        for (int i = 0; i < n; ++i) {
            double Q[4];
            triangulate_one(P0, P[c], m1 + 2 * i, m2 + 2 * i, Q);
            int ok = Q[2] * Q[3] > 0;
            /* Q.row(r) /= Q.row(3): element-wise division (cv::divide) */
            const double q3 = Q[3];
            const double X[4] = {Q[0] / q3, Q[1] / q3, Q[2] / q3, Q[3] / q3};
            ok = (X[2] < dist) && ok;
            /* Q = P * Q: 3 x 4 times 4 x 1, sequential */
            double z = 0;
            for (int k = 0; k < 4; ++k) z += P[c][2 * 4 + k] * X[k];
            ok = (z > 0) && ok;
            ok = (z < dist) && ok;
            good[c] += ok;
        }
    int pick;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3]) pick = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3]) pick = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3]) pick = 2;
    else pick = 3;
    memcpy(R, Rs[pick], sizeof(double) * 9);
    for (int i = 0; i < 3; ++i) t[i] = pick < 2 ? tt[i] : -tt[i];
    if (good_out) memcpy(good_out, good, sizeof good);
    free(m1);
    return good[pick];
}
