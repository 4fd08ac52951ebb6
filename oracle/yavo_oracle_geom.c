/*
 * yavo_oracle_geom.c -- CPU restatement of YA_VO's geometry rows.
 *
 * TEST INFRASTRUCTURE ONLY (see yavo_oracle.h).  -ffp-contract=off: every expression rounds as written.
 *
 *   F-RANSAC / 8-point F      src/3DHandler.cc:17-195 with cv::SVD = OpenCV JacobiSVDImpl_<double>
 *                             (modules/core/src/lapack.cpp, scalar loops) and
 *                             cv::Mat products as sequential dot products (OpenCV's small-matrix gemm)
 *   triangulation             src/LoopHandler.cc:658-726, 867-885, 908-915 with Eigen::BDCSVD -> JacobiSVD
 *                             (matrices with < 16 columns), two-sided Jacobi, no QR preconditioner (square)
 *   SE3 / SO3                 Sophus 1.x: exp (SO3::expAndTheta, V from Omega), quaternion product with
 *                             renormalisation, _transformVector, toRotationMatrix
 *   world2Camera              src/Frame.cc:16-28
 *   pose-only LM              src/LoopHandler.cc:730-861 + include/Optimizer.hpp:40-135 with g2o
 *                             OptimizationAlgorithmLevenberg / BlockSolver_6_3 / LinearSolverDense (Eigen LDLT),
 *                             RobustKernelHuber(delta 1)
 *   Gauss-Newton              src/test.cc:172-244
 *
 * Sums over edges (chi2, H, b) are done either sequentially in edge order (the reference) or in the fixed
 * tree order of the GPU kernels (sum_mode m >= 1: per-thread strided partial sums over 128 << m threads --
 * 512 for the pose LM (mode 2), 256 for GN (mode 1) -- then a halving tree), so GPU parity can be tested
 * bit-for-bit and the two orders compared within tolerance.
 * sin / cos in SO3::exp use one fixed polynomial kernel (fdlibm's, |x| <= pi/4) on both sides; the
 * reference's std::sin / std::cos may differ by 1 ulp (unpinned).
 */
#include "yavo_oracle.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ========================================================================================== */
/* OpenCV JacobiSVDImpl_<double>                                                                */
/* ========================================================================================== */

static double cv_hypot(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    if (a > b) {
        b /= a;
        return a * sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * sqrt(1 + a * a);
    }
    return 0;
}

/* cv::RNG (multiply-with-carry, CV_RNG_COEFF 4164903690) */
static uint32_t cv_rng_next(uint64_t* state) {
    *state = (uint64_t)(uint32_t)*state * 4164903690ULL + (uint32_t)(*state >> 32);
    return (uint32_t)*state;
}

/* At: n rows of m (row stride astep); W: n; Vt: n x n (row stride vstep) or NULL; n1 rows of At to
 * normalise into left singular vectors. */
void or_cv_jacobi_svd(double* At, int astep, double* Wout, double* Vt, int vstep, int m, int n, int n1) {
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    double W[32];
    int i, j, k, iter, max_iter = m > 30 ? m : 30;
    double c, s, sd;
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sd;
        if (Vt) {
            for (k = 0; k < n; k++) Vt[i * vstep + k] = 0;
            Vt[i * vstep + i] = 1;
        }
    }
    for (iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (i = 0; i < n - 1; i++)
            for (j = i + 1; j < n; j++) {
                double *Ai = At + i * astep, *Aj = At + j * astep;
                double a = W[i], p = 0, b = W[j];
                for (k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = cv_hypot(p, beta);
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                if (Vt) {
                    double *Vi = Vt + i * vstep, *Vj = Vt + j * vstep;
                    for (k = 0; k < n; k++) {
                        double t0 = c * Vi[k] + s * Vj[k];
                        double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
    for (i = 0; i < n - 1; i++) {
        j = i;
        for (k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            if (Vt) {
                for (k = 0; k < m; k++) { t = At[i * astep + k]; At[i * astep + k] = At[j * astep + k]; At[j * astep + k] = t; }
                for (k = 0; k < n; k++) { t = Vt[i * vstep + k]; Vt[i * vstep + k] = Vt[j * vstep + k]; Vt[j * vstep + k] = t; }
            }
        }
    }
    for (i = 0; i < n; i++) Wout[i] = W[i];
    if (!Vt) return;
    uint64_t rng = 0x12345678;
    for (i = 0; i < n1; i++) {
        sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / m;
            for (k = 0; k < m; k++) At[i * astep + k] = (cv_rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (iter = 0; iter < 2; iter++) {
                for (j = 0; j < i; j++) {
                    sd = 0;
                    for (k = 0; k < m; k++) sd += At[i * astep + k] * At[j * astep + k];
                    double asum = 0;
                    for (k = 0; k < m; k++) {
                        double t = At[i * astep + k] - sd * At[j * astep + k];
                        At[i * astep + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (k = 0; k < m; k++) At[i * astep + k] *= asum;
                }
            }
            sd = 0;
            for (k = 0; k < m; k++) {
                double t = At[i * astep + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        s = sd > minval ? 1 / sd : 0.;
        for (k = 0; k < m; k++) At[i * astep + k] *= s;
    }
}

/* cv::SVD(src, FULL_UV) of a square n x n matrix (row-major): w [n], u [n x n], vt [n x n]. */
static void cv_svd_square(const double* src, int n, double* w, double* u, double* vt) {
    double At[81], V[81];
    /* _SVDcompute: temp_a = transpose(src) (m = n rows of A are At's columns) */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) At[i * n + j] = src[j * n + i];
    or_cv_jacobi_svd(At, n, w, V, n, n, n, n);
    if (u)
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) u[i * n + j] = At[j * n + i]; /* u = transpose(temp_u) */
    if (vt) memcpy(vt, V, sizeof(double) * (size_t)(n * n));
}

/* 3x3 product, sequential dot products (OpenCV small-matrix gemm) */
static void mm3(const double* A, const double* B, double* C) {
    double R[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
    memcpy(C, R, sizeof R);
}

/* ========================================================================================== */
/* _3DHandler: getMeanVar / constructNormMatrix / getFundamentalMatrix / getFRANSAC             */
/* ========================================================================================== */

static double mean_of(const double* v, int n) { /* getMeanVar, src/3DHandler.cc:17-25 */
    double mean = 0.0;
    for (int i = 0; i < n; ++i) mean += v[i];
    mean /= n;
    return mean;
}

static void norm_matrix(const double* xs, const double* ys, int n, double xm, double ym, double N[9]) {
    /* constructNormMatrix, src/3DHandler.cc:28-47 */
    double scaleDenom = 0.0;
    for (int i = 0; i < n; i++) {
        double xh = xs[i] - xm, yh = ys[i] - ym;
        scaleDenom += sqrt(xh * xh + yh * yh);
    }
    double scale = sqrt(2.0) / (scaleDenom / n);
    N[0] = scale; N[1] = 0; N[2] = -scale * xm;
    N[3] = 0; N[4] = scale; N[5] = -scale * ym;
    N[6] = 0; N[7] = 0; N[8] = 1;
}

/* getFundamentalMatrix, src/3DHandler.cc:50-142; pts = [n][4] (x1, y1, x2, y2) in (row, col) pixels. */
int or_fundamental_8pt(const double* pts, int n, double F[9]) {
    if (n < 8 || n > 4096) return 0;
    double *x1 = (double*)malloc(sizeof(double) * 4 * (size_t)n), *y1 = x1 + n, *x2 = y1 + n, *y2 = x2 + n;
    for (int i = 0; i < n; ++i) { x1[i] = pts[4 * i]; y1[i] = pts[4 * i + 1]; x2[i] = pts[4 * i + 2]; y2[i] = pts[4 * i + 3]; }
    double N1[9], N2[9];
    norm_matrix(x1, y1, n, mean_of(x1, n), mean_of(y1, n), N1);
    norm_matrix(x2, y2, n, mean_of(x2, n), mean_of(y2, n), N2);
    /* A^T A accumulated as OpenCV's gemm(A^T, A): AtA[i][j] = sum_k A[k][i] A[k][j], k ascending */
    double AtA[81];
    memset(AtA, 0, sizeof AtA);
    double* A = (double*)malloc(sizeof(double) * 9 * (size_t)n);
    for (int i = 0; i < n; i++) {
        /* normImage * (x, y, 1): rows of the 3x3 times the column, sequential */
        double nx1 = N1[0] * x1[i] + N1[1] * y1[i] + N1[2] * 1.0;
        double ny1 = N1[3] * x1[i] + N1[4] * y1[i] + N1[5] * 1.0;
        double nx2 = N2[0] * x2[i] + N2[1] * y2[i] + N2[2] * 1.0;
        double ny2 = N2[3] * x2[i] + N2[4] * y2[i] + N2[5] * 1.0;
        double* r = A + 9 * i;
        r[0] = nx1 * nx2; r[1] = nx1 * ny2; r[2] = nx1;
        r[3] = ny1 * nx2; r[4] = ny1 * ny2; r[5] = ny1;
        r[6] = nx2; r[7] = ny2; r[8] = 1;
    }
    for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) {
            double s = 0;
            for (int k = 0; k < n; ++k) s += A[9 * k + i] * A[9 * k + j];
            AtA[i * 9 + j] = s;
        }
    double w9[9], vt9[81];
    cv_svd_square(AtA, 9, w9, NULL, vt9);
    double F0[9];
    for (int i = 0; i < 9; ++i) F0[i] = vt9[8 * 9 + i]; /* vt.row(8).reshape(1, 3) */
    double w3[3], u3[9], vt3[9];
    cv_svd_square(F0, 3, w3, u3, vt3);
    w3[2] = 0;
    double D[9] = {w3[0], 0, 0, 0, w3[1], 0, 0, 0, w3[2]};
    double T[9];
    mm3(u3, D, T);
    mm3(T, vt3, F0);
    /* normImage2.t() * F * normImage1 */
    double N2t[9] = {N2[0], N2[3], N2[6], N2[1], N2[4], N2[7], N2[2], N2[5], N2[8]};
    mm3(N2t, F0, T);
    mm3(T, N1, F0);
    /* F / F(2,2): MatExpr a * (1/s) */
    double inv = 1. / F0[8];
    for (int i = 0; i < 9; ++i) F[i] = F0[i] * inv + 0.0;
    free(x1);
    free(A);
    return 1;
}

/* |p2^T F p1| as (p2.t() * F) * p1 with cv::Mat products */
static double epipolar_error(const double F[9], double x1, double y1, double x2, double y2) {
    double r0 = x2 * F[0] + y2 * F[3] + 1.0 * F[6];
    double r1 = x2 * F[1] + y2 * F[4] + 1.0 * F[7];
    double r2 = x2 * F[2] + y2 * F[5] + 1.0 * F[8];
    return r0 * x1 + r1 * y1 + r2 * 1.0;
}

/* getFRANSAC, src/3DHandler.cc:145-195, with the std::random_device draws replaced by sample_idx
 * [iters][8].  Returns 0 (false) when n < 8.  F = the best hypothesis (strictly more inliers wins). */
int or_f_ransac(const yv_match* m, int n, const int32_t* sample_idx, int iters, double thr, double F[9],
                int* max_inliers) {
    if (n < 8) return 0;
    int best = INT32_MIN;
    double pts8[32], Fh[9];
    for (int it = 0; it < iters; ++it) {
        for (int j = 0; j < 8; ++j) {
            const yv_match* s = &m[sample_idx[8 * it + j]];
            pts8[4 * j] = s->pt1.x; pts8[4 * j + 1] = s->pt1.y; pts8[4 * j + 2] = s->pt2.x; pts8[4 * j + 3] = s->pt2.y;
        }
        or_fundamental_8pt(pts8, 8, Fh);
        int cnt = 0;
        for (int k = 0; k < n; ++k)
            if (fabs(epipolar_error(Fh, m[k].pt1.x, m[k].pt1.y, m[k].pt2.x, m[k].pt2.y)) < thr) cnt++;
        if (cnt > best) {
            best = cnt;
            memcpy(F, Fh, sizeof Fh);
        }
    }
    *max_inliers = best;
    return 1;
}

/* ========================================================================================== */
/* Eigen JacobiSVD (square, two-sided, no preconditioner)                                      */
/* ========================================================================================== */

typedef struct { double c, s; } jrot;

static int make_jacobi(double x, double y, double z, jrot* r) { /* JacobiRotation::makeJacobi(real) */
    double deno = 2 * fabs(y);
    if (deno < DBL_MIN) {
        r->c = 1; r->s = 0;
        return 0;
    }
    double tau = (x - z) / deno;
    double w = sqrt(tau * tau + 1);
    double t = tau > 0 ? 1 / (tau + w) : 1 / (tau - w);
    double sign_t = t > 0 ? 1 : -1;
    double nn = 1 / sqrt(t * t + 1);
    r->s = -sign_t * (y / fabs(y)) * fabs(t) * nn;
    r->c = nn;
    return 1;
}

/* apply_rotation_in_the_plane(x, y, j): x' = c x + s y, y' = -s x + c y */
static void rot_rows(double* M, int n, int p, int q, jrot j) { /* applyOnTheLeft(p, q, j), col-major M */
    if (j.c == 1 && j.s == 0) return;
    for (int i = 0; i < n; ++i) {
        double xi = M[p + i * n], yi = M[q + i * n];
        M[p + i * n] = j.c * xi + j.s * yi;
        M[q + i * n] = -j.s * xi + j.c * yi;
    }
}

static void rot_cols(double* M, int n, int p, int q, jrot j) { /* applyOnTheRight(p, q, j) = rotation by j^T */
    jrot t = {j.c, -j.s};
    if (t.c == 1 && t.s == 0) return;
    for (int i = 0; i < n; ++i) {
        double xi = M[i + p * n], yi = M[i + q * n];
        M[i + p * n] = t.c * xi + t.s * yi;
        M[i + q * n] = -t.s * xi + t.c * yi;
    }
}

/* real_2x2_jacobi_svd(matrix, p, q, &j_left, &j_right) */
static void real_2x2_jacobi_svd(const double* M, int n, int p, int q, jrot* jl, jrot* jr) {
    double m00 = M[p + p * n], m01 = M[p + q * n], m10 = M[q + p * n], m11 = M[q + q * n];
    jrot rot1;
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
    /* m.applyOnTheLeft(0, 1, rot1) */
    if (!(rot1.c == 1 && rot1.s == 0)) {
        double a0 = m00, b0 = m10, a1 = m01, b1 = m11;
        m00 = rot1.c * a0 + rot1.s * b0;
        m10 = -rot1.s * a0 + rot1.c * b0;
        m01 = rot1.c * a1 + rot1.s * b1;
        m11 = -rot1.s * a1 + rot1.c * b1;
    }
    make_jacobi(m00, m01, m11, jr);
    /* j_left = rot1 * j_right.transpose() */
    jrot jt = {jr->c, -jr->s};
    jl->c = rot1.c * jt.c - rot1.s * jt.s;
    jl->s = rot1.c * jt.s + rot1.s * jt.c;
}

/* JacobiSVD<MatrixXd>(A, ComputeThinU | ComputeThinV) for square n <= 8, A column-major.
 * sv [n] descending, V column-major n x n.  Returns 0 on non-finite input (Eigen 3.4 InvalidInput). */
int or_eigen_jacobi_svd(const double* A, int n, double* sv, double* V) {
    double Wk[64];
    double scale = 0;
    for (int i = 0; i < n * n; ++i) {
        double a = fabs(A[i]);
        if (a != a) return 0;
        if (a > scale) scale = a;
    }
    if (!isfinite(scale)) return 0;
    if (scale == 0) scale = 1;
    for (int i = 0; i < n * n; ++i) Wk[i] = A[i] / scale;
    for (int i = 0; i < n * n; ++i) V[i] = 0;
    for (int i = 0; i < n; ++i) V[i + i * n] = 1;
    const double considerAsZero = DBL_MIN, precision = 2 * DBL_EPSILON;
    double maxDiag = 0;
    for (int i = 0; i < n; ++i) {
        double a = fabs(Wk[i + i * n]);
        if (a > maxDiag) maxDiag = a;
    }
    int finished = 0;
    while (!finished) {
        finished = 1;
        for (int p = 1; p < n; ++p)
            for (int q = 0; q < p; ++q) {
                double threshold = considerAsZero > precision * maxDiag ? considerAsZero : precision * maxDiag;
                if (fabs(Wk[p + q * n]) > threshold || fabs(Wk[q + p * n]) > threshold) {
                    finished = 0;
                    jrot jl, jr;
                    real_2x2_jacobi_svd(Wk, n, p, q, &jl, &jr);
                    rot_rows(Wk, n, p, q, jl);
                    rot_cols(Wk, n, p, q, jr);
                    rot_cols(V, n, p, q, jr);
                    double a = fabs(Wk[p + p * n]), b = fabs(Wk[q + q * n]);
                    double mx = a > b ? a : b;
                    if (mx > maxDiag) maxDiag = mx;
                }
            }
    }
    for (int i = 0; i < n; ++i) sv[i] = fabs(Wk[i + i * n]);
    for (int i = 0; i < n; ++i) sv[i] *= scale;
    for (int i = 0; i < n; ++i) {
        int pos = 0;
        double mx = sv[i];
        for (int k = i + 1; k < n; ++k)
            if (sv[k] > mx) { mx = sv[k]; pos = k - i; } /* maxCoeff: first index of the maximum */
        if (mx == 0) break;
        if (pos) {
            pos += i;
            double t = sv[i]; sv[i] = sv[pos]; sv[pos] = t;
            for (int r = 0; r < n; ++r) { t = V[r + pos * n]; V[r + pos * n] = V[r + i * n]; V[r + i * n] = t; }
        }
    }
    return 1;
}

/* ========================================================================================== */
/* Sophus SE3 (pose = {qx, qy, qz, qw, tx, ty, tz}, SE3d::data() layout)                        */
/* ========================================================================================== */

int or_libm_flavour = 0;
void or_set_libm_flavour(int flavour) { or_libm_flavour = flavour ? 1 : 0; }

/* or_cube (flavour 0) or the C library's pow(t, 3) (flavour 1) over n arguments */
void or_cube_batch(const double* t, int n, int flavour, double* out) {
    for (int i = 0; i < n; ++i) out[i] = flavour ? pow(t[i], 3) : or_cube(t[i]);
}

/* fdlibm __kernel_sin / __kernel_cos (|x| <= pi/4); larger |x|, or the libm flavour, call the C library. */
static double k_sin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    if (or_libm_flavour || !(fabs(x) <= 0.78539816339744827900)) return sin(x);
    double z = x * x, v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}

static double k_cos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    if (or_libm_flavour || !(fabs(x) <= 0.78539816339744827900)) return cos(x);
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * 0.0));
}

double or_ksin(double x) { return k_sin(x); }
double or_kcos(double x) { return k_cos(x); }

static void quat_mul(const double* a, const double* b, double* r) { /* Eigen quat_product (x, y, z, w) */
    double ax = a[0], ay = a[1], az = a[2], aw = a[3], bx = b[0], by = b[1], bz = b[2], bw = b[3];
    r[3] = aw * bw - ax * bx - ay * by - az * bz;
    r[0] = aw * bx + ax * bw + ay * bz - az * by;
    r[1] = aw * by + ay * bw + az * bx - ax * bz;
    r[2] = aw * bz + az * bw + ax * by - ay * bx;
}

/* Eigen QuaternionBase::_transformVector */
static void quat_rotate(const double* q, const double* v, double* out) {
    double uv0 = q[1] * v[2] - q[2] * v[1];
    double uv1 = q[2] * v[0] - q[0] * v[2];
    double uv2 = q[0] * v[1] - q[1] * v[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    double c0 = q[1] * uv2 - q[2] * uv1;
    double c1 = q[2] * uv0 - q[0] * uv2;
    double c2 = q[0] * uv1 - q[1] * uv0;
    out[0] = v[0] + q[3] * uv0 + c0;
    out[1] = v[1] + q[3] * uv1 + c1;
    out[2] = v[2] + q[3] * uv2 + c2;
}

/* Eigen QuaternionBase::toRotationMatrix, row-major R */
void or_quat_to_R(const double* q, double* R) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

/* SE3 * point = so3 * p + t */
void or_se3_act(const double* T, const double* p, double* out) {
    double r[3];
    quat_rotate(T, p, r);
    out[0] = r[0] + T[4];
    out[1] = r[1] + T[5];
    out[2] = r[2] + T[6];
}

/* SE3 * SE3: t = tA + soA * tB; q = qA * qB renormalised by 2 / (1 + |q|^2) when |q|^2 != 1 */
void or_se3_mul(const double* A, const double* B, double* out) {
    double r[3], q[4];
    quat_rotate(A, B + 4, r);
    double t0 = A[4] + r[0], t1 = A[5] + r[1], t2 = A[6] + r[2];
    quat_mul(A, B, q);
    double sn = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    if (sn != 1.0) {
        double sc = 2.0 / (1.0 + sn);
        for (int i = 0; i < 4; ++i) q[i] *= sc;
    }
    out[0] = q[0]; out[1] = q[1]; out[2] = q[2]; out[3] = q[3];
    out[4] = t0; out[5] = t1; out[6] = t2;
}

/* Sophus SE3::inverse (LoopHandler: lastFrame->pose.inverse(), SE3(R, t).inverse(), src/LoopHandler.cc:160,285,
 * 644-648): invR = SO3(q.conjugate()) -- the SO3 quaternion constructor normalises: q / |q| with Eigen's SSE2
 * packet redux of the Vector4d squared norm, (x^2 + z^2) + (y^2 + w^2) -- and t' = invR * (t * -1). */
void or_se3_inverse(const double* T, double* out) {
    double q[4] = {-T[0], -T[1], -T[2], T[3]};
    const double len = sqrt((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
    for (int i = 0; i < 4; ++i) q[i] = q[i] / len;
    const double mt[3] = {T[4] * -1.0, T[5] * -1.0, T[6] * -1.0};
    double r[3];
    quat_rotate(q, mt, r);
    out[0] = q[0]; out[1] = q[1]; out[2] = q[2]; out[3] = q[3];
    out[4] = r[0]; out[5] = r[1]; out[6] = r[2];
}

/* Sophus SE3d(Matrix3d R, Vector3d t) (src/LoopHandler.cc:283, 643): SO3(R) = Eigen's Quaternion from a rotation
 * matrix (quaternion_assign_impl<3,3>: the trace branch, else the largest-diagonal branch; no normalisation).
 * R row-major. */
void or_se3_from_Rt(const double* R, const double* t, double* out) {
#define M(i, j) R[3 * (i) + (j)]
    double q[4];  /* x, y, z, w */
    double tr = (M(0, 0) + M(1, 1)) + M(2, 2);
    if (tr > 0.0) {
        tr = sqrt(tr + 1.0);
        q[3] = 0.5 * tr;
        tr = 0.5 / tr;
        q[0] = (M(2, 1) - M(1, 2)) * tr;
        q[1] = (M(0, 2) - M(2, 0)) * tr;
        q[2] = (M(1, 0) - M(0, 1)) * tr;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        tr = sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        q[i] = 0.5 * tr;
        tr = 0.5 / tr;
        q[3] = (M(k, j) - M(j, k)) * tr;
        q[j] = (M(j, i) + M(i, j)) * tr;
        q[k] = (M(k, i) + M(i, k)) * tr;
    }
#undef M
    for (int i = 0; i < 4; ++i) out[i] = q[i];
    out[4] = t[0]; out[5] = t[1]; out[6] = t[2];
}

/* SE3::exp(a), a = (upsilon, omega) */
void or_se3_exp(const double* a, double* out) {
    const double* om = a + 3;
    const double eps = 1e-10; /* Sophus::Constants<double>::epsilon() */
    double theta_sq = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
    double theta, imag, real;
    if (theta_sq < eps * eps) {
        theta = 0;
        double theta_po4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_po4;
        real = 1 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_po4;
    } else {
        theta = sqrt(theta_sq);
        double half = 0.5 * theta;
        imag = k_sin(half) / theta;
        real = k_cos(half);
    }
    double q[4] = {imag * om[0], imag * om[1], imag * om[2], real};
    /* Omega = hat(omega), Omega^2 */
    double O[9] = {0, -om[2], om[1], om[2], 0, -om[0], -om[1], om[0], 0};
    double O2[9];
    mm3(O, O, O2);
    double V[9];
    if (theta < eps) {
        or_quat_to_R(q, V); /* V = so3.matrix() */
    } else {
        double theta_sq2 = theta * theta;
        double a1 = (1 - k_cos(theta)) / theta_sq2;
        double a2 = (theta - k_sin(theta)) / (theta_sq2 * theta);
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + a1 * O[i] + a2 * O2[i];
    }
    out[0] = q[0]; out[1] = q[1]; out[2] = q[2]; out[3] = q[3];
    for (int i = 0; i < 3; ++i) out[4 + i] = V[3 * i] * a[0] + V[3 * i + 1] * a[1] + V[3 * i + 2] * a[2];
}

/* Frame::world2Camera, src/Frame.cc:16-28: (K * [R|t]) * [X; 1] */
void or_world2camera(const double* X, int n, const double* T, const double* K, double* out) {
    double R[9], M[12], KM[12];
    or_quat_to_R(T, R);
    for (int i = 0; i < 3; ++i) {
        M[4 * i] = R[3 * i]; M[4 * i + 1] = R[3 * i + 1]; M[4 * i + 2] = R[3 * i + 2]; M[4 * i + 3] = T[4 + i];
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) KM[4 * i + j] = K[3 * i] * M[j] + K[3 * i + 1] * M[4 + j] + K[3 * i + 2] * M[8 + j];
    for (int k = 0; k < n; ++k)
        for (int i = 0; i < 3; ++i)
            out[3 * k + i] = KM[4 * i] * X[3 * k] + KM[4 * i + 1] * X[3 * k + 1] + KM[4 * i + 2] * X[3 * k + 2] + KM[4 * i + 3] * 1.0;
}

/* ========================================================================================== */
/* triangulation / triangulate2View                                                            */
/* ========================================================================================== */

/* LoopHandler::triangulation, src/LoopHandler.cc:867-885, two poses; pts = camera-normalised (x, y). */
int or_triangulate_one(const double* Ta, const double* Tb, const double* pa, const double* pb, double* Xw) {
    double A[16]; /* column-major 4x4 */
    const double* Ts[2] = {Ta, Tb};
    const double* ps[2] = {pa, pb};
    for (int i = 0; i < 2; ++i) {
        double R[9], m[12];
        or_quat_to_R(Ts[i], R);
        for (int r = 0; r < 3; ++r) {
            m[4 * r] = R[3 * r]; m[4 * r + 1] = R[3 * r + 1]; m[4 * r + 2] = R[3 * r + 2]; m[4 * r + 3] = Ts[i][4 + r];
        }
        for (int j = 0; j < 4; ++j) {
            A[(2 * i) + 4 * j] = ps[i][0] * m[8 + j] - m[j];
            A[(2 * i + 1) + 4 * j] = ps[i][1] * m[8 + j] - m[4 + j];
        }
    }
    double sv[4], V[16];
    if (!or_eigen_jacobi_svd(A, 4, sv, V)) {
        Xw[0] = Xw[1] = Xw[2] = NAN;
        return 0;
    }
    Xw[0] = V[0 + 3 * 4] / V[3 + 3 * 4];
    Xw[1] = V[1 + 3 * 4] / V[3 + 3 * 4];
    Xw[2] = V[2 + 3 * 4] / V[3 + 3 * 4];
    return sv[3] / sv[2] < 1e-2 ? 1 : 0;
}

/* triangulate2View (src/LoopHandler.cc:665-676): pixel2camera of (row, col) then triangulation; ok[i] =
 * triangulation succeeded and pworld[2] > 0. */
int or_triangulate_matches(const double* Ta, const double* Tb, const double* K, const yv_match* m, int n,
                           double* Xw, uint8_t* ok) {
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        /* pixel2camera(cv::Point p, K): ((p.x - cx) * 1 / fx, (p.y - cy) * 1 / fy, 1) */
        double pa[2] = {((double)m[i].pt1.x - K[2]) * 1.0 / K[0], ((double)m[i].pt1.y - K[5]) * 1.0 / K[4]};
        double pb[2] = {((double)m[i].pt2.x - K[2]) * 1.0 / K[0], ((double)m[i].pt2.y - K[5]) * 1.0 / K[4]};
        int s = or_triangulate_one(Ta, Tb, pa, pb, Xw + 3 * i);
        ok[i] = (uint8_t)(s && Xw[3 * i + 2] > 0);
        cnt += ok[i];
    }
    return cnt;
}

/* ========================================================================================== */
/* Eigen LDLT (robust Cholesky with diagonal pivoting), 6 x 6                                  */
/* ========================================================================================== */

/* variant 0 (dynamic MatrixXd, g2o LinearSolverDense): A21 -= A20*temp as a column-wise GEMV
 * (sequential subtraction per term); variant 1 (fixed Matrix6d, test.cc): A21 -= dot(A20 row, temp). */
static int ldlt6_solve(const double* Hin, const double* b, double* x, int variant) {
    double mat[36];
    int tr[6];
    memcpy(mat, Hin, sizeof mat); /* row-major; only the lower triangle (i >= j) is read */
    const int n = 6;
    int sign = 0; /* 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite */
    int found_zero_pivot = 0, ret = 1;
    double temp[6];
#define L(i, j) mat[(i) * 6 + (j)]
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = fabs(L(k, k));
        for (int i = k + 1; i < n; ++i)
            if (fabs(L(i, i)) > bv) { bv = fabs(L(i, i)); big = i; }
        tr[k] = big;
        if (k != big) {
            int s = n - big - 1;
            for (int j = 0; j < k; ++j) { double t = L(k, j); L(k, j) = L(big, j); L(big, j) = t; }
            for (int j = 0; j < s; ++j) { double t = L(big + 1 + j, k); L(big + 1 + j, k) = L(big + 1 + j, big); L(big + 1 + j, big) = t; }
            { double t = L(k, k); L(k, k) = L(big, big); L(big, big) = t; }
            for (int i = k + 1; i < big; ++i) { double t = L(i, k); L(i, k) = L(big, i); L(big, i) = t; }
        }
        int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = L(j, j) * L(k, j);
            double dot = L(k, 0) * temp[0];
            for (int j = 1; j < k; ++j) dot = dot + L(k, j) * temp[j];
            L(k, k) -= dot;
            for (int i = k + 1; i < n; ++i) {
                if (variant == 0) {
                    double acc = L(i, k);
                    for (int j = 0; j < k; ++j) acc = acc - L(i, j) * temp[j];
                    L(i, k) = acc;
                } else {
                    double d = L(i, 0) * temp[0];
                    for (int j = 1; j < k; ++j) d = d + L(i, j) * temp[j];
                    L(i, k) = L(i, k) - d;
                }
            }
        }
        double akk = L(k, k);
        int valid = fabs(akk) > 0;
        if (k == 0 && !valid) {
            sign = 0;
            for (int j = 0; j < n; ++j) tr[j] = j;
            ret = 0;
            break;
        }
        if (rs > 0 && valid) {
            for (int i = k + 1; i < n; ++i) L(i, k) /= akk;
        } else if (rs > 0) {
            for (int i = k + 1; i < n; ++i) ret = ret && (L(i, k) == 0);
        }
        if (found_zero_pivot && valid) ret = 0;
        else if (!valid) found_zero_pivot = 1;
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    (void)ret;
    int positive = (sign == 1 || sign == 0);
    /* solve: x = P b ; L y = x ; y /= D ; L^T z = y ; x = P^T z */
    double v[6];
    memcpy(v, b, sizeof v);
    for (int k = 0; k < n; ++k) { double t = v[k]; v[k] = v[tr[k]]; v[tr[k]] = t; }
    for (int j = 0; j < n; ++j)
        for (int i = j + 1; i < n; ++i) v[i] = v[i] - L(i, j) * v[j];
    for (int i = 0; i < n; ++i) {
        if (fabs(L(i, i)) > DBL_MIN) v[i] /= L(i, i);
        else v[i] = 0;
    }
    for (int j = n - 1; j >= 0; --j)
        for (int i = 0; i < j; ++i) v[i] = v[i] - L(j, i) * v[j];
    for (int k = n - 1; k >= 0; --k) { double t = v[k]; v[k] = v[tr[k]]; v[tr[k]] = t; }
#undef L
    memcpy(x, v, sizeof v);
    return positive;
}

/* ========================================================================================== */
/* pose-only edge (include/Optimizer.hpp:64-126)                                               */
/* ========================================================================================== */

/* computeError: e = meas - (K * (T * X)).head(2) / z */
static void edge_error(const double* T, const double* K, const double* X, const double* meas, double* e) {
    double pc[3];
    or_se3_act(T, X, pc);
    double u0 = K[0] * pc[0] + K[1] * pc[1] + K[2] * pc[2];
    double u1 = K[3] * pc[0] + K[4] * pc[1] + K[5] * pc[2];
    double u2 = K[6] * pc[0] + K[7] * pc[1] + K[8] * pc[2];
    e[0] = meas[0] - u0 / u2;
    e[1] = meas[1] - u1 / u2;
}

/* linearizeOplus: 2 x 6 Jacobian w.r.t. (rho, phi), no cx / cy */
static void edge_jacobian(const double* T, const double* K, const double* X, double* J) {
    double pc[3];
    or_se3_act(T, X, pc);
    double fx = K[0], fy = K[4];
    double x = pc[0], y = pc[1], z = pc[2];
    double zinv = 1.0 / (z + 1e-18);
    double zinv2 = zinv * zinv;
    J[0] = -fx * zinv; J[1] = 0; J[2] = fx * x * zinv2; J[3] = fx * x * y * zinv2;
    J[4] = -fx - fx * x * x * zinv2; J[5] = fx * y * zinv;
    J[6] = 0; J[7] = -fy * zinv; J[8] = fy * y * zinv2; J[9] = fy + fy * y * y * zinv2;
    J[10] = -fy * x * y * zinv2; J[11] = -fy * x * zinv;
}

/* ---- summation orders ----
 * mode 0: sequential in edge order (the reference).  mode m >= 1: the GPU kernels' order over NT = 128 << m
 * threads (1: 256 threads, the GN kernel; 2: 512, the pose-LM kernel): edge k adds into thread k % NT's
 * partial.  Mode 1 then sums the pairwise tree p[t] += p[t + off] for off = NT/2 .. 1.  Mode 2 (512 threads)
 * and mode 3 (256 threads, the pose-LM kernel) halve once (p[t] += p[t + NT/2]), sum each of 16 runs of
 * NT/32 partials left to right (q[s] = p[Rs] + p[Rs+1] + ... , R = NT/32) and finish with the tree
 * q[s] += q[s + off], off = 8, 4, 2, 1.  Modes 4, 5, 6, 7 (the pose-LM kernel at 64, 128, 256, 512 threads): the halving
 * tree p[l] += p[l + off], off = 32 .. 1, inside each 64-thread wave, then the wave totals left to right. */
#define OR_NT_MAX 1024
typedef struct { int mode, nt; double part[OR_NT_MAX]; } or_sum;

static void sum_reset(or_sum* s, int mode) {
    s->mode = mode;
    s->nt = mode >= 4 ? 64 << (mode - 4) : mode == 3 ? 256 : mode >= 1 ? 128 << mode : 1;
    memset(s->part, 0, sizeof(double) * (size_t)s->nt);
}
/* term of edge index k (in the active-edge order) */
static void sum_add(or_sum* s, int k, double v) {
    if (s->mode == 0) s->part[0] = s->part[0] + v;
    else s->part[k % s->nt] = s->part[k % s->nt] + v;
}
static double sum_total(or_sum* s) {
    if (s->mode == 0) return s->part[0];
    double p[OR_NT_MAX];
    memcpy(p, s->part, sizeof(double) * (size_t)s->nt);
    if (s->mode >= 4) {
        double tot = 0.0;
        for (int w = 0; w < s->nt / 64; ++w) {
            double* q = p + 64 * w;
            for (int off = 32; off > 0; off >>= 1)
                for (int t = 0; t < off; ++t) q[t] = q[t] + q[t + off];
            tot = w == 0 ? q[0] : tot + q[0];
        }
        return tot;
    }
    if (s->mode == 2 || s->mode == 3) {
        /* segmented: NT threads, halve once, 16 runs of NT/32 partials summed left to right, tree over runs */
        const int half = s->nt / 2, run = half / 16;
        double q[16];
        for (int t = 0; t < half; ++t) p[t] = p[t] + p[t + half];
        for (int g = 0; g < 16; ++g) {
            q[g] = p[run * g];
            for (int i = 1; i < run; ++i) q[g] = q[g] + p[run * g + i];
        }
        for (int off = 8; off > 0; off >>= 1)
            for (int g = 0; g < off; ++g) q[g] = q[g] + q[g + off];
        return q[0];
    }
    for (int off = s->nt / 2; off > 0; off >>= 1)
        for (int t = 0; t < off; ++t) p[t] = p[t] + p[t + off];
    return p[0];
}

/* ========================================================================================== */
/* g2o Levenberg-Marquardt on one VertexPose + unary EdgeProjectionPoseOnly edges               */
/* ========================================================================================== */

typedef struct {
    int n_active;
    const int* active;     /* active edge indices, insertion order */
    const double *X, *uv, *K;
    const uint8_t* robust; /* per edge: Huber kernel attached */
    double* err;           /* per edge error (2), as last computed */
    int sum_mode;
} lm_problem;

static void compute_active_errors(lm_problem* P, const double* T) {
    for (int a = 0; a < P->n_active; ++a) {
        int i = P->active[a];
        edge_error(T, P->K, P->X + 3 * i, P->uv + 2 * i, P->err + 2 * i);
    }
}

static double huber_rho(double e2, double* rho1) { /* RobustKernelHuber::robustify, delta = 1 */
    const double delta = 1.0, dsqr = delta * delta;
    if (e2 <= dsqr) {
        *rho1 = 1.;
        return e2;
    }
    double sqrte = sqrt(e2);
    *rho1 = delta / sqrte;
    return 2 * sqrte * delta - dsqr;
}

static double edge_chi2(const double* e) { return e[0] * e[0] + e[1] * e[1]; }

static double active_robust_chi2(lm_problem* P) {
    or_sum s;
    sum_reset(&s, P->sum_mode);
    for (int a = 0; a < P->n_active; ++a) {
        int i = P->active[a];
        double c2 = edge_chi2(P->err + 2 * i);
        if (P->robust[i]) {
            double r1;
            sum_add(&s, a, huber_rho(c2, &r1));
        } else {
            sum_add(&s, a, c2);
        }
    }
    return sum_total(&s);
}

/* BlockSolver::buildSystem for the single pose block: H (full 6x6, row-major) and b */
static void build_system(lm_problem* P, const double* T, double* H, double* b) {
    or_sum* sH = (or_sum*)malloc(sizeof(or_sum) * 42);
    or_sum* sb = sH + 36;
    for (int i = 0; i < 36; ++i) sum_reset(&sH[i], P->sum_mode);
    for (int i = 0; i < 6; ++i) sum_reset(&sb[i], P->sum_mode);
    for (int a = 0; a < P->n_active; ++a) {
        int i = P->active[a];
        double J[12];
        edge_jacobian(T, P->K, P->X + 3 * i, J);
        const double* e = P->err + 2 * i;
        double w = 1.0;
        if (P->robust[i]) huber_rho(edge_chi2(e), &w);
        /* (J^T W) with W = w * I (robust) or I: T(r, k) = J(0, r) W(0, k) + J(1, r) W(1, k) */
        for (int r = 0; r < 6; ++r) {
            double t0 = J[r] * w + J[6 + r] * 0.0;
            double t1 = J[r] * 0.0 + J[6 + r] * w;
            for (int c = 0; c < 6; ++c) sum_add(&sH[r * 6 + c], a, t0 * J[c] + t1 * J[6 + c]);
            /* b -= (rho1 J^T) Omega e */
            double s0 = (w * J[r]) * 1.0 + (w * J[6 + r]) * 0.0;
            double s1 = (w * J[r]) * 0.0 + (w * J[6 + r]) * 1.0;
            sum_add(&sb[r], a, -(s0 * e[0] + s1 * e[1]));
        }
    }
    for (int i = 0; i < 36; ++i) H[i] = sum_total(&sH[i]);
    for (int i = 0; i < 6; ++i) b[i] = sum_total(&sb[i]);
    free(sH);
}

/* pass statistics (diagnostics for the kernel design: builds / trials / accepted trials) */
static long g_lm_stats[3];
void or_lm_stats(long* out, int reset) {
    for (int i = 0; i < 3; ++i) {
        out[i] = g_lm_stats[i];
        if (reset) g_lm_stats[i] = 0;
    }
}

/* SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg::solve per iteration.
 * Returns the number of iterations run (-1 when there is no active edge). */
static int lm_optimize(lm_problem* P, double* T, int iterations) {
    if (P->n_active == 0) return -1;
    double lambda = 0, ni = 2;
    const double tau = 1e-5, goodLower = 1.0 / 3.0, goodUpper = 2.0 / 3.0;
    int it;
    for (it = 0; it < iterations; ++it) {
        compute_active_errors(P, T);
        double currentChi = active_robust_chi2(P);
        double H[36], b[6];
        build_system(P, T, H, b);
        g_lm_stats[0]++;
        if (it == 0) {
            double maxDiag = 0;
            for (int j = 0; j < 6; ++j) maxDiag = fabs(H[j * 7]) > maxDiag ? fabs(H[j * 7]) : maxDiag;
            lambda = tau * maxDiag;
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        double tempChi;
        do {
            double Tbak[7];
            memcpy(Tbak, T, sizeof Tbak);
            double Hl[36], x[6];
            memcpy(Hl, H, sizeof Hl);
            for (int j = 0; j < 6; ++j) Hl[j * 7] += lambda;
            int ok2 = ldlt6_solve(Hl, b, x, 0);
            double Tn[7];
            or_se3_exp(x, Tn); /* VertexPose::oplusImpl: exp(update) * estimate */
            double Tnew[7];
            or_se3_mul(Tn, T, Tnew);
            memcpy(T, Tnew, sizeof Tnew);
            compute_active_errors(P, T);
            tempChi = active_robust_chi2(P);
            if (!ok2) tempChi = DBL_MAX;
            rho = currentChi - tempChi;
            double scale = 1;
            if (ok2) {
                double sc = 0;
                for (int j = 0; j < 6; ++j) sc += x[j] * (lambda * x[j] + b[j]);
                scale = sc + 1e-3;
            }
            rho /= scale;
            g_lm_stats[1]++;
            if (rho > 0 && isfinite(tempChi) && ok2) {
                g_lm_stats[2]++;
                double t = 2 * rho - 1;
                double alpha = 1. - or_lm_cube(t);
                alpha = alpha < goodUpper ? alpha : goodUpper;
                double sf = goodLower > alpha ? goodLower : alpha;
                lambda *= sf;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                memcpy(T, Tbak, sizeof Tbak); /* pop */
                if (!isfinite(lambda)) break;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0 || !isfinite(lambda)) {
            it++;
            break; /* Terminate */
        }
    }
    return it;
}

/* LoopHandler::optimizePoseOnly, src/LoopHandler.cc:730-861.  X [n][3] world points, uv [n][2] measurements
 * (kp.x = row, kp.y = col), K row-major 3x3, pose in/out (SE3d::data()).  outlier[n] = final flags.
 * Returns the inlier count (n - outliers). */
int or_pose_lm(const double* X, const double* uv, int n, const double* K, double* pose, uint8_t* outlier,
               int sum_mode) {
    uint8_t* level = (uint8_t*)calloc((size_t)n + 1, 1);
    uint8_t* robust = (uint8_t*)malloc((size_t)n + 1);
    int* active = (int*)malloc(sizeof(int) * ((size_t)n + 1));
    double* err = (double*)calloc(2 * (size_t)n + 2, sizeof(double));
    memset(robust, 1, (size_t)n + 1);
    memset(outlier, 0, (size_t)n);
    const double chi2th = 5.991;
    double prior[7], T[7];
    memcpy(prior, pose, sizeof prior);
    int outlierCount = 0;
    for (int round = 0; round < 4; ++round) {
        memcpy(T, prior, sizeof T); /* vertexPose->setEstimate(currentFrame->pose) */
        int na = 0;
        for (int i = 0; i < n; ++i)
            if (level[i] == 0) active[na++] = i; /* initializeOptimization(): level-0 edges */
        lm_problem P = {na, active, X, uv, K, robust, err, sum_mode};
        lm_optimize(&P, T, 10);
        outlierCount = 0;
        for (int i = 0; i < n; ++i) {
            if (outlier[i]) edge_error(T, K, X + 3 * i, uv + 2 * i, err + 2 * i); /* e->computeError() */
            if (edge_chi2(err + 2 * i) > chi2th) {
                outlier[i] = 1;
                level[i] = 1;
                outlierCount++;
            } else {
                outlier[i] = 0;
                level[i] = 0;
            }
            if (round == 2) robust[i] = 0; /* e->setRobustKernel(nullptr) */
        }
    }
    memcpy(pose, T, sizeof T);
    free(level); free(robust); free(active); free(err);
    return n - outlierCount;
}

/* bundleAdjustmentGaussNewton, src/test.cc:172-244 (cx, cy in the projection; 10 iterations; stop on cost
 * increase or |dx| < 1e-6; NaN guard). Returns iterations accepted. */
int or_pose_gn(const double* X, const double* uv, int n, const double* K, double* pose, int sum_mode) {
    const int iterations = 10;
    double cost = 0, lastCost = 0;
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    int acc = 0;
    or_sum* sums = (or_sum*)malloc(sizeof(or_sum) * 43);
    for (int iter = 0; iter < iterations; iter++) {
        or_sum *sH = sums, *sb = sums + 36, *scp = sums + 42;
#define sc (*scp)
        for (int i = 0; i < 36; ++i) sum_reset(&sH[i], sum_mode);
        for (int i = 0; i < 6; ++i) sum_reset(&sb[i], sum_mode);
        sum_reset(&sc, sum_mode);
        for (int i = 0; i < n; i++) {
            double pc[3];
            or_se3_act(pose, X + 3 * i, pc);
            double inv_z = 1.0 / pc[2];
            double inv_z2 = inv_z * inv_z;
            double proj0 = fx * pc[0] / pc[2] + cx, proj1 = fy * pc[1] / pc[2] + cy;
            double e0 = uv[2 * i] - proj0, e1 = uv[2 * i + 1] - proj1;
            sum_add(&sc, i, e0 * e0 + e1 * e1);
            double J[12] = {-fx * inv_z, 0, fx * pc[0] * inv_z2, fx * pc[0] * pc[1] * inv_z2,
                            -fx - fx * pc[0] * pc[0] * inv_z2, fx * pc[1] * inv_z,
                            0, -fy * inv_z, fy * pc[1] * inv_z2, fy + fy * pc[1] * pc[1] * inv_z2,
                            -fy * pc[0] * pc[1] * inv_z2, -fy * pc[0] * inv_z};
            for (int r = 0; r < 6; ++r) {
                for (int c = 0; c < 6; ++c) sum_add(&sH[r * 6 + c], i, J[r] * J[c] + J[6 + r] * J[6 + c]);
                /* b += -J^T e */
                sum_add(&sb[r], i, (-J[r]) * e0 + (-J[6 + r]) * e1);
            }
        }
        cost = sum_total(&sc);
        double H[36], b[6], dx[6];
        for (int i = 0; i < 36; ++i) H[i] = sum_total(&sH[i]);
        for (int i = 0; i < 6; ++i) b[i] = sum_total(&sb[i]);
        ldlt6_solve(H, b, dx, 1);
        if (isnan(dx[0])) break;
        if (iter > 0 && cost >= lastCost) break;
        double Tn[7], Tnew[7];
        or_se3_exp(dx, Tn);
        or_se3_mul(Tn, pose, Tnew);
        memcpy(pose, Tnew, sizeof Tnew);
        lastCost = cost;
        acc++;
        /* dx.norm(): Eigen's unrolled packet redux over Vector6d: (d0^2 + (d2^2 + d4^2)) + (d1^2 + (d3^2 + d5^2)) */
        double q0 = dx[0] * dx[0] + (dx[2] * dx[2] + dx[4] * dx[4]);
        double q1 = dx[1] * dx[1] + (dx[3] * dx[3] + dx[5] * dx[5]);
        double nrm = sqrt(q0 + q1);
        if (nrm < 1e-6) break;
#undef sc
    }
    free(sums);
    return acc;
}

/* exported helpers for tests */
int or_ldlt6_solve(const double* H, const double* b, double* x, int variant) { return ldlt6_solve(H, b, x, variant); }
void or_cv_svd(const double* src, int n, double* w, double* u, double* vt) { cv_svd_square(src, n, w, u, vt); }
