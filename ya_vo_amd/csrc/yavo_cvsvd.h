// yavo_cvsvd.h -- device restatements of OpenCV's small dense linear algebra shared by the geometry kernels:
// JacobiSVDImpl_<double> (lapack.cpp; with the FULL_UV completion by cv::RNG(0x12345678)), its hypot, and cv::RNG's
// multiply-with-carry step.  Per lane, private arrays; every expression in OpenCV's order (files are built with
// -ffp-contract=off), matching oracle/yavo_oracle_geom.c or_cv_jacobi_svd.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

namespace yavo {
namespace cv {

__device__ __forceinline__ double cv_hypot(double a, double b) {
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

__device__ __forceinline__ uint32_t cv_rng_next(uint64_t* state) {
    *state = (uint64_t)(uint32_t)*state * 4164903690ULL + (uint32_t)(*state >> 32);
    return (uint32_t)*state;
}

// Lane-private arrays in LDS laid out [element][lane] (element e of lane l at p[e * L]): a wave's access to one element
// is one conflict-free ds_*_b64, and dynamic indices cost no scratch.  Indexing and pointer arithmetic as on a double*.
template <int L>
struct LdsArr {
    double* p;
    __device__ __forceinline__ double& operator[](int i) const { return p[i * L]; }
    __device__ __forceinline__ LdsArr operator+(int o) const { return LdsArr{p + o * L}; }
};

// At: N1 rows of M (the first N are the input vectors), Vt: N x N; n1 = N1 rows normalised / completed.  PA / PV:
// double* (private arrays) or LdsArr<L>.
template <int M, int N, int N1, class PA = double*, class PV = double*>
__device__ void cv_jacobi_svd_mn(PA At, double* Wout, PV Vt) {
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    double W[N];
    const int m = M, n = N, max_iter = m > 30 ? m : 30;
    double c, s, sd;
    for (int i = 0; i < n; i++) {
        sd = 0;
        for (int k = 0; k < m; k++) {
            double t = At[i * M + k];
            sd += t * t;
        }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * N + k] = 0;
        Vt[i * N + i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                auto Ai = At + i * M;
                auto Aj = At + j * M;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
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
                for (int k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                auto Vi = Vt + i * N;
                auto Vj = Vt + j * N;
                for (int k = 0; k < n; k++) {
                    double t0 = c * Vi[k] + s * Vj[k];
                    double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        sd = 0;
        for (int k = 0; k < m; k++) {
            double t = At[i * M + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            for (int k = 0; k < m; k++) { t = At[i * M + k]; At[i * M + k] = At[j * M + k]; At[j * M + k] = t; }
            for (int k = 0; k < n; k++) { t = Vt[i * N + k]; Vt[i * N + k] = Vt[j * N + k]; Vt[j * N + k] = t; }
        }
    }
    for (int i = 0; i < n; i++) Wout[i] = W[i];
    uint64_t rng = 0x12345678;
    for (int i = 0; i < N1; i++) {
        sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / m;
            for (int k = 0; k < m; k++) At[i * M + k] = (cv_rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (int it2 = 0; it2 < 2; it2++) {
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; k++) sd += At[i * M + k] * At[j * M + k];
                    double asum = 0;
                    for (int k = 0; k < m; k++) {
                        double t = At[i * M + k] - sd * At[j * M + k];
                        At[i * M + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * M + k] *= asum;
                }
            }
            sd = 0;
            for (int k = 0; k < m; k++) {
                double t = At[i * M + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; k++) At[i * M + k] *= s;
    }
}

// square: m = n = N, astep = vstep = N, n1 = N
template <int N>
__device__ void cv_jacobi_svd(double* At, double* Wout, double* Vt) {
    cv_jacobi_svd_mn<N, N, N>(At, Wout, Vt);
}

}  // namespace cv
}  // namespace yavo
