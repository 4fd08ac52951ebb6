/*
 * yavo_oracle.c -- CPU restatement of YA_VO's detect / describe / match path.
 *
 * TEST INFRASTRUCTURE ONLY (see yavo_oracle.h).  Compiled with -O2 -ffp-contract=off -fno-fast-math so
 * that every float/double expression rounds exactly as written, like the reference's x86-64 build.
 */
#include "yavo_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ========================================================================================== */
/* FAST ring: FastDetector::getBresenhamCirclePoints, src/FastDetector.cc:50-112              */
/* ========================================================================================== */

/* The reference keeps two std::set<std::pair<int,int>> with comparators that order by .second only
 * (src/FastDetector.cc:19-45; their `true;` / `false;` statements are no-ops, so pairs with equal
 * .second compare equivalent and the second insert is dropped).  ordFirstHalf ascends by .second
 * (compFirst), ordSecHalf descends (compSec). */
typedef struct { int first, second; } or_pair;
typedef struct { or_pair v[32]; int n; int ascending; } or_pairset;

static void pairset_insert(or_pairset* s, or_pair p) {
    int pos = 0;
    for (pos = 0; pos < s->n; ++pos) {
        const or_pair* q = &s->v[pos];
        if (q->second == p.second) return; /* equivalent under the comparator: not inserted */
        if (s->ascending ? (p.second < q->second) : (p.second > q->second)) break;
    }
    memmove(&s->v[pos + 1], &s->v[pos], (size_t)(s->n - pos) * sizeof(or_pair));
    s->v[pos] = p;
    s->n++;
}

void or_bresenham_ring(int xc, int yc, int out[16][2]) {
    const int bresRadius = 3; /* include/FastDetector.hpp:34 */
    int xLoop = 0, yLoop = bresRadius, d = 3 - 2 * bresRadius;
    or_pairset first = {.n = 0, .ascending = 1}, second = {.n = 0, .ascending = 0};
    while (yLoop >= xLoop) {
        xLoop++;
        if (d <= 0) {
            d = d + 4 * xLoop + 6;
        } else {
            yLoop--;
            d = d + 4 * (xLoop - yLoop) + 10;
        }
        /* getAllSymPoints (src/FastDetector.cc:114-116) */
        const int sym[8][2] = {{xLoop, yLoop},   {yLoop, xLoop},   {yLoop, -xLoop}, {xLoop, -yLoop},
                               {-xLoop, -yLoop}, {-yLoop, -xLoop}, {-yLoop, xLoop}, {-xLoop, yLoop}};
        for (int i = 0; i < 8; ++i) {
            int xAct = sym[i][0] >= 0 ? xc + abs(sym[i][0]) : xc - abs(sym[i][0]);
            int yAct = sym[i][1] >= 0 ? yc - abs(sym[i][1]) : yc + abs(sym[i][1]);
            or_pair p = {xAct, yAct};
            if (sym[i][0] >= 0) pairset_insert(&first, p);
            else pairset_insert(&second, p);
        }
    }
    or_pair pf = {xc + bresRadius, yc}, ps = {xc - bresRadius, yc};
    pairset_insert(&first, pf);
    pairset_insert(&second, ps);
    int k = 0;
    out[k][0] = xc; out[k][1] = yc - bresRadius; k++;
    for (int i = 0; i < first.n && k < 16; ++i) { out[k][0] = first.v[i].first; out[k][1] = first.v[i].second; k++; }
    if (k < 16) { out[k][0] = xc; out[k][1] = yc + bresRadius; k++; }
    for (int i = 0; i < second.n && k < 16; ++i) { out[k][0] = second.v[i].first; out[k][1] = second.v[i].second; k++; }
}

/* checkInBetween, src/FastDetector.cc:155-161: uint8 operands promoted to int. */
static inline int or_similar(int cent, int cond, int thr) {
    return (cent > cond - thr) && (cent < cond + thr);
}

/* checkContiguousPixels, src/FastDetector.cc:135-153: >= 12 consecutive "different" ring pixels,
 * scanning index 0 -> 15 with no wrap-around.  getPixelVal(i, j) = data[i*cols + j] (src/Image.cc:15-17). */
int or_check_contiguous(uint8_t cent, const int ring[16][2], const uint8_t* img, int stride, int thr) {
    int currInd = 0, pixCount = 0;
    while (currInd < 16) {
        if (or_similar(cent, img[(size_t)ring[currInd][0] * stride + ring[currInd][1]], thr)) {
            pixCount = 0;
            currInd++;
        } else {
            pixCount++;
            currInd++;
        }
        if (pixCount >= 12) return 1;
    }
    return 0;
}

/* ========================================================================================== */
/* Harris response: getHarrisCornerResponse, src/FastDetector.cc:244-273                     */
/* ========================================================================================== */

/* OpenCV's internal hypot used by JacobiImpl_ (modules/core/src/lapack.cpp): a*sqrt(1+(b/a)^2). */
static inline float cv_hypotf(float a, float b) {
    a = fabsf(a);
    b = fabsf(b);
    if (a > b) {
        b /= a;
        return a * sqrtf(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * sqrtf(1 + a * a);
    }
    return 0;
}

/* cv::eigen(M, evals) for CV_32F without HAVE_EIGEN -> JacobiImpl_<float>(A, astep, W, V=0, ..., n)
 * (OpenCV 4.x modules/core/src/lapack.cpp).  Eigenvalues returned in descending order. */
void or_eigen_jacobi_f32(const float* Ain, int n, float* W) {
    float A[64];
    int indR[8], indC[8];
    const float eps = FLT_EPSILON;
    int i, j, k, m, iters, maxIters = n * n * 30;
    float mv = 0.f;
    if (n > 8) return;
    memcpy(A, Ain, sizeof(float) * (size_t)(n * n));
    const int astep = n;
    for (k = 0; k < n; k++) {
        W[k] = A[(astep + 1) * k];
        if (k < n - 1) {
            for (m = k + 1, mv = fabsf(A[astep * k + m]), i = k + 2; i < n; i++) {
                float val = fabsf(A[astep * k + i]);
                if (mv < val) mv = val, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            for (m = 0, mv = fabsf(A[k]), i = 1; i < k; i++) {
                float val = fabsf(A[astep * i + k]);
                if (mv < val) mv = val, m = i;
            }
            indC[k] = m;
        }
    }
    if (n > 1)
        for (iters = 0; iters < maxIters; iters++) {
            for (k = 0, mv = fabsf(A[indR[0]]), i = 1; i < n - 1; i++) {
                float val = fabsf(A[astep * i + indR[i]]);
                if (mv < val) mv = val, k = i;
            }
            int l = indR[k];
            for (i = 1; i < n; i++) {
                float val = fabsf(A[astep * indC[i] + i]);
                if (mv < val) mv = val, k = indC[i], l = i;
            }
            float p = A[astep * k + l];
            if (fabsf(p) <= eps) break;
            float y = (float)((double)(W[l] - W[k]) * 0.5);
            float t = fabsf(y) + cv_hypotf(p, y);
            float s = cv_hypotf(p, t);
            float c = t / s;
            s = p / s;
            t = (p / t) * p;
            if (y < 0) s = -s, t = -t;
            A[astep * k + l] = 0;
            W[k] -= t;
            W[l] += t;
            float a0, b0;
#define OR_ROTATE(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
            for (i = 0; i < k; i++) OR_ROTATE(A[astep * i + k], A[astep * i + l]);
            for (i = k + 1; i < l; i++) OR_ROTATE(A[astep * k + i], A[astep * i + l]);
            for (i = l + 1; i < n; i++) OR_ROTATE(A[astep * k + i], A[astep * l + i]);
#undef OR_ROTATE
            for (j = 0; j < 2; j++) {
                int idx = j == 0 ? k : l;
                if (idx < n - 1) {
                    for (m = idx + 1, mv = fabsf(A[astep * idx + m]), i = idx + 2; i < n; i++) {
                        float val = fabsf(A[astep * idx + i]);
                        if (mv < val) mv = val, m = i;
                    }
                    indR[idx] = m;
                }
                if (idx > 0) {
                    for (m = 0, mv = fabsf(A[idx]), i = 1; i < idx; i++) {
                        float val = fabsf(A[astep * i + idx]);
                        if (mv < val) mv = val, m = i;
                    }
                    indC[idx] = m;
                }
            }
        }
    /* sort eigenvalues descending (selection sort, as JacobiImpl_) */
    for (k = 0; k < n - 1; k++) {
        m = k;
        for (i = k + 1; i < n; i++)
            if (W[m] < W[i]) m = i;
        if (k != m) { float tmp = W[m]; W[m] = W[k]; W[k] = tmp; }
    }
}

/* cv::eigen(M, evals) for CV_32F in an OpenCV built WITH_EIGEN (HAVE_EIGEN, modules/core/src/lapack.cpp):
 * Eigen::SelfAdjointEigenSolver<MatrixXf>::compute(M, EigenvaluesOnly), eigenvalues reversed to descending.
 * Restated from Eigen 3.4.0 (Eigenvalues/SelfAdjointEigenSolver.h, Tridiagonalization.h, Jacobi/Jacobi.h), the
 * release the reference's macOS / Ubuntu setup installs (macInstalltion.txt; parity with a running build unpinned):
 *   - the lower triangle scaled by s = max |m_ij| (1 if 0); for n = 2 the tridiagonalisation is the identity
 *     (a one-element Householder vector: tau = 0, beta = m10; the rank update adds -0 terms only), so
 *     diag = (m00 / s, m11 / s), subdiag = m10 / s;
 *   - computeFromTridiagonal_impl: deflate when |e| < FLT_MIN or (e / FLT_EPSILON)^2 <= |d0| + |d1|, otherwise one
 *     implicit Wilkinson-shift QR step (tridiagonal_qr_step with numext::hypot and JacobiRotation::makeGivens), at
 *     most 30 n iterations; the eigenvalues are sorted ascending and multiplied back by s. */
static inline float eig_hypotf(float x, float y) {
    /* numext::hypot -> positive_real_hypot(|x|, |y|) */
    x = fabsf(x);
    y = fabsf(y);
    if (isinf(x) || isinf(y)) return INFINITY;
    if (isnan(x) || isnan(y)) return NAN;
    const float p = x > y ? x : y;  /* numext::maxi(x, y) = std::max */
    if (p == 0.0f) return 0.0f;
    const float qp = (y < x ? y : x) / p;  /* numext::mini(y, x) = std::min */
    return p * sqrtf(1.0f + qp * qp);
}

static inline void eig_make_givens(float p, float q, float* c, float* s) {
    if (q == 0.0f) {
        *c = p < 0.0f ? -1.0f : 1.0f;
        *s = 0.0f;
    } else if (p == 0.0f) {
        *c = 0.0f;
        *s = q < 0.0f ? 1.0f : -1.0f;
    } else if (fabsf(p) > fabsf(q)) {
        const float t = q / p;
        float u = sqrtf(1.0f + t * t);
        if (p < 0.0f) u = -u;
        *c = 1.0f / u;
        *s = -t * *c;
    } else {
        const float t = p / q;
        float u = sqrtf(1.0f + t * t);
        if (q < 0.0f) u = -u;
        *s = -1.0f / u;
        *c = -t * *s;
    }
}

void or_eigen_selfadjoint2_f32(float m00, float m01, float m11, float* W) {
    float scale = fabsf(m00);
    if (fabsf(m01) > scale) scale = fabsf(m01);
    if (fabsf(m11) > scale) scale = fabsf(m11);
    if (scale == 0.0f) scale = 1.0f;
    float d0 = m00 / scale, d1 = m11 / scale, e = m01 / scale;
    const float considerAsZero = FLT_MIN, precision_inv = 1.0f / FLT_EPSILON;
    int iter = 0, ok = 1;
    while (1) {
        if (fabsf(e) < considerAsZero) {
            e = 0.0f;
        } else {
            const float se = precision_inv * e;
            if (se * se <= (fabsf(d0) + fabsf(d1))) e = 0.0f;
        }
        if (e == 0.0f) break;
        iter++;
        if (iter > 30 * 2) { ok = 0; break; }
        /* tridiagonal_qr_step(start 0, end 1): Wilkinson shift, one Givens rotation */
        const float td = (d0 - d1) * 0.5f;
        float mu = d1;
        if (td == 0.0f) {
            mu -= fabsf(e);
        } else if (e != 0.0f) {
            const float e2 = e * e;
            const float h = eig_hypotf(td, e);
            if (e2 == 0.0f) mu -= e / ((td + (td > 0.0f ? h : -h)) / e);
            else mu -= e2 / (td + (td > 0.0f ? h : -h));
        }
        const float x = d0 - mu, z = e;
        if (z != 0.0f) {
            float c, sn;
            eig_make_givens(x, z, &c, &sn);
            const float sdk = sn * d0 + c * e;
            const float dkp1 = sn * e + c * d1;
            const float nd0 = c * (c * d0 - sn * e) - sn * (c * e - sn * d1);
            const float nd1 = sn * sdk + c * dkp1;
            const float ne = c * sdk - sn * dkp1;
            d0 = nd0;
            d1 = nd1;
            e = ne;
        }
    }
    /* ascending sort (only on success; NoConvergence leaves them, and cv::eigen then returns false with the output
     * array unwritten -- not reachable for 2 x 2 in practice), scale back, reverse to descending */
    if (ok && d1 < d0) { const float t = d0; d0 = d1; d1 = t; }
    d0 *= scale;
    d1 *= scale;
    W[0] = d1;
    W[1] = d0;
}

/* which cv::eigen the Harris response uses: 0 = JacobiImpl_ (OpenCV without Eigen), 1 = HAVE_EIGEN */
static int g_harris_eigen = 0;
void or_set_harris_eigen(int flavour) { g_harris_eigen = flavour; }

/* src/FastDetector.cc:264-272: eigenValues(0) is the larger.  The expression is
 *   (float)( (double)(float)(e0*e1) - 0.04 * std::pow((double)(float)(e1+e0), 2) )
 * std::pow(float,int) promotes to double; the square of a float is exact in double. */
float or_harris_response(float m00, float m01, float m11) {
    float M[4] = {m00, m01, m01, m11};
    float ev[2];
    if (g_harris_eigen == 1) or_eigen_selfadjoint2_f32(m00, m01, m11, ev);
    else or_eigen_jacobi_f32(M, 2, ev);
    float prod = ev[0] * ev[1];
    float sum = ev[1] + ev[0];
    double sq = (double)sum * (double)sum;
    double r = (double)prod - 0.04 * sq;
    return (float)r;
}

/* preComputeHarris (src/FastDetector.cc:204-214) via convolve2d (:164-200): 3x3 Sobel *correlation*
 * with a zero border; output(r, c) is written for r < H-2, c < W-2 and those pixels see image rows
 * r-1..r+1 (row -1 reads the zero border).  The remaining last two rows / cols stay 0. */
static void or_sobel(const uint8_t* img, int H, int W, int stride, float* Ix, float* Iy) {
    memset(Ix, 0, sizeof(float) * (size_t)H * W);
    memset(Iy, 0, sizeof(float) * (size_t)H * W);
    const float kx[3][3] = {{-1, 0, 1}, {-2, 0, 2}, {-1, 0, 1}};
    const float ky[3][3] = {{-1, -2, -1}, {0, 0, 0}, {1, 2, 1}};
    for (int r = 0; r < H - 2; ++r)
        for (int c = 0; c < W - 2; ++c) {
            float sx = 0, sy = 0;
            for (int k = 0; k < 3; ++k)
                for (int l = 0; l < 3; ++l) {
                    int rr = r + k - 1, cc = c + l - 1;
                    float p = (rr < 0 || cc < 0) ? 0.f : (float)img[(size_t)rr * stride + cc];
                    sx += kx[k][l] * p;
                    sy += ky[k][l] * p;
                }
            Ix[(size_t)r * W + c] = sx;
            Iy[(size_t)r * W + c] = sy;
        }
}

/* Literal getHarrisCornerResponse: three whole-image products per call (src/FastDetector.cc:249-251). */
static float or_harris_literal(const float* Ix, const float* Iy, int H, int W, int x, int y) {
    size_t P = (size_t)H * W;
    float* Ix2 = (float*)malloc(P * sizeof(float));
    float* Iy2 = (float*)malloc(P * sizeof(float));
    float* Ixy = (float*)malloc(P * sizeof(float));
    for (size_t i = 0; i < P; ++i) {
        Ix2[i] = Ix[i] * Ix[i];
        Iy2[i] = Iy[i] * Iy[i];
        Ixy[i] = Ix[i] * Iy[i];
    }
    float m00 = 0, m01 = 0, m10 = 0, m11 = 0;
    for (int i = x - 1; i <= x + 1; i++)
        for (int j = y - 1; j <= y + 1; j++) {
            m00 += Ix2[(size_t)i * W + j];
            m01 += Ixy[(size_t)i * W + j];
            m10 += Ixy[(size_t)i * W + j];
            m11 += Iy2[(size_t)i * W + j];
        }
    (void)m10;
    free(Ix2); free(Iy2); free(Ixy);
    return or_harris_response(m00, m01, m11);
}

static float or_harris_local(const float* Ix, const float* Iy, int W, int x, int y) {
    float m00 = 0, m01 = 0, m11 = 0;
    for (int i = x - 1; i <= x + 1; i++)
        for (int j = y - 1; j <= y + 1; j++) {
            float gx = Ix[(size_t)i * W + j], gy = Iy[(size_t)i * W + j];
            m00 += gx * gx;
            m01 += gx * gy;
            m11 += gy * gy;
        }
    return or_harris_response(m00, m01, m11);
}

/* ========================================================================================== */
/* getFastFeatures, src/FastDetector.cc:277-369                                                */
/* ========================================================================================== */

typedef struct { int x, y; float resp; int idx; } or_fastfeat;

/* std::sort by response descending (src/FastDetector.cc:343-345) is unstable; the restatement uses
 * the canonical total order (response desc, row-major scan index asc), i.e. what a stable sort of the
 * scan-ordered list gives.  Responses are compared as floats (so -0 == +0 as in the reference). */
static int or_fastfeat_cmp(const void* a, const void* b) {
    const or_fastfeat* A = (const or_fastfeat*)a;
    const or_fastfeat* B = (const or_fastfeat*)b;
    if (A->resp > B->resp) return -1;
    if (A->resp < B->resp) return 1;
    return (A->idx > B->idx) - (A->idx < B->idx);
}

int or_fast_detect(const uint8_t* img, int H, int W, int stride, int thr, int max_kp, int mode,
                   int32_t* rc, float* resp, int* n, int* n_cand,
                   int32_t* cand_idx, float* cand_resp, int cand_cap) {
    if (!img || H < 9 || W < 9 || stride < W || max_kp < 0) return -1;
    size_t P = (size_t)H * W;
    float* Ix = (float*)malloc(P * sizeof(float));
    float* Iy = (float*)malloc(P * sizeof(float));
    or_fastfeat* feats = (or_fastfeat*)malloc(sizeof(or_fastfeat) * (size_t)(H - 8) * (W - 8) + 1);
    if (!Ix || !Iy || !feats) { free(Ix); free(Iy); free(feats); return -2; }
    or_sobel(img, H, W, stride, Ix, Iy);

    int nf = 0;
    int ring0[16][2];
    or_bresenham_ring(0, 0, ring0);
    for (int i = 4; i < H - 4; i++) {
        for (int j = 4; j < W - 4; j++) {
            uint8_t cent = img[(size_t)i * stride + j];
            int ring[16][2];
            if (mode == 0) {
                /* rebuilt per pixel with the reference's std::vector / std::set containers, as it does */
                or_bresenham_ring_stl(i, j, ring);
            } else {
                for (int k = 0; k < 16; ++k) { ring[k][0] = i + ring0[k][0]; ring[k][1] = j + ring0[k][1]; }
            }
            /* pretest on ring indices 0, 7, 4, 12 (src/FastDetector.cc:304-317) */
            uint8_t p1 = img[(size_t)ring[0][0] * stride + ring[0][1]];
            uint8_t p8 = img[(size_t)ring[7][0] * stride + ring[7][1]];
            uint8_t p5 = img[(size_t)ring[4][0] * stride + ring[4][1]];
            uint8_t p13 = img[(size_t)ring[12][0] * stride + ring[12][1]];
            if (!or_similar(cent, p1, thr) && !or_similar(cent, p8, thr)) {
                if (!or_similar(cent, p5, thr) || !or_similar(cent, p13, thr)) {
                    if (or_check_contiguous(cent, ring, img, stride, thr)) {
                        float s = mode == 0 ? or_harris_literal(Ix, Iy, H, W, i, j)
                                            : or_harris_local(Ix, Iy, W, i, j);
                        feats[nf].x = i; feats[nf].y = j; feats[nf].resp = s; feats[nf].idx = i * W + j;
                        nf++;
                    }
                }
            }
        }
    }
    if (cand_idx || cand_resp) {
        for (int k = 0; k < nf && k < cand_cap; ++k) {
            if (cand_idx) cand_idx[k] = feats[k].idx;
            if (cand_resp) cand_resp[k] = feats[k].resp;
        }
    }
    qsort(feats, (size_t)nf, sizeof(or_fastfeat), or_fastfeat_cmp);
    int keep = nf > max_kp ? max_kp : nf; /* src/FastDetector.cc:353-362 */
    for (int k = 0; k < keep; ++k) {
        rc[2 * k] = feats[k].x;
        rc[2 * k + 1] = feats[k].y;
        if (resp) resp[k] = feats[k].resp;
    }
    *n = keep;
    if (n_cand) *n_cand = nf;
    free(Ix); free(Iy); free(feats);
    return 0;
}

/* ========================================================================================== */
/* Gaussian blur: cv::GaussianBlur(img, out, Size(9, 9), 2.5, 2.5), src/BriefDescriptor.cc:90   */
/* ========================================================================================== */

/* getGaussianKernelBitExact + getGaussianKernelFixedPoint_ED (OpenCV >= 3.4, modules/imgproc/src/
 * smooth.dispatch.cpp), restated in IEEE double (OpenCV uses softdouble; identical for these sizes,
 * checked against the published 9/2.5 kernel [12,22,31,41,44,41,31,22,12] in tests). */
void or_gauss_kernel_fixed(int n, double sigma, int ed, uint16_t* out) {
    double values[64];
    if (n <= 0 || n > 127 || !(n & 1)) return;
    double sigmaX = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
    double scale2X = -0.125 / (sigmaX * sigmaX);
    int n2_ = (n - 1) / 2;
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2_; i++, x += 2) {
        double t = exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2;
    sum += 1;
    double mul1 = 1.0 / sum;
    double k[128];
    for (int i = 0; i < n2_; i++) {
        double t = values[i] * mul1;
        k[i] = t;
        k[n - 1 - i] = t;
    }
    k[n2_] = mul1;
    const double mult = 256.0; /* ufixedpoint16: 8 fractional bits */
    double err = 0;
    long long s = 0;
    for (int i = 0; i < n2_; i++) {
        double adj = k[i] * mult + (ed ? err : 0.0);
        long long v0 = llrint(adj); /* cvRound: round half to even */
        err = adj - (double)v0;
        out[i] = (uint16_t)v0;
        out[n - 1 - i] = (uint16_t)v0;
        s += v0;
    }
    s *= 2;
    out[n2_] = (uint16_t)llrint(mult - (double)s);
}

/* BORDER_REFLECT_101 (cv::borderInterpolate): gfedcb|abcdefgh|gfedcba */
static inline int or_reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

/* GaussianBlurFixedPoint<uint8_t, ufixedpoint16> (smooth.simd.hpp): horizontal pass
 * h = sum_j kx_j * p (exact, <= 255*256), vertical pass v = sum_i ky_i * h_i (exact u32), output
 * (v + 2^15) >> 16. */
void or_gaussian_blur_u8(const uint8_t* img, int H, int W, int stride, const uint16_t* k, int n,
                         uint8_t* out) {
    int half = n / 2;
    uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)H * W);
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) {
            uint32_t acc = 0;
            for (int j = 0; j < n; ++j) acc += (uint32_t)k[j] * img[(size_t)r * stride + or_reflect101(c + j - half, W)];
            h[(size_t)r * W + c] = acc;
        }
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) {
            uint32_t acc = 0;
            for (int i = 0; i < n; ++i) acc += (uint32_t)k[i] * h[(size_t)or_reflect101(r + i - half, H) * W + c];
            uint32_t v = (acc + (1u << 15)) >> 16;
            out[(size_t)r * W + c] = (uint8_t)(v > 255 ? 255 : v);
        }
    free(h);
}

/* ========================================================================================== */
/* BRIEF: src/BriefDescriptor.cc                                                                */
/* ========================================================================================== */

/* checkBoundry (src/BriefDescriptor.cc:128-136), called as checkBoundry(kp.y=col, kp.x=row, W, H). */
static inline int or_check_boundary(int x, int y, int width, int height) {
    if (x - 8 < 0 || x + 8 > width) return 0;
    if (y - 8 < 0 || y + 8 > height) return 0;
    return 1;
}

/* Image::getPixelVal(i, j) = data[i*cols + j] (src/Image.cc:15-17) on the blurred copy.  The boundary
 * check admits row = H-8 / col = W-8 with offsets up to +8, so the linear index can run one row into
 * the next (reproduced) or past the buffer end (UB in the reference; 0 here). */
static inline uint8_t or_blur_pix(const uint8_t* blur, int H, int W, int i, int j) {
    long long idx = (long long)i * W + j;
    if (idx < 0 || idx >= (long long)H * W) return 0;
    return blur[idx];
}

int or_compute_brief_blurred(const uint8_t* blur, int H, int W, const int8_t* offsets,
                             const int32_t* rc, int n, yv_keypoint* out, int* n_out) {
    int m = 0;
    for (int i = 0; i < n; i++) {
        yv_keypoint kp;
        memset(&kp, 0, sizeof(kp));
        kp.x = rc[2 * i];
        kp.y = rc[2 * i + 1];
        kp.id = i;
        kp.matched = 0;
        if (or_check_boundary(kp.y, kp.x, W, H)) {
            for (int j = 0; j < 256; j++) { /* patchSize = 256 (src/LoopHandler.cc:7) */
                int p1x = kp.x + offsets[4 * j + 0], p1y = kp.y + offsets[4 * j + 1];
                int p2x = kp.x + offsets[4 * j + 2], p2y = kp.y + offsets[4 * j + 3];
                int byte = j / 8;
                if (or_blur_pix(blur, H, W, p1x, p1y) > or_blur_pix(blur, H, W, p2x, p2y))
                    kp.featVec[byte] |= (uint8_t)(1 << (j % 8));
                else
                    kp.featVec[byte] &= (uint8_t)~(1 << (j % 8));
            }
            out[m++] = kp;
        }
    }
    *n_out = m;
    return 0;
}

int or_compute_brief(const uint8_t* img, int H, int W, int stride, const uint16_t* k9,
                     const int8_t* offsets, const int32_t* rc, int n, yv_keypoint* out, int* n_out) {
    uint8_t* blur = (uint8_t*)malloc((size_t)H * W);
    if (!blur) return -2;
    or_gaussian_blur_u8(img, H, W, stride, k9, 9, blur);
    int rcode = or_compute_brief_blurred(blur, H, W, offsets, rc, n, out, n_out);
    free(blur);
    return rcode;
}

/* ---- std::mt19937 + libstdc++ uniform_int_distribution<int>(-8, 8) (GCC >= 11) ---- */
typedef struct { uint32_t mt[624]; int idx; } or_mt19937;

static void mt_seed(or_mt19937* g, uint32_t seed) {
    g->mt[0] = seed;
    for (int i = 1; i < 624; ++i) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->idx = 624;
}

static uint32_t mt_next(or_mt19937* g) {
    if (g->idx >= 624) {
        for (int i = 0; i < 624; ++i) {
            uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
            g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        g->idx = 0;
    }
    uint32_t y = g->mt[g->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* libstdc++ uniform_int_distribution::operator() downscaling branch for a 32-bit engine:
 * Lemire's nearly-divisionless method (_S_nd). */
static int mt_uniform_int(or_mt19937* g, int a, int b) {
    uint32_t range = (uint32_t)(b - a) + 1u;
    uint64_t product = (uint64_t)mt_next(g) * range;
    uint32_t low = (uint32_t)product;
    if (low < range) {
        uint32_t threshold = (uint32_t)(-range) % range;
        while (low < threshold) {
            product = (uint64_t)mt_next(g) * range;
            low = (uint32_t)product;
        }
    }
    return a + (int)(product >> 32);
}

void or_brief_offsets_mt19937(uint32_t seed, int8_t* out) {
    or_mt19937 g;
    mt_seed(&g, seed);
    for (int i = 0; i < 256; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (int8_t)mt_uniform_int(&g, -8, 8);
}

/* A persistent std::mt19937 drawing uniform_int_distribution<int>(a, b) values, as the C++ LoopHandler's getFRANSAC
 * draws its 400 x 8 sample indices (ya_vo_amd/frontend/loop_handler.cpp: one engine seeded once, a fresh
 * distribution of range [0, n - 1] per call; the reference seeds from std::random_device, src/3DHandler.cc:157-159). */
void* or_mt19937_new(uint32_t seed) {
    or_mt19937* g = (or_mt19937*)malloc(sizeof(or_mt19937));
    if (g) mt_seed(g, seed);
    return g;
}

void or_mt19937_uniform_ints(void* g, int a, int b, int count, int32_t* out) {
    for (int i = 0; i < count; ++i) out[i] = mt_uniform_int((or_mt19937*)g, a, b);
}

void or_mt19937_free(void* g) { free(g); }

/* Brief::popCount, src/BriefDescriptor.cc:151-160 (bit loop kept literally). */
static int or_popcount_literal(uint8_t v) {
    int count = 0;
    while (v != 0) {
        if (v & 0x1) count++;
        v = (uint8_t)(v >> 1);
    }
    return count;
}

int or_hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += or_popcount_literal((uint8_t)(a[i] ^ b[i]));
    return d;
}

/* Brief::matchFeatures, src/BriefDescriptor.cc:163-183: first index of the minimum wins (strict <).
 * pt1 is a full copy of the query keypoint; pt2 = KeyPoint(x, y, id) of the best train point with
 * matched=false and a zero descriptor; an empty train set leaves pt2 = (0,0,0), distance = INT_MAX. */
int or_match(const yv_keypoint* q, int nq, const yv_keypoint* t, int nt, yv_match* out) {
    for (int i = 0; i < nq; i++) {
        int minDist = INT_MAX;
        yv_keypoint kp2;
        memset(&kp2, 0, sizeof(kp2));
        for (int j = 0; j < nt; j++) {
            int d = or_hamming(q[i].featVec, t[j].featVec);
            if (d < minDist) {
                minDist = d;
                kp2.x = t[j].x;
                kp2.y = t[j].y;
                kp2.id = t[j].id;
            }
        }
        memset(&out[i], 0, sizeof(yv_match));
        out[i].pt1 = q[i];
        memset(out[i].pt1._pad, 0, 3);
        out[i].pt2 = kp2;
        out[i].distance = minDist;
    }
    return 0;
}

/* Brief::removeOutliers, src/BriefDescriptor.cc:213-231.  keep iff distance < max(2*min_dist, thr);
 * kept copies get matched=true on both points.  2*min is evaluated with int wrap-around (the reference
 * overflows when every distance is INT_MAX); an empty list yields nothing (reference: UB deref). */
int or_remove_outliers(const yv_match* in, int n, int thr, yv_match* out, int* n_out) {
    int m = 0;
    if (n <= 0) { *n_out = 0; return 0; }
    int minD = in[0].distance;
    for (int i = 1; i < n; i++)
        if (in[i].distance < minD) minD = in[i].distance;
    int twice = (int)((unsigned)minD * 2u);
    int lim = twice > thr ? twice : thr;
    for (int i = 0; i < n; i++) {
        if (in[i].distance < lim) {
            out[m] = in[i];
            out[m].pt1.matched = 1;
            out[m].pt2.matched = 1;
            m++;
        }
    }
    *n_out = m;
    return 0;
}

/* ========================================================================================== */
/* parseCalibString, src/Utils.cc:4-28                                                          */
/* ========================================================================================== */
int or_parse_calib_string(const char* s, double out[16]) {
    /* getline(f, s, ' ') splits on single spaces; std::stod on each token; tokens that do not start a
     * number ("P0:") throw and are skipped.  The reference indexes matValues[0..15] unconditionally. */
    double vals[64];
    int nv = 0;
    const char* p = s;
    while (*p && nv < 64) {
        const char* q = p;
        while (*q && *q != ' ') q++;
        size_t len = (size_t)(q - p);
        if (len > 0 && len < 63) {
            char tok[64];
            memcpy(tok, p, len);
            tok[len] = 0;
            char* end = NULL;
            /* std::stod skips leading whitespace and accepts a numeric prefix */
            double d = strtod(tok, &end);
            if (end != tok) vals[nv++] = d;
        }
        p = *q ? q + 1 : q;
    }
    for (int i = 0; i < 16; ++i) out[i] = i < nv ? vals[i] : 0.0;
    return nv;
}
