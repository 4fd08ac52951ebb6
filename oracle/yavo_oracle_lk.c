/*
 * yavo_oracle_lk.c -- CPU restatement of cv::calcOpticalFlowPyrLK as the reference calls it
 * (src/LoopHandler.cc:372-375: winSize 11x11, maxLevel 3, TermCriteria(COUNT+EPS, 30, 0.01), flags 0,
 * minEigThreshold 0.001).  TEST INFRASTRUCTURE ONLY (see yavo_oracle.h).
 *
 * OpenCV (4.x, version unpinned by the reference, CMakeLists.txt:6) is not present in this image; this is a
 * restatement of its published algorithm (modules/video/src/lkpyramid.cpp), the scalar code path:
 *   buildOpticalFlowPyramid  pyrDown levels (5x5 [1 4 6 4 1]^2 / 256, BORDER_REFLECT_101), each level bordered
 *                            by winSize with BORDER_REFLECT_101; stop when the next level is <= winSize
 *   calcSharrDeriv           3x3 Scharr, int16 (dx, dy) interleaved, REFLECT_101 rows/cols; the derivative
 *                            image is bordered with zeros (BORDER_CONSTANT)
 *   LKTrackerInvoker         14-bit fixed-point bilinear weights (cvRound), CV_DESCALE, float sums of the
 *                            integer products, minEig test, Newton steps with the eps^2 test and the
 *                            oscillation check, the level-0 error (mean |diff| / 32)
 * Sums over the 11x11 window are taken either in OpenCV's scalar order (sum_mode 0, row-major) or in the
 * GPU kernel's order (sum_mode 1: 16 lanes per point, S = ceil(win / 4); lane g owns the S x S task at rows
 * S (g >> 2) .., columns S (g & 3) .. of the window and adds its in-window terms row-major from 0.0f; the 16
 * partials are then combined by the butterfly q[l] = q[l] + q[l ^ off], off = 8, 4, 2, 1, whose lane-0 value
 * is the tree p[l] += p[l + off]).  The
 * reference's x86 OpenCV build runs a 4-lane SIMD path for x < 8 of each row, another float order: parity
 * with the reference binary is unpinned (no fixture holds LK outputs).
 */
#include "yavo_oracle.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        if (p >= len) p = 2 * len - p - 2;
    }
    return p;
}

/* cv::pyrDown for CV_8U, BORDER_REFLECT_101: dst (H+1)/2 x (W+1)/2, dst(y, x) = (sum_ij w_i w_j
 * src(2y+i-2, 2x+j-2) + 128) >> 8, w = {1, 4, 6, 4, 1} (integer: exact in any order). */
void or_pyr_down(const uint8_t* src, int H, int W, int sstride, uint8_t* dst) {
    static const int w[5] = {1, 4, 6, 4, 1};
    const int Hd = (H + 1) / 2, Wd = (W + 1) / 2;
    for (int y = 0; y < Hd; ++y)
        for (int x = 0; x < Wd; ++x) {
            int acc = 0;
            for (int i = 0; i < 5; ++i) {
                const int r = reflect101(2 * y + i - 2, H);
                int row = 0;
                for (int j = 0; j < 5; ++j) row += w[j] * src[r * sstride + reflect101(2 * x + j - 2, W)];
                acc += w[i] * row;
            }
            dst[y * Wd + x] = (uint8_t)((acc + 128) >> 8);
        }
}

/* calcSharrDeriv: dx = t0(x+1) - t0(x-1), t0 = 3 (s(y-1) + s(y+1)) + 10 s(y); dy = 3 (t1(x+1) + t1(x-1))
 * + 10 t1(x), t1 = s(y+1) - s(y-1); rows and columns REFLECT_101.  d = [H][W][2] int16. */
void or_scharr(const uint8_t* src, int H, int W, int sstride, int16_t* d) {
    int* t0 = (int*)malloc(sizeof(int) * (size_t)W);
    int* t1 = (int*)malloc(sizeof(int) * (size_t)W);
    for (int y = 0; y < H; ++y) {
        const uint8_t* s0 = src + reflect101(y - 1, H) * sstride;
        const uint8_t* s1 = src + y * sstride;
        const uint8_t* s2 = src + reflect101(y + 1, H) * sstride;
        for (int x = 0; x < W; ++x) {
            t0[x] = (s0[x] + s2[x]) * 3 + s1[x] * 10;
            t1[x] = s2[x] - s0[x];
        }
        for (int x = 0; x < W; ++x) {
            const int xl = reflect101(x - 1, W), xr = reflect101(x + 1, W);
            d[(y * W + x) * 2] = (int16_t)(t0[xr] - t0[xl]);
            d[(y * W + x) * 2 + 1] = (int16_t)((t1[xr] + t1[xl]) * 3 + t1[x] * 10);
        }
    }
    free(t0);
    free(t1);
}

typedef struct {
    int H, W;
    const uint8_t* img;  /* [H][W] */
    const int16_t* der;  /* [H][W][2], NULL for J */
} lk_level;

/* bordered accesses: image REFLECT_101, derivative image zero outside */
static int img_at(const lk_level* L, int y, int x) { return L->img[reflect101(y, L->H) * L->W + reflect101(x, L->W)]; }
static int der_at(const lk_level* L, int y, int x, int c) {
    if (y < 0 || y >= L->H || x < 0 || x >= L->W) return 0;
    return L->der[(y * L->W + x) * 2 + c];
}

#define LK_W_BITS 14
#define LK_DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

/* window sums in the requested order; terms[p] for p = 0 .. win^2 - 1 in row-major window order */
static float lk_sum(const float* terms, int win, int sum_mode) {
    if (sum_mode == 0) {
        float s = 0.0f;
        for (int p = 0; p < win * win; ++p) s = s + terms[p];
        return s;
    }
    const int S = (win + 3) / 4;
    float part[16];
    for (int g = 0; g < 16; ++g) {
        part[g] = 0.0f;
        for (int i = 0; i < S; ++i)
            for (int j = 0; j < S; ++j) {
                const int y = S * (g >> 2) + i, x = S * (g & 3) + j;
                if (y < win && x < win) part[g] = part[g] + terms[y * win + x];
            }
    }
    for (int off = 8; off > 0; off >>= 1)
        for (int l = 0; l < off; ++l) part[l] = part[l] + part[l + off];
    return part[0];
}

static void lk_weights(float a, float b, int* iw) {
    iw[0] = (int)lrintf((1.f - a) * (1.f - b) * (float)(1 << LK_W_BITS));
    iw[1] = (int)lrintf(a * (1.f - b) * (float)(1 << LK_W_BITS));
    iw[2] = (int)lrintf((1.f - a) * b * (float)(1 << LK_W_BITS));
    iw[3] = (1 << LK_W_BITS) - iw[0] - iw[1] - iw[2];
}

/* One point at one level (LKTrackerInvoker::operator() body). */
static void lk_point(const lk_level* I, const lk_level* J, int level, int max_level, int win, int max_count,
                     double eps2, double min_eig_thr, const float* prev_pt, float* next_pt, uint8_t* status,
                     float* err, int sum_mode) {
    const float halfw = (float)((win - 1) * 0.5f);
    const float scale = (float)(1. / (1 << level));
    float px = prev_pt[0] * scale, py = prev_pt[1] * scale;
    float nx, ny;
    if (level == max_level) {
        nx = px;
        ny = py;
    } else {
        nx = next_pt[0] * 2.f;
        ny = next_pt[1] * 2.f;
    }
    next_pt[0] = nx;
    next_pt[1] = ny;
    px -= halfw;
    py -= halfw;
    const int ipx = (int)floorf(px), ipy = (int)floorf(py);
    if (ipx < -win || ipx >= I->W || ipy < -win || ipy >= I->H) {
        if (level == 0) {
            *status = 0;
            *err = 0;
        }
        return;
    }
    int iw[4];
    lk_weights(px - (float)ipx, py - (float)ipy, iw);
    const int n = win * win;
    int16_t* Iw = (int16_t*)malloc(sizeof(int16_t) * (size_t)n * 3);
    float* t11 = (float*)malloc(sizeof(float) * (size_t)n * 3);
    float *t12 = t11 + n, *t22 = t11 + 2 * n;
    for (int y = 0; y < win; ++y)
        for (int x = 0; x < win; ++x) {
            const int yy = ipy + y, xx = ipx + x, p = y * win + x;
            const int ival = LK_DESCALE(img_at(I, yy, xx) * iw[0] + img_at(I, yy, xx + 1) * iw[1] +
                                            img_at(I, yy + 1, xx) * iw[2] + img_at(I, yy + 1, xx + 1) * iw[3],
                                        LK_W_BITS - 5);
            const int ixv = LK_DESCALE(der_at(I, yy, xx, 0) * iw[0] + der_at(I, yy, xx + 1, 0) * iw[1] +
                                           der_at(I, yy + 1, xx, 0) * iw[2] + der_at(I, yy + 1, xx + 1, 0) * iw[3],
                                       LK_W_BITS);
            const int iyv = LK_DESCALE(der_at(I, yy, xx, 1) * iw[0] + der_at(I, yy, xx + 1, 1) * iw[1] +
                                           der_at(I, yy + 1, xx, 1) * iw[2] + der_at(I, yy + 1, xx + 1, 1) * iw[3],
                                       LK_W_BITS);
            Iw[3 * p] = (int16_t)ival;
            Iw[3 * p + 1] = (int16_t)ixv;
            Iw[3 * p + 2] = (int16_t)iyv;
            t11[p] = (float)(ixv * ixv);
            t12[p] = (float)(ixv * iyv);
            t22[p] = (float)(iyv * iyv);
        }
    const float FLT_SCALE = 1.f / (1 << 20);
    const float A11 = lk_sum(t11, win, sum_mode) * FLT_SCALE;
    const float A12 = lk_sum(t12, win, sum_mode) * FLT_SCALE;
    const float A22 = lk_sum(t22, win, sum_mode) * FLT_SCALE;
    float D = A11 * A22 - A12 * A12;
    const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win * win);
    if (minEig < min_eig_thr || D < FLT_EPSILON) {
        if (level == 0) *status = 0;
        free(Iw);
        free(t11);
        return;
    }
    D = 1.f / D;
    nx -= halfw;
    ny -= halfw;
    float pdx = 0.f, pdy = 0.f;
    float* tb = t11;  /* reuse: tb1 = t11, tb2 = t12 */
    for (int j = 0; j < max_count; ++j) {
        const int inx = (int)floorf(nx), iny = (int)floorf(ny);
        if (inx < -win || inx >= J->W || iny < -win || iny >= J->H) {
            if (level == 0) *status = 0;
            break;
        }
        lk_weights(nx - (float)inx, ny - (float)iny, iw);
        for (int y = 0; y < win; ++y)
            for (int x = 0; x < win; ++x) {
                const int yy = iny + y, xx = inx + x, p = y * win + x;
                const int diff = LK_DESCALE(img_at(J, yy, xx) * iw[0] + img_at(J, yy, xx + 1) * iw[1] +
                                                img_at(J, yy + 1, xx) * iw[2] + img_at(J, yy + 1, xx + 1) * iw[3],
                                            LK_W_BITS - 5) - Iw[3 * p];
                tb[p] = (float)(diff * Iw[3 * p + 1]);
                t12[p] = (float)(diff * Iw[3 * p + 2]);
            }
        const float b1 = lk_sum(tb, win, sum_mode) * FLT_SCALE;
        const float b2 = lk_sum(t12, win, sum_mode) * FLT_SCALE;
        const float dx = (float)((A12 * b2 - A22 * b1) * D);
        const float dy = (float)((A12 * b1 - A11 * b2) * D);
        nx += dx;
        ny += dy;
        next_pt[0] = nx + halfw;
        next_pt[1] = ny + halfw;
        if ((double)dx * dx + (double)dy * dy <= eps2) break;
        if (j > 0 && fabsf(dx + pdx) < 0.01 && fabsf(dy + pdy) < 0.01) {
            next_pt[0] -= dx * 0.5f;
            next_pt[1] -= dy * 0.5f;
            break;
        }
        pdx = dx;
        pdy = dy;
    }
    if (*status && level == 0) {
        const float ex = next_pt[0] - halfw, ey = next_pt[1] - halfw;
        const int inx = (int)floorf(ex), iny = (int)floorf(ey);
        if (inx < -win || inx >= J->W || iny < -win || iny >= J->H) {
            *status = 0;
        } else {
            lk_weights(ex - (float)inx, ey - (float)iny, iw);
            for (int y = 0; y < win; ++y)
                for (int x = 0; x < win; ++x) {
                    const int yy = iny + y, xx = inx + x, p = y * win + x;
                    const int diff = LK_DESCALE(img_at(J, yy, xx) * iw[0] + img_at(J, yy, xx + 1) * iw[1] +
                                                    img_at(J, yy + 1, xx) * iw[2] + img_at(J, yy + 1, xx + 1) * iw[3],
                                                LK_W_BITS - 5) - Iw[3 * p];
                    tb[p] = fabsf((float)diff);
                }
            *err = lk_sum(tb, win, sum_mode) * 1.f / (float)(32 * win * win);
        }
    }
    free(Iw);
    free(t11);
}

/* cv::calcOpticalFlowPyrLK(prev, next, prevPts, nextPts, status, err, Size(win, win), max_level,
 * TermCriteria(COUNT+EPS, max_count, eps), 0, min_eig) on u8 images [H][W].  pts are (x = column,
 * y = row) as cv::Point2f.  Returns the number of pyramid levels - 1 actually used. */
int or_lk_pyr(const uint8_t* prev, const uint8_t* next, int H, int W, const float* prev_pts, int n, int win,
              int max_level, int max_count, double eps, double min_eig, float* next_pts, uint8_t* status,
              float* err, int sum_mode) {
    /* pyramid sizes (buildOpticalFlowPyramid: stop when the next level would be <= winSize) */
    int Hs[16], Ws[16], levels = 0;
    Hs[0] = H;
    Ws[0] = W;
    for (int l = 0; l < max_level && l < 15; ++l) {
        const int h = (Hs[l] + 1) / 2, w = (Ws[l] + 1) / 2;
        if (w <= win || h <= win) break;
        Hs[l + 1] = h;
        Ws[l + 1] = w;
        levels = l + 1;
    }
    uint8_t* pp[16];
    uint8_t* np[16];
    pp[0] = (uint8_t*)prev;
    np[0] = (uint8_t*)next;
    for (int l = 1; l <= levels; ++l) {
        pp[l] = (uint8_t*)malloc((size_t)Hs[l] * Ws[l]);
        np[l] = (uint8_t*)malloc((size_t)Hs[l] * Ws[l]);
        or_pyr_down(pp[l - 1], Hs[l - 1], Ws[l - 1], Ws[l - 1], pp[l]);
        or_pyr_down(np[l - 1], Hs[l - 1], Ws[l - 1], Ws[l - 1], np[l]);
    }
    for (int i = 0; i < n; ++i) {
        status[i] = 1;
        err[i] = 0.f;
    }
    /* TermCriteria: eps clipped to [0, 10] and squared; maxCount clipped to [0, 100] */
    double e = eps < 0 ? 0 : (eps > 10 ? 10 : eps);
    const double eps2 = e * e;
    const int mc = max_count < 0 ? 0 : (max_count > 100 ? 100 : max_count);
    for (int l = levels; l >= 0; --l) {
        int16_t* der = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)Hs[l] * Ws[l]);
        or_scharr(pp[l], Hs[l], Ws[l], Ws[l], der);
        lk_level I = {Hs[l], Ws[l], pp[l], der}, J = {Hs[l], Ws[l], np[l], NULL};
        for (int i = 0; i < n; ++i)
            lk_point(&I, &J, l, levels, win, mc, eps2, min_eig, prev_pts + 2 * i, next_pts + 2 * i, status + i,
                     err + i, sum_mode);
        free(der);
    }
    for (int l = 1; l <= levels; ++l) {
        free(pp[l]);
        free(np[l]);
    }
    return levels;
}
