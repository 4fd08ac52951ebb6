/*
 * yavo_oracle_ba.c -- CPU restatement of the sliding-window bundle adjustment of BASELINE.json config 5 / SURVEY.md
 * 8d-8e (20 keyframe poses, ~10k landmarks, ~5 observations each).  TEST INFRASTRUCTURE ONLY (see yavo_oracle.h).
 *
 * The reference has no multi-pose BA: Optimizer::partialBA (src/Optimizer.cc:17-60) is a pose-only Gauss-Newton
 * stub and src/test.cc:318-360 is pose-only too.  What it does have is the machinery such a BA is built from, and
 * this restates that machinery:
 *   edge            the reference's projection edge (include/Optimizer.hpp:64-126): e = meas - (K (T X)).xy / z,
 *                   J_pose = its linearizeOplus (2 x 6, (rho, phi), no cx / cy); the landmark half of a binary
 *                   pose-landmark edge is J_point = J_pose[:, 0:3] R (g2o EdgeProjectXYZ2UV's form)
 *   vertices        VertexPose::oplusImpl T <- exp(dx) T (Optimizer.hpp:51-57); landmark X <- X + dx; the first
 *                   n_fixed poses are fixed (gauge)
 *   solver          g2o OptimizationAlgorithmLevenberg (as or_pose_lm: lambda init tau = 1e-5 times the largest
 *                   Hessian diagonal, up to 10 trials, rho / scale with scale = x.(lambda x + b) + 1e-3, good-step
 *                   factor max(1/3, min(2/3, 1 - (2 rho - 1)^3)), bad step lambda *= ni, ni *= 2) over
 *                   BlockSolver_6_3: H_pp (block diagonal: no pose-pose edges), H_ll (3 x 3 per landmark), H_pl
 *                   (6 x 3 per edge); lambda on every diagonal; Schur complement with explicit 3 x 3 inverses;
 *                   LinearSolverDense = Eigen LDLT (unblocked, diagonal pivoting) on the reduced pose system;
 *                   landmark back-substitution
 * Summation orders (the GPU kernels, yavo_ba.hip, follow them bit for bit; g2o's own orders are not exposed, so
 * parity with a g2o build is unpinned):
 *   tree4096  values indexed k = 0 .. n-1: partial[t] = sum of items k = t mod 4096 in ascending k (from 0.0), then
 *             p[t] += p[t + off], off = 2048 .. 1; used for each pose's H_pp / b_p over its edges (edge order), for
 *             each Schur block entry's sum over the co-visible pairs of its two poses (landmark order), v = base -
 *             total, for each b_schur entry's sum over the pose's edges (edge order)
 *   landmark blocks  chi2 and the landmarks' part of the LM scale: per landmark a sequential sum from 0.0 (|e|^2 over
 *             its edges in edge order / its three x (lambda x + b) items), blocks of 256 landmarks as a halving tree
 *             over 256 slots (0.0 past L), block totals into 256 leaves (block b into leaf b mod 256, ascending b,
 *             from 0.0), a halving tree over the leaves; the scale = (the free poses' items in tree256 order: leaf
 *             t = items j = t mod 256 ascending, halving tree) + (the landmark part)
 *   sequential per landmark over its edges (edge order) for H_ll / b_l and the back-substitution
 * g2o order (or_ba_lm_mode(..., mode 1), the check the kernel order is measured against, never the GPU's order):
 *   g2o's own loops restated as sequential chains (g2o BlockSolver<Traits>::buildSystem / solve, SparseOptimizer::
 *   activeRobustChi2, OptimizationAlgorithmLevenberg::computeScale; g2o is not vendored by the reference, its version
 *   unpinned, CMakeLists.txt:22-23): H_pp / b_p accumulated edge by edge in edge (id) order from 0.0 (each edge's
 *   constructQuadraticForm, `from->A() += AtO * A`, `b += A^T omega_r` with omega_r = -e); the Schur block of poses
 *   (p1 <= p2) starts at H_pp + lambda I (or 0) and each co-visible landmark, ascending, subtracts its
 *   BDinv * B_j^T term (`(*Hi1i2).noalias() -= BDinv * Bj->transpose()`, BDinv = B_i Dinv); LinearSolverDense
 *   copies each upper block and then its transpose, so a diagonal block enters the dense matrix transposed (its
 *   lower triangle, the one Eigen's LDLT reads, holds block(b, a)); b_schur = b_p - coefficients, where the
 *   coefficients accumulate B_i (Dinv b_l) landmark by landmark (ascending; poses of a landmark ascending);
 *   the landmark update cl = b_l + B^T (-x_p) over the landmark's poses ascending (SparseBlockMatrixCCS::
 *   rightMultiply), x_l = Dinv cl; chi2 = sum over edges in edge order from 0.0 of e.(Omega e); the scale =
 *   sum over x = [x_p; x_l] in vector order from 0.0.  Small fixed-size products (3- and 6-term inner products)
 *   are left to right, as in the kernel order (Eigen's SIMD association of them is build-dependent).
 * (Rounds 1-4 summed the Schur and b_schur entries as one sequential chain each, and H_pp / b_p, chi2 and the scale
 * in a 256-leaf tree. A 3,800-term chain is latency-bound on one GPU lane, and 256 leaves leave each GPU lane ~15
 * dependent loads (and chi2's chains 300-450 dependent additions); with 4096 leaves a configs[2] window's sums have
 * at most one item per leaf for the blocks and ~28 for chi2, so the loads are in flight at once. Round 5 then moved
 * chi2 and the scale to the landmark-block order: the GPU's step kernel, one lane per landmark, sums them where it
 * forms the trial state, without a separate pass over the stored |e|^2 and scale items.)
 */
#include "yavo_oracle.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BA_NW 4096
typedef struct {
    double part[BA_NW];
    int used;  /* leaves [used, BA_NW) are still 0.0 */
} tree4096;
static void w_reset(tree4096* t) { t->used = 0; }
static void w_add(tree4096* t, int k, double v) {
    const int i = k % BA_NW;
    while (t->used <= i) t->part[t->used++] = 0.0;
    t->part[i] = t->part[i] + v;
}
/* the halving tree over all 4096 leaves; the untouched leaves are 0.0 (x + 0.0 is x except -0.0 + 0.0 = 0.0, so a
 * level that adds a zero leaf is applied as an addition, not skipped) */
static double w_total(tree4096* t) {
    double* p = t->part;
    int n = t->used;  /* p[i] for i >= n is 0.0 */
    for (int off = BA_NW / 2; off > 0; off >>= 1) {
        const int m = n < off ? n : off;  /* p[i], i < m, are the live leaves this level adds to */
        for (int i = 0; i < m; ++i) p[i] = p[i] + (i + off < n ? p[i + off] : 0.0);
        n = m;
    }
    return n > 0 ? p[0] : 0.0;
}

/* e = meas - (K (T X)).xy / z  (or_se3_act = Sophus T * X) */
static void ba_error(const double* T, const double* K, const double* X, const double* meas, double* e) {
    double pc[3];
    or_se3_act(T, X, pc);
    const double u0 = K[0] * pc[0] + K[1] * pc[1] + K[2] * pc[2];
    const double u1 = K[3] * pc[0] + K[4] * pc[1] + K[5] * pc[2];
    const double u2 = K[6] * pc[0] + K[7] * pc[1] + K[8] * pc[2];
    e[0] = meas[0] - u0 / u2;
    e[1] = meas[1] - u1 / u2;
}

/* J_pose (2 x 6, the reference's linearizeOplus) and J_point = J_pose[:, 0:3] R (2 x 3) */
static void ba_jacobians(const double* T, const double* K, const double* X, double* Jp, double* Jl) {
    double pc[3], R[9];
    or_se3_act(T, X, pc);
    or_quat_to_R(T, R);
    const double fx = K[0], fy = K[4];
    const double x = pc[0], y = pc[1], z = pc[2];
    const double zinv = 1.0 / (z + 1e-18);
    const double zinv2 = zinv * zinv;
    Jp[0] = -fx * zinv; Jp[1] = 0; Jp[2] = fx * x * zinv2; Jp[3] = fx * x * y * zinv2;
    Jp[4] = -fx - fx * x * x * zinv2; Jp[5] = fx * y * zinv;
    Jp[6] = 0; Jp[7] = -fy * zinv; Jp[8] = fy * y * zinv2; Jp[9] = fy + fy * y * y * zinv2;
    Jp[10] = -fy * x * y * zinv2; Jp[11] = -fy * x * zinv;
    for (int r = 0; r < 2; ++r)
        for (int c = 0; c < 3; ++c)
            Jl[r * 3 + c] = Jp[r * 6 + 0] * R[0 * 3 + c] + Jp[r * 6 + 1] * R[1 * 3 + c] + Jp[r * 6 + 2] * R[2 * 3 + c];
}

/* Eigen LDLT (dynamic size, g2o LinearSolverDense: column-wise GEMV subtraction) on a symmetric n x n (lower
 * triangle read), solve in place.  Returns isPositive. */
int or_ldlt_solve(const double* Hin, int n, const double* b, double* x) {
    double* mat = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* temp = (double*)malloc(sizeof(double) * (size_t)n);
    int* tr = (int*)malloc(sizeof(int) * (size_t)n);
    memcpy(mat, Hin, sizeof(double) * (size_t)n * n);
#define L(i, j) mat[(size_t)(i) * n + (j)]
    int sign = 0, found_zero_pivot = 0;
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = fabs(L(k, k));
        for (int i = k + 1; i < n; ++i)
            if (fabs(L(i, i)) > bv) { bv = fabs(L(i, i)); big = i; }
        tr[k] = big;
        if (k != big) {
            const int s = n - big - 1;
            for (int j = 0; j < k; ++j) { double t = L(k, j); L(k, j) = L(big, j); L(big, j) = t; }
            for (int j = 0; j < s; ++j) { double t = L(big + 1 + j, k); L(big + 1 + j, k) = L(big + 1 + j, big); L(big + 1 + j, big) = t; }
            { double t = L(k, k); L(k, k) = L(big, big); L(big, big) = t; }
            for (int i = k + 1; i < big; ++i) { double t = L(i, k); L(i, k) = L(big, i); L(big, i) = t; }
        }
        const int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = L(j, j) * L(k, j);
            double dot = L(k, 0) * temp[0];
            for (int j = 1; j < k; ++j) dot = dot + L(k, j) * temp[j];
            L(k, k) -= dot;
            for (int i = k + 1; i < n; ++i) {
                double acc = L(i, k);
                for (int j = 0; j < k; ++j) acc = acc - L(i, j) * temp[j];
                L(i, k) = acc;
            }
        }
        const double akk = L(k, k);
        const int valid = fabs(akk) > 0;
        if (k == 0 && !valid) {
            sign = 0;
            for (int j = 0; j < n; ++j) tr[j] = j;
            break;
        }
        if (rs > 0 && valid)
            for (int i = k + 1; i < n; ++i) L(i, k) /= akk;
        if (!valid) found_zero_pivot = 1;
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    (void)found_zero_pivot;
    double* v = temp;
    memcpy(v, b, sizeof(double) * (size_t)n);
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
    memcpy(x, v, sizeof(double) * (size_t)n);
    free(mat);
    free(temp);
    free(tr);
    return sign == 1 || sign == 0;
}

/* 3 x 3 inverse: adjugate / determinant (row-major) */
static void inv3(const double* a, double* o) {
    const double c00 = a[4] * a[8] - a[5] * a[7], c01 = a[5] * a[6] - a[3] * a[8], c02 = a[3] * a[7] - a[4] * a[6];
    const double det = a[0] * c00 + a[1] * c01 + a[2] * c02;
    const double id = 1.0 / det;
    o[0] = c00 * id; o[1] = (a[2] * a[7] - a[1] * a[8]) * id; o[2] = (a[1] * a[5] - a[2] * a[4]) * id;
    o[3] = c01 * id; o[4] = (a[0] * a[8] - a[2] * a[6]) * id; o[5] = (a[2] * a[3] - a[0] * a[5]) * id;
    o[6] = c02 * id; o[7] = (a[1] * a[6] - a[0] * a[7]) * id; o[8] = (a[0] * a[4] - a[1] * a[3]) * id;
}

typedef struct {
    int P, L, E, nf;
    const double* K;
    const int32_t* ep;
    const int32_t* el;
    const double* meas;
    /* structure */
    int* pe_off; int* pe;  /* edges per pose (edge order) */
    int* le_off; int* le;  /* edges per landmark (edge order) */
    int* cv_off; int* cv_l; int* cv_e1; int* cv_e2;  /* per pose pair (p1 <= p2, row-major upper): shared landmarks */
} ba_struct;

static void ba_build_struct(ba_struct* s) {
    const int P = s->P, L = s->L, E = s->E;
    s->pe_off = (int*)calloc((size_t)P + 1, sizeof(int));
    s->le_off = (int*)calloc((size_t)L + 1, sizeof(int));
    for (int e = 0; e < E; ++e) { s->pe_off[s->ep[e] + 1]++; s->le_off[s->el[e] + 1]++; }
    for (int p = 0; p < P; ++p) s->pe_off[p + 1] += s->pe_off[p];
    for (int l = 0; l < L; ++l) s->le_off[l + 1] += s->le_off[l];
    s->pe = (int*)malloc(sizeof(int) * (size_t)(E > 0 ? E : 1));
    s->le = (int*)malloc(sizeof(int) * (size_t)(E > 0 ? E : 1));
    int* cp = (int*)calloc((size_t)P, sizeof(int));
    int* cl = (int*)calloc((size_t)L, sizeof(int));
    for (int e = 0; e < E; ++e) {
        s->pe[s->pe_off[s->ep[e]] + cp[s->ep[e]]++] = e;
        s->le[s->le_off[s->el[e]] + cl[s->el[e]]++] = e;
    }
    free(cp);
    free(cl);
    /* co-visibility: pairs (p1 <= p2) x landmarks ascending; for each landmark every ordered pair of its edges */
    const int NB = P * P;
    s->cv_off = (int*)calloc((size_t)NB + 1, sizeof(int));
    for (int l = 0; l < L; ++l)
        for (int a = s->le_off[l]; a < s->le_off[l + 1]; ++a)
            for (int b = s->le_off[l]; b < s->le_off[l + 1]; ++b) {
                const int p1 = s->ep[s->le[a]], p2 = s->ep[s->le[b]];
                if (p1 <= p2) s->cv_off[p1 * P + p2 + 1]++;
            }
    for (int i = 0; i < NB; ++i) s->cv_off[i + 1] += s->cv_off[i];
    const int nc = s->cv_off[NB];
    s->cv_l = (int*)malloc(sizeof(int) * (size_t)(nc > 0 ? nc : 1));
    s->cv_e1 = (int*)malloc(sizeof(int) * (size_t)(nc > 0 ? nc : 1));
    s->cv_e2 = (int*)malloc(sizeof(int) * (size_t)(nc > 0 ? nc : 1));
    int* fill = (int*)calloc((size_t)NB, sizeof(int));
    for (int l = 0; l < L; ++l)
        for (int a = s->le_off[l]; a < s->le_off[l + 1]; ++a)
            for (int b = s->le_off[l]; b < s->le_off[l + 1]; ++b) {
                const int p1 = s->ep[s->le[a]], p2 = s->ep[s->le[b]];
                if (p1 > p2) continue;
                const int k = s->cv_off[p1 * P + p2] + fill[p1 * P + p2]++;
                s->cv_l[k] = l;
                s->cv_e1[k] = s->le[a];
                s->cv_e2[k] = s->le[b];
            }
    free(fill);
}

static void ba_free_struct(ba_struct* s) {
    free(s->pe_off); free(s->pe); free(s->le_off); free(s->le);
    free(s->cv_off); free(s->cv_l); free(s->cv_e1); free(s->cv_e2);
}

/* the halving tree over 256 values: v[t] += v[t + off], off = 128 .. 1 */
static double tree256(double* v) {
    for (int off = 128; off > 0; off >>= 1)
        for (int t = 0; t < off; ++t) v[t] = v[t] + v[t + off];
    return v[0];
}

/* landmark-block order: c[l] per landmark; block b = landmarks [256 b, 256 b + 256) summed as tree256 over its slots
 * (0.0 past L); leaf t = the block totals b = t mod 256 in ascending b (from 0.0); tree256 over the leaves */
static double lblock_total(const double* c, int L) {
    double leaf[256], v[256];
    for (int t = 0; t < 256; ++t) leaf[t] = 0.0;
    for (int b = 0; 256 * b < L; ++b) {
        for (int t = 0; t < 256; ++t) v[t] = 256 * b + t < L ? c[256 * b + t] : 0.0;
        leaf[b % 256] = leaf[b % 256] + tree256(v);
    }
    return tree256(leaf);
}

/* chi2 in the landmark-block order of c[l] = 0.0 + |e|^2 over the landmark's edges (edge order); c: [L] scratch */
static double ba_chi2(const ba_struct* s, const double* poses, const double* X, double* c) {
    for (int l = 0; l < s->L; ++l) {
        double acc = 0.0;
        for (int k = s->le_off[l]; k < s->le_off[l + 1]; ++k) {
            const int e = s->le[k];
            double r[2];
            ba_error(poses + 7 * s->ep[e], s->K, X + 3 * l, s->meas + 2 * e, r);
            acc = acc + (r[0] * r[0] + r[1] * r[1]);
        }
        c[l] = acc;
    }
    return lblock_total(c, s->L);
}

/* diagnostics (tests only): when or_ba_dump_iter >= 0, the first damping trial of that iteration copies its
 * buffers into or_ba_dump[which] (the order of yv_ba_debug_read; S before factorisation) where non-NULL */
int or_ba_dump_iter = -1;
double* or_ba_dump[16];

static void ba_dump(int which, const double* src, size_t n) {
    if (or_ba_dump[which]) memcpy(or_ba_dump[which], src, sizeof(double) * n);
}

/* or_ba_lm: g2o LM with BlockSolver_6_3 (see the header); poses [P][7] (T_cw, SE3d::data()), X [L][3] in / out.
 * chi2_log [max_iters + 1] (may be NULL): chi2 before iteration 0 and after each iteration.  Returns the
 * iterations run (an iteration that fails 10 trials ends the run, as g2o's Terminate). */
/* chi2 in g2o's order: activeRobustChi2, sequential over the edges in edge order from 0.0 */
static double ba_chi2_g2o(const ba_struct* s, const double* poses, const double* X) {
    double chi = 0.0;
    for (int e = 0; e < s->E; ++e) {
        double r[2];
        ba_error(poses + 7 * s->ep[e], s->K, X + 3 * s->el[e], s->meas + 2 * e, r);
        chi = chi + (r[0] * r[0] + r[1] * r[1]);
    }
    return chi;
}

int or_ba_lm(double* poses, int P, int n_fixed, double* X, int L, const int32_t* ep, const int32_t* el,
             const double* meas, int E, const double* K, int max_iters, double* chi2_log) {
    return or_ba_lm_mode(poses, P, n_fixed, X, L, ep, el, meas, E, K, max_iters, chi2_log, 0);
}

int or_ba_lm_mode(double* poses, int P, int n_fixed, double* X, int L, const int32_t* ep, const int32_t* el,
                  const double* meas, int E, const double* K, int max_iters, double* chi2_log, int mode) {
    const int g2o = mode == 1;
    ba_struct s = {P, L, E, n_fixed, K, ep, el, meas, 0, 0, 0, 0, 0, 0, 0, 0};
    ba_build_struct(&s);
    const int np = P - n_fixed, ns = 6 * np;
    double* Jp = (double*)malloc(sizeof(double) * 12 * (size_t)E);
    double* Jl = (double*)malloc(sizeof(double) * 6 * (size_t)E);
    double* err = (double*)malloc(sizeof(double) * 2 * (size_t)E);
    double* Hpl = (double*)malloc(sizeof(double) * 18 * (size_t)E);
    double* W = (double*)malloc(sizeof(double) * 18 * (size_t)E);
    double* Hpp = (double*)malloc(sizeof(double) * 36 * (size_t)P);
    double* bp = (double*)malloc(sizeof(double) * 6 * (size_t)P);
    double* Hll = (double*)malloc(sizeof(double) * 9 * (size_t)L);
    double* bl = (double*)malloc(sizeof(double) * 3 * (size_t)L);
    double* Dinv = (double*)malloc(sizeof(double) * 9 * (size_t)L);
    double* S = (double*)malloc(sizeof(double) * (size_t)ns * ns + 1);
    double* bs = (double*)malloc(sizeof(double) * (size_t)ns + 1);
    double* xp = (double*)malloc(sizeof(double) * (size_t)ns + 1);
    double* xl = (double*)malloc(sizeof(double) * 3 * (size_t)L);
    double* bak_p = (double*)malloc(sizeof(double) * 7 * (size_t)P);
    double* bak_X = (double*)malloc(sizeof(double) * 3 * (size_t)L);
    tree4096* wt = (tree4096*)malloc(sizeof(tree4096));
    double* lsum = (double*)malloc(sizeof(double) * (size_t)(L > 0 ? L : 1));
    double* coef = (double*)malloc(sizeof(double) * (size_t)ns + 1);
    double currentChi = g2o ? ba_chi2_g2o(&s, poses, X) : ba_chi2(&s, poses, X, lsum);
    if (chi2_log) chi2_log[0] = currentChi;
    double lambda = 0, ni = 2;
    int it;
    for (it = 0; it < max_iters; ++it) {
        /* buildSystem at the current estimate */
        for (int e = 0; e < E; ++e) {
            const double* T = poses + 7 * ep[e];
            const double* Xe = X + 3 * el[e];
            ba_error(T, K, Xe, meas + 2 * e, err + 2 * e);
            ba_jacobians(T, K, Xe, Jp + 12 * e, Jl + 6 * e);
            const double* jp = Jp + 12 * e;
            const double* jl = Jl + 6 * e;
            for (int a = 0; a < 6; ++a)
                for (int c = 0; c < 3; ++c) Hpl[18 * e + 3 * a + c] = jp[a] * jl[c] + jp[6 + a] * jl[3 + c];
        }
        for (int p = n_fixed; p < P && g2o; ++p) {
            /* g2o buildSystem: edge by edge in edge order, from 0.0 */
            double h[36], g[6];
            for (int i = 0; i < 36; ++i) h[i] = 0.0;
            for (int a = 0; a < 6; ++a) g[a] = 0.0;
            for (int k = s.pe_off[p]; k < s.pe_off[p + 1]; ++k) {
                const int e = s.pe[k];
                const double* jp = Jp + 12 * e;
                const double o0 = -err[2 * e], o1 = -err[2 * e + 1];
                for (int a = 0; a < 6; ++a) {
                    for (int b = 0; b < 6; ++b) h[6 * a + b] = h[6 * a + b] + (jp[a] * jp[b] + jp[6 + a] * jp[6 + b]);
                    g[a] = g[a] + (jp[a] * o0 + jp[6 + a] * o1);
                }
            }
            memcpy(Hpp + 36 * p, h, sizeof h);
            memcpy(bp + 6 * p, g, sizeof g);
        }
        for (int p = n_fixed; p < P && !g2o; ++p) {
            for (int a = 0; a < 6; ++a)
                for (int b = a; b < 6; ++b) {
                    w_reset(wt);
                    for (int k = s.pe_off[p]; k < s.pe_off[p + 1]; ++k) {
                        const double* jp = Jp + 12 * s.pe[k];
                        w_add(wt, k - s.pe_off[p], jp[a] * jp[b] + jp[6 + a] * jp[6 + b]);
                    }
                    Hpp[36 * p + 6 * a + b] = Hpp[36 * p + 6 * b + a] = w_total(wt);
                }
            for (int a = 0; a < 6; ++a) {
                w_reset(wt);
                for (int k = s.pe_off[p]; k < s.pe_off[p + 1]; ++k) {
                    const int e = s.pe[k];
                    const double* jp = Jp + 12 * e;
                    w_add(wt, k - s.pe_off[p], jp[a] * err[2 * e] + jp[6 + a] * err[2 * e + 1]);
                }
                bp[6 * p + a] = -w_total(wt);
            }
        }
        for (int l = 0; l < L; ++l) {
            double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
            for (int k = s.le_off[l]; k < s.le_off[l + 1]; ++k) {
                const int e = s.le[k];
                const double* jl = Jl + 6 * e;
                for (int a = 0; a < 3; ++a) {
                    for (int b = a; b < 3; ++b) h[3 * a + b] = h[3 * a + b] + (jl[a] * jl[b] + jl[3 + a] * jl[3 + b]);
                    g[a] = g[a] + (jl[a] * err[2 * e] + jl[3 + a] * err[2 * e + 1]);
                }
            }
            for (int a = 0; a < 3; ++a) {
                for (int b = a; b < 3; ++b) Hll[9 * l + 3 * a + b] = Hll[9 * l + 3 * b + a] = h[3 * a + b];
                bl[3 * l + a] = -g[a];
            }
        }
        if (it == 0) {
            double maxd = 0;
            for (int p = n_fixed; p < P; ++p)
                for (int a = 0; a < 6; ++a) maxd = fmax(maxd, fabs(Hpp[36 * p + 7 * a]));
            for (int l = 0; l < L; ++l)
                for (int a = 0; a < 3; ++a) maxd = fmax(maxd, fabs(Hll[9 * l + 4 * a]));
            lambda = 1e-5 * maxd;
            ni = 2;
        }
        double rho = 0;
        int q = 0;
        do {
            memcpy(bak_p, poses, sizeof(double) * 7 * (size_t)P);
            memcpy(bak_X, X, sizeof(double) * 3 * (size_t)L);
            /* landmark blocks with lambda: Dinv, W_e = H_pl Dinv */
            for (int l = 0; l < L; ++l) {
                double d[9];
                memcpy(d, Hll + 9 * l, sizeof d);
                for (int a = 0; a < 3; ++a) d[4 * a] = d[4 * a] + lambda;
                inv3(d, Dinv + 9 * l);
                for (int k = s.le_off[l]; k < s.le_off[l + 1]; ++k) {
                    const int e = s.le[k];
                    for (int a = 0; a < 6; ++a)
                        for (int c = 0; c < 3; ++c)
                            W[18 * e + 3 * a + c] = Hpl[18 * e + 3 * a + 0] * Dinv[9 * l + 0 * 3 + c] +
                                                    Hpl[18 * e + 3 * a + 1] * Dinv[9 * l + 1 * 3 + c] +
                                                    Hpl[18 * e + 3 * a + 2] * Dinv[9 * l + 2 * 3 + c];
                }
            }
            /* Schur: S(p1, p2) = [p1 == p2] (H_pp + lambda I) - sum_l W_e1 H_pl(e2)^T ; upper blocks, mirrored */
            for (int p1 = n_fixed; p1 < P && g2o; ++p1)
                for (int p2 = p1; p2 < P; ++p2)
                    for (int a = 0; a < 6; ++a)
                        for (int b = 0; b < 6; ++b) {
                            /* g2o solve(): the block starts at H_pp + lambda I (or 0); each co-visible landmark,
                             * ascending, subtracts its term */
                            double v = p1 == p2 ? Hpp[36 * p1 + 6 * a + b] + (a == b ? lambda : 0.0) : 0.0;
                            for (int k = s.cv_off[p1 * P + p2]; k < s.cv_off[p1 * P + p2 + 1]; ++k) {
                                const double* w = W + 18 * s.cv_e1[k] + 3 * a;
                                const double* h = Hpl + 18 * s.cv_e2[k] + 3 * b;
                                v = v - (w[0] * h[0] + w[1] * h[1] + w[2] * h[2]);
                            }
                            const int r = 6 * (p1 - n_fixed) + a, c = 6 * (p2 - n_fixed) + b;
                            /* LinearSolverDense: H.block(r, c) = block, then H.block(c, r) = block^T -- a diagonal
                             * block ends up transposed */
                            if (p1 != p2) S[(size_t)r * ns + c] = v;
                            S[(size_t)c * ns + r] = v;
                        }
            for (int p1 = n_fixed; p1 < P && !g2o; ++p1)
                for (int p2 = p1; p2 < P; ++p2)
                    for (int a = 0; a < 6; ++a)
                        for (int b = 0; b < 6; ++b) {
                            const double base = p1 == p2 ? Hpp[36 * p1 + 6 * a + b] + (a == b ? lambda : 0.0) : 0.0;
                            const int k0 = s.cv_off[p1 * P + p2];
                            w_reset(wt);
                            for (int k = k0; k < s.cv_off[p1 * P + p2 + 1]; ++k) {
                                const double* w = W + 18 * s.cv_e1[k] + 3 * a;
                                const double* h = Hpl + 18 * s.cv_e2[k] + 3 * b;
                                w_add(wt, k - k0, w[0] * h[0] + w[1] * h[1] + w[2] * h[2]);
                            }
                            const double v = base - w_total(wt);
                            const int r = 6 * (p1 - n_fixed) + a, c = 6 * (p2 - n_fixed) + b;
                            S[(size_t)r * ns + c] = v;
                            S[(size_t)c * ns + r] = v;
                        }
            if (g2o) {
                /* coefficients += B_i (Dinv b_l), landmark by landmark; b_schur = b_p - coefficients */
                for (int i = 0; i < ns; ++i) coef[i] = 0.0;
                for (int l = 0; l < L; ++l) {
                    const double* D = Dinv + 9 * l;
                    const double* g = bl + 3 * l;
                    double db[3];
                    for (int c = 0; c < 3; ++c) db[c] = D[3 * c] * g[0] + D[3 * c + 1] * g[1] + D[3 * c + 2] * g[2];
                    for (int k = s.le_off[l]; k < s.le_off[l + 1]; ++k) {
                        const int e = s.le[k], p = ep[e];
                        if (p < n_fixed) continue;
                        const double* h = Hpl + 18 * e;
                        for (int a = 0; a < 6; ++a)
                            coef[6 * (p - n_fixed) + a] = coef[6 * (p - n_fixed) + a] +
                                                          (h[3 * a] * db[0] + h[3 * a + 1] * db[1] + h[3 * a + 2] * db[2]);
                    }
                }
                for (int p = n_fixed; p < P; ++p)
                    for (int a = 0; a < 6; ++a) bs[6 * (p - n_fixed) + a] = bp[6 * p + a] - coef[6 * (p - n_fixed) + a];
            }
            for (int p = n_fixed; p < P && !g2o; ++p)
                for (int a = 0; a < 6; ++a) {
                    w_reset(wt);
                    for (int k = s.pe_off[p]; k < s.pe_off[p + 1]; ++k) {
                        const int e = s.pe[k];
                        const double* w = W + 18 * e + 3 * a;
                        const double* g = bl + 3 * el[e];
                        w_add(wt, k - s.pe_off[p], w[0] * g[0] + w[1] * g[1] + w[2] * g[2]);
                    }
                    bs[6 * (p - n_fixed) + a] = bp[6 * p + a] - w_total(wt);
                }
            const int ok2 = ns > 0 ? or_ldlt_solve(S, ns, bs, xp) : 1;
            const int dump = it == or_ba_dump_iter && q == 0;
            if (dump) {
                ba_dump(0, err, 2 * (size_t)E); ba_dump(1, Jp, 12 * (size_t)E); ba_dump(2, Jl, 6 * (size_t)E);
                ba_dump(3, Hpl, 18 * (size_t)E); ba_dump(4, W, 18 * (size_t)E); ba_dump(5, Hpp, 36 * (size_t)P);
                ba_dump(6, bp, 6 * (size_t)P); ba_dump(7, Hll, 9 * (size_t)L); ba_dump(8, bl, 3 * (size_t)L);
                ba_dump(9, Dinv, 9 * (size_t)L); ba_dump(10, S, (size_t)ns * ns); ba_dump(11, bs, (size_t)ns);
                ba_dump(12, xp, (size_t)ns);
            }
            /* landmarks: x_l = Dinv (b_l - sum_e H_pl(e)^T x_p(e)) */
            for (int l = 0; l < L; ++l) {
                double t[3] = {bl[3 * l], bl[3 * l + 1], bl[3 * l + 2]};
                const int k0 = s.le_off[l], k1 = s.le_off[l + 1];
                for (int kk = k0; kk < k1; ++kk) {
                    int k = kk;
                    if (g2o) {
                        /* rightMultiply walks the landmark's column in pose order: the (kk - k0)-th smallest pose
                         * (ties in edge order) */
                        int best = -1;
                        for (int j = k0; j < k1; ++j) {
                            int rank = 0;
                            for (int i = k0; i < k1; ++i)
                                rank += ep[s.le[i]] < ep[s.le[j]] || (ep[s.le[i]] == ep[s.le[j]] && i < j);
                            if (rank == kk - k0) best = j;
                        }
                        k = best;
                    }
                    const int e = s.le[k], p = ep[e];
                    if (p < n_fixed) continue;
                    const double* xpp = xp + 6 * (p - n_fixed);
                    for (int c = 0; c < 3; ++c) {
                        double d = Hpl[18 * e + c] * xpp[0];
                        for (int a = 1; a < 6; ++a) d = d + Hpl[18 * e + 3 * a + c] * xpp[a];
                        t[c] = t[c] - d;
                    }
                }
                const double* D = Dinv + 9 * l;
                for (int c = 0; c < 3; ++c) xl[3 * l + c] = D[3 * c] * t[0] + D[3 * c + 1] * t[1] + D[3 * c + 2] * t[2];
            }
            /* update */
            for (int p = n_fixed; p < P; ++p) {
                double dT[7], Tn[7];
                or_se3_exp(xp + 6 * (p - n_fixed), dT);
                or_se3_mul(dT, poses + 7 * p, Tn);
                memcpy(poses + 7 * p, Tn, sizeof Tn);
            }
            for (int i = 0; i < 3 * L; ++i) X[i] = X[i] + xl[i];
            if (dump) {
                ba_dump(13, xl, 3 * (size_t)L); ba_dump(14, poses, 7 * (size_t)P); ba_dump(15, X, 3 * (size_t)L);
            }
            double tempChi = g2o ? ba_chi2_g2o(&s, poses, X) : ba_chi2(&s, poses, X, lsum);
            if (!ok2) tempChi = DBL_MAX;
            rho = currentChi - tempChi;
            /* computeScale over the variables: the free poses' items in tree256 order (leaf t = items j = t mod 256
             * ascending from 0.0), plus the landmarks' in the landmark-block order of 0.0 + their three items */
            double scale;
            if (g2o) {
                scale = 0.0;  /* computeScale: x = [x_p; x_l] in vector order */
                for (int j = 0; j < ns; ++j) scale += xp[j] * (lambda * xp[j] + bp[6 * n_fixed + j]);
                for (int i = 0; i < 3 * L; ++i) scale += xl[i] * (lambda * xl[i] + bl[i]);
            } else {
            double leaf[256];
            for (int t = 0; t < 256; ++t) leaf[t] = 0.0;
            for (int j = 0; j < ns; ++j) leaf[j % 256] = leaf[j % 256] + xp[j] * (lambda * xp[j] + bp[6 * n_fixed + j]);
            const double pose_part = tree256(leaf);
            for (int l = 0; l < L; ++l) {
                double acc = 0.0;
                for (int c = 0; c < 3; ++c) acc = acc + xl[3 * l + c] * (lambda * xl[3 * l + c] + bl[3 * l + c]);
                lsum[l] = acc;
            }
            scale = pose_part + lblock_total(lsum, L);
            }
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && isfinite(tempChi)) {
                double alpha = 1. - or_lm_cube(2 * rho - 1);  /* pow(2 rho - 1, 3): correctly rounded, or libm */
                alpha = fmin(alpha, 2. / 3.);
                const double sf = fmax(1. / 3., alpha);
                lambda *= sf;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                memcpy(poses, bak_p, sizeof(double) * 7 * (size_t)P);
                memcpy(X, bak_X, sizeof(double) * 3 * (size_t)L);
            }
            q++;
        } while (rho < 0 && q < 10);
        if (chi2_log) chi2_log[it + 1] = currentChi;
        if (q == 10 || rho == 0 || !isfinite(lambda)) {
            ++it;
            break;
        }
    }
    free(Jp); free(Jl); free(err); free(Hpl); free(W); free(Hpp); free(bp); free(Hll); free(bl); free(Dinv);
    free(S); free(bs); free(xp); free(xl); free(bak_p); free(bak_X); free(wt); free(lsum); free(coef);
    ba_free_struct(&s);
    return it;
}
