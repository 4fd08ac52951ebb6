/*
 * yavo_oracle.h -- CPU restatement of the YA_VO per-frame hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP path: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product library
 * (ya_vo_amd/lib/libyavo.so) never links, calls or falls back to it.
 *
 * Every function restates the reference's arithmetic literally (file:line cited at each definition in
 * yavo_oracle.c / yavo_oracle_geom.c).  The reference itself cannot be compiled here (OpenCV, Eigen,
 * Sophus, g2o, jsoncpp, Boost, Pangolin absent), so the third-party arithmetic it calls
 * (cv::eigen, cv::GaussianBlur, cv::SVD, Eigen JacobiSVD/LDLT, Sophus exp, g2o LM) is restated from the
 * published algorithms and named per function.  Pinned by: the reference's ring fixture
 * (tests/testBresenham.png), the contiguity tests (tests/FastDetectorTest.cc:38-80) and the calib parser
 * test (tests/UtilsTest.cc:4-15).  Everything past the FAST candidate test is "parity unpinned" against
 * the real reference binary (no fixtures exist for it); see DESIGN.md.
 */
#ifndef YAVO_ORACLE_H
#define YAVO_ORACLE_H

#include <math.h>
#include <stdint.h>
#include "../include/yavo/yavo_types.h"

/* pow(t, 3) of g2o's Levenberg-Marquardt step scaling (OptimizationAlgorithmLevenberg::solve: alpha = 1 -
 * pow(2 rho - 1, 3)) correctly rounded: t^2 = p + e1 and p t = q + e2 exactly (fma), t^3 = q + (e2 + e1 t) rounded
 * once.  glibc's pow (< 0.52 ulp) returns the same double in all but ~0.09% of arguments; t * t * t (two roundings)
 * differs in ~26%.  Both LMs (pose-only and the window BA) and their GPU kernels use this function. */
static inline double or_cube(double t) {
    const double p = t * t, e1 = fma(t, t, -p);
    const double q = p * t, e2 = fma(p, t, -q);
    return q + (e2 + e1 * t);
}

/* libm flavour of the oracle's geometry (or_set_libm_flavour): 0 (default) = the restated functions the GPU kernels
 * share (or_cube above for g2o's pow(2 rho - 1, 3); fdlibm's __kernel_sin / __kernel_cos in Sophus' SO3::exp);
 * 1 = the host C library's pow / sin / cos, as g2o (OptimizationAlgorithmLevenberg::solve) and Sophus (std::sin /
 * std::cos) call them in the reference's build.  Flavour 1 measures what the substitution moves. */
extern int or_libm_flavour;
void or_set_libm_flavour(int flavour);
void or_cube_batch(const double* t, int n, int flavour, double* out);
static inline double or_lm_cube(double t) { return or_libm_flavour ? pow(t, 3) : or_cube(t); }

#ifdef __cplusplus
extern "C" {
#endif

/* ---- FAST ring / candidate test (src/FastDetector.cc) ---- */
/* Literal Bresenham ring with the reference's two std::set orderings (src/FastDetector.cc:50-112).
 * out[k][0] = row, out[k][1] = col (absolute), k = 0..15. */
void or_bresenham_ring(int xc, int yc, int out[16][2]);
/* The same ring built with the reference's std::vector / std::set containers (yavo_oracle_sort.cc): the literal
 * CPU baseline's per-pixel cost. */
void or_bresenham_ring_stl(int xc, int yc, int out[16][2]);
/* checkContiguousPixels (src/FastDetector.cc:135-153) with checkInBetween (:155-161). */
int or_check_contiguous(uint8_t cent, const int ring[16][2], const uint8_t* img, int stride, int thr);

/* getFastFeatures (src/FastDetector.cc:277-369).  mode 0 = literal costs (per-pixel ring rebuild, three
 * full-image products per corner); mode 1 = same outputs, local arithmetic.  Writes up to max_kp
 * (row, col) pairs + responses in output order, *n = count, *n_cand = corners before the cut.
 * cand_idx/cand_resp (optional, may be NULL, capacity cand_cap) receive the unsorted candidate list in
 * scan order. */
int or_fast_detect(const uint8_t* img, int H, int W, int stride, int thr, int max_kp, int mode,
                   int32_t* rc, float* resp, int* n, int* n_cand,
                   int32_t* cand_idx, float* cand_resp, int cand_cap);

/* Harris response from the 3x3-summed structure tensor (src/FastDetector.cc:244-273). */
float or_harris_response(float m00, float m01, float m11);
/* OpenCV JacobiImpl_<float> eigenvalues (descending), the cv::eigen path without HAVE_EIGEN. */
void or_eigen_jacobi_f32(const float* A, int n, float* w);
/* cv::eigen with HAVE_EIGEN: Eigen 3.4 SelfAdjointEigenSolver<MatrixXf> on [m00 m01; m01 m11], descending. */
void or_eigen_selfadjoint2_f32(float m00, float m01, float m11, float* w);
/* the cv::eigen flavour of or_harris_response: 0 = JacobiImpl_ (default), 1 = HAVE_EIGEN */
void or_set_harris_eigen(int flavour);

/* ---- Gaussian blur (cv::GaussianBlur(img, out, Size(9,9), 2.5, 2.5): src/BriefDescriptor.cc:90) ---- */
/* Bit-exact 8U fixed-point kernel: error-diffusion rounding (ed=1, OpenCV >= 3.4 bit-exact path) or
 * plain rounding (ed=0).  out has n entries summing to 256. */
void or_gauss_kernel_fixed(int n, double sigma, int ed, uint16_t* out);
/* Separable 8U fixed-point blur with BORDER_REFLECT_101; out is H x W contiguous. */
void or_gaussian_blur_u8(const uint8_t* img, int H, int W, int stride, const uint16_t* k, int n,
                         uint8_t* out);

/* ---- BRIEF (src/BriefDescriptor.cc) ---- */
/* Brief::computeBrief (:86-124) on an already blurred H x W contiguous image.  offsets: 256 x 4 int8
 * (o0=drow1, o1=dcol1, o2=drow2, o3=dcol2).  Reads past the buffer end return 0 (reference: UB). */
int or_compute_brief_blurred(const uint8_t* blur, int H, int W, const int8_t* offsets,
                             const int32_t* rc, int n, yv_keypoint* out, int* n_out);
/* Blur + describe, i.e. the whole computeBrief call. */
int or_compute_brief(const uint8_t* img, int H, int W, int stride, const uint16_t* k9,
                     const int8_t* offsets, const int32_t* rc, int n, yv_keypoint* out, int* n_out);
/* Brief::preComputeOffsets (:4-20) with an explicit seed instead of std::random_device:
 * std::mt19937(seed) + uniform_int_distribution<int>(-8, 8) (libstdc++ algorithm). */
void or_brief_offsets_mt19937(uint32_t seed, int8_t* out /* 1024 */);
/* a persistent std::mt19937(seed); or_mt19937_uniform_ints draws `count` uniform_int_distribution<int>(a, b) values */
void* or_mt19937_new(uint32_t seed);
void or_mt19937_uniform_ints(void* g, int a, int b, int count, int32_t* out);
void or_mt19937_free(void* g);

/* Brief::popCount (:151-160) / hammingDistance (:139-146). */
int or_hamming(const uint8_t* a, const uint8_t* b);
/* Brief::matchFeatures (:163-183).  out has nq records. */
int or_match(const yv_keypoint* q, int nq, const yv_keypoint* t, int nt, yv_match* out);
/* Brief::removeOutliers (:213-231). */
int or_remove_outliers(const yv_match* in, int n, int thr, yv_match* out, int* n_out);

/* ---- utils ---- */
/* parseCalibString (src/Utils.cc:4-28): reads the numbers after the "Pn:" tag into a row-major
 * 4x4 (missing values -> 0; the reference reads past a 12-value vector). returns #values parsed. */
int or_parse_calib_string(const char* s, double out[16]);

/* ---- geometry (yavo_oracle_geom.c) ---- */
/* Poses are Sophus::SE3d::data(): {qx, qy, qz, qw, tx, ty, tz} (T_cw).  K is row-major 3x3. */
/* OpenCV JacobiSVDImpl_<double> on At (n rows of m), as cv::SVD calls it. */
void or_cv_jacobi_svd(double* At, int astep, double* W, double* Vt, int vstep, int m, int n, int n1);
/* cv::SVD(src, FULL_UV) for square row-major n x n (n <= 9). */
void or_cv_svd(const double* src, int n, double* w, double* u, double* vt);
/* _3DHandler::getFundamentalMatrix (src/3DHandler.cc:50-142); pts [n][4] = (x1, y1, x2, y2). */
int or_fundamental_8pt(const double* pts, int n, double F[9]);
/* _3DHandler::getFRANSAC (src/3DHandler.cc:145-195) with explicit samples [iters][8]. */
int or_f_ransac(const yv_match* m, int n, const int32_t* sample_idx, int iters, double thr, double F[9],
                int* max_inliers);
/* Eigen JacobiSVD (square, column-major): sv descending, V column-major. */
int or_eigen_jacobi_svd(const double* A, int n, double* sv, double* V);
/* LoopHandler::triangulation (src/LoopHandler.cc:867-885) for two poses and normalised points. */
int or_triangulate_one(const double* Ta, const double* Tb, const double* pa, const double* pb, double* Xw);
/* triangulate2View's per-match part (src/LoopHandler.cc:665-676): returns #ok. */
int or_triangulate_matches(const double* Ta, const double* Tb, const double* K, const yv_match* m, int n,
                           double* Xw, uint8_t* ok);
/* Sophus pieces */
void or_se3_exp(const double* a, double* out);
void or_se3_mul(const double* A, const double* B, double* out);
void or_se3_act(const double* T, const double* p, double* out);
void or_se3_inverse(const double* T, double* out);
void or_se3_from_Rt(const double* R, const double* t, double* out);
void or_quat_to_R(const double* q, double* R);
double or_ksin(double x);
double or_kcos(double x);
/* Frame::world2Camera (src/Frame.cc:16-28): out [n][3] = K [R|t] [X; 1]. */
void or_world2camera(const double* X, int n, const double* T, const double* K, double* out);
/* Eigen LDLT solve of a 6x6 (variant 0: MatrixXd / g2o, 1: Matrix6d / test.cc). Returns isPositive. */
int or_ldlt6_solve(const double* H, const double* b, double* x, int variant);
/* LoopHandler::optimizePoseOnly (src/LoopHandler.cc:730-861); returns inliers.  sum_mode 0 = sequential
 * edge sums (reference), 1 = 256-thread tree (GN kernel), 2 / 3 = 512- / 256-thread segmented (earlier LM
 * kernels), 4 / 5 / 6 / 7 = 64- / 128- / 256- / 512-thread wave trees (the LM kernel: yv_lm_sum_mode(),
 * yv_pose_lm_sum_mode(n)). */
int or_pose_lm(const double* X, const double* uv, int n, const double* K, double* pose, uint8_t* outlier,
               int sum_mode);
/* bundleAdjustmentGaussNewton (src/test.cc:172-244); returns accepted iterations (GPU order: sum_mode 1). */
/* Pose-LM diagnostics: {builds, trials, accepted trials} since the last reset. */
void or_lm_stats(long* out, int reset);
int or_pose_gn(const double* X, const double* uv, int n, const double* K, double* pose, int sum_mode);

/* ---- cv::calcOpticalFlowPyrLK (yavo_oracle_lk.c) ---- */
/* cv::pyrDown, CV_8U, BORDER_REFLECT_101: dst [(H+1)/2][(W+1)/2]. */
void or_pyr_down(const uint8_t* src, int H, int W, int sstride, uint8_t* dst);
/* calcSharrDeriv: d [H][W][2] = (dx, dy) int16. */
void or_scharr(const uint8_t* src, int H, int W, int sstride, int16_t* d);
/* calcOpticalFlowPyrLK with flags 0 (src/LoopHandler.cc:372-375).  pts (x = col, y = row) float pairs.
 * sum_mode 0 = OpenCV's scalar window-sum order, 1 = the GPU kernel's.  Returns the top level used. */
int or_lk_pyr(const uint8_t* prev, const uint8_t* next, int H, int W, const float* prev_pts, int n, int win,
              int max_level, int max_count, double eps, double min_eig, float* next_pts, uint8_t* status,
              float* err, int sum_mode);

/* ---- cv::findEssentialMat (RANSAC) + cv::recoverPose (yavo_oracle_essential.c) ---- */
/* getSubset draws of RANSACPointSetRegistrator::run (cv::RNG((uint64)-1)): idx [iters][5] */
void or_em_subsets(int count, int iters, int32_t* idx);
/* the 10 x 20 cubic-constraint matrix from the null-space basis EE [4][9] */
void or_em_coeff_mat(const double* EE, double* A);
/* det B(z) of the 3 x 13 elimination matrix -> c[0..10] ascending */
void or_em_det_poly(const double* B, double* c);
/* cv::solvePoly (Durand-Kerner) on real c[0..n0] ascending; roots [n0][2] (re, im); returns iterations run */
int or_solve_poly(const double* c, int n0, int max_iters, double* roots);
/* EMEstimatorCallback::runKernel on 5 normalised correspondences; models [10][9]; returns the model count */
int or_em_kernel(const double* q1, const double* q2, double* models);
/* (p - c) / f as OpenCV's MatExpr evaluates it */
void or_normalize_points(const double* pts, int n, double fx, double fy, double cx, double cy, double* out);
/* findEssentialMat(pts1, pts2, focal, (ppx, ppy), RANSAC, prob, threshold, mask) with maxIters; pts [n][2] pixels.
 * stats (optional) = {iterations run, models scored, best inlier count}.  Returns 1 when E was found. */
int or_find_essential(const double* pts1, const double* pts2, int n, double focal, double ppx, double ppy, double prob,
                      double threshold, int max_iters, double E[9], uint8_t* mask, int* stats);
/* decomposeEssentialMat */
void or_decompose_essential(const double E[9], double R1[9], double R2[9], double t[3]);
/* recoverPose(E, pts1, pts2, K, R, t) (distanceThresh 50, no input mask); good[4] per candidate; returns the count */
int or_recover_pose(const double E[9], const double* pts1, const double* pts2, int n, const double K[9], double R[9],
                    double t[3], int good[4]);

/* ---- sliding-window bundle adjustment (BASELINE config 5; yavo_oracle_ba.c) ---- */
/* Eigen LDLT (dynamic, g2o LinearSolverDense) on a symmetric n x n; returns isPositive */
int or_ldlt_solve(const double* H, int n, const double* b, double* x);
/* g2o LM + BlockSolver_6_3 (Schur) over P poses (first n_fixed fixed) and L landmarks with E pose-landmark
 * edges (pose ep[e], landmark el[e], measurement meas[e][2] in the reference's (row, col) convention).
 * poses [P][7] / X [L][3] in / out; chi2_log [max_iters + 1] optional.  Returns the iterations run. */
int or_ba_lm(double* poses, int P, int n_fixed, double* X, int L, const int32_t* ep, const int32_t* el,
             const double* meas, int E, const double* K, int max_iters, double* chi2_log);
/* mode 0 = the kernel order above (bit-exact with yavo_ba.hip); mode 1 = g2o's own loop orders as sequential chains
 * (yavo_oracle_ba.c header): the order the trajectory tolerance is measured against */
int or_ba_lm_mode(double* poses, int P, int n_fixed, double* X, int L, const int32_t* ep, const int32_t* el,
                  const double* meas, int E, const double* K, int max_iters, double* chi2_log, int mode);
extern int or_ba_dump_iter;
extern double* or_ba_dump[16];

/* ---- shared map blocks (include/yavo/yavo_map.h; src/Map.cc:9-40) -- yavo_oracle_map.c ---- */
int64_t or_map_block_bytes(int max_kf, int lm_stride);
void or_map_chunk(const double* rel, int n, int64_t first_frame, int kf_every, const int32_t* edge_count,
                  const double* edge_X, const uint8_t* edge_outlier, int max_kp, int max_kf, void* block);
void or_map_place(void* blocks, int world, int64_t bb, double* base, double* anchors);

#ifdef __cplusplus
}
#endif
#endif
