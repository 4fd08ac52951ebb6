// yavo_se3.h -- device restatements of the Sophus SE3d operations the geometry kernels share (pose = SE3d::data()
// = {qx, qy, qz, qw, tx, ty, tz}): Eigen quaternion product / rotation / toRotationMatrix, SE3 act / mul (with
// Sophus' renormalisation) and SE3::exp with fdlibm's sin / cos kernels (oracle/yavo_oracle_geom.c: or_se3_*).
// Every expression in the oracle's order; files are built with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

namespace yavo {
namespace se3 {

// 3 x 3 product, sequential dot products (OpenCV small-matrix gemm)
__device__ __forceinline__ void mm3(const double* A, const double* B, double* C) {
    double R[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) R[i * 3 + j] = A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j] + A[i * 3 + 2] * B[2 * 3 + j];
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = R[i];
}

// the library's full-range sin / cos (Payne-Hanek reduction and all): rare (|x| > pi/4), and register-hungry, so kept
// out of line -- inlined into the pose LM's lane-0 step they set the whole kernel's register peak
__device__ __noinline__ double k_sin_full(double x) { return sin(x); }
__device__ __noinline__ double k_cos_full(double x) { return cos(x); }

__device__ __forceinline__ double k_sin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    if (!(fabs(x) <= 0.78539816339744827900)) return k_sin_full(x);
    double z = x * x, v = z * x;
    double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}

__device__ __forceinline__ double k_cos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    if (!(fabs(x) <= 0.78539816339744827900)) return k_cos_full(x);
    double z = x * x;
    double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * 0.0));
}

__device__ __forceinline__ void quat_mul(const double* a, const double* b, double* r) {
    double ax = a[0], ay = a[1], az = a[2], aw = a[3], bx = b[0], by = b[1], bz = b[2], bw = b[3];
    r[3] = aw * bw - ax * bx - ay * by - az * bz;
    r[0] = aw * bx + ax * bw + ay * bz - az * by;
    r[1] = aw * by + ay * bw + az * bx - ax * bz;
    r[2] = aw * bz + az * bw + ax * by - ay * bx;
}

__device__ __forceinline__ void quat_rotate(const double* q, const double* v, double* out) {
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

__device__ __forceinline__ void quat_to_R(const double* q, double* R) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

__device__ __forceinline__ void se3_act(const double* T, const double* p, double* out) {
    double r[3];
    quat_rotate(T, p, r);
    out[0] = r[0] + T[4];
    out[1] = r[1] + T[5];
    out[2] = r[2] + T[6];
}

__device__ __forceinline__ void se3_mul(const double* A, const double* B, double* out) {
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

__device__ void se3_exp(const double* a, double* out) {
    const double* om = a + 3;
    const double eps = 1e-10;
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
    double O[9] = {0, -om[2], om[1], om[2], 0, -om[0], -om[1], om[0], 0};
    double O2[9];
    mm3(O, O, O2);
    double V[9];
    if (theta < eps) {
        quat_to_R(q, V);
    } else {
        double theta_sq2 = theta * theta;
        double a1 = (1 - k_cos(theta)) / theta_sq2;
        double a2 = (theta - k_sin(theta)) / (theta_sq2 * theta);
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.0 : 0.0) + a1 * O[i] + a2 * O2[i];
    }
    out[0] = q[0]; out[1] = q[1]; out[2] = q[2]; out[3] = q[3];
    for (int i = 0; i < 3; ++i) out[4 + i] = V[3 * i] * a[0] + V[3 * i + 1] * a[1] + V[3 * i + 2] * a[2];
}

}  // namespace se3
}  // namespace yavo
