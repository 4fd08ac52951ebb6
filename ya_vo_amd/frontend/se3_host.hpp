// se3_host.hpp -- the Sophus SE3d operations LoopHandler composes on the host (pose = SE3d::data() =
// {qx, qy, qz, qw, tx, ty, tz}, T_cw as the reference stores Frame::pose).  Every expression is the one the
// device kernels (ya_vo_amd/csrc/yavo_se3.h) and the oracle (oracle/yavo_oracle_geom.c: or_se3_*) evaluate, and
// this file is compiled with -ffp-contract=off, so host poses are bit-identical to the oracle loop's.
#pragma once

#include <cmath>

namespace yavo_fe {

struct SE3 {
    double d[7] = {0, 0, 0, 1, 0, 0, 0};  // identity: Sophus::SE3d()
};

namespace se3 {

// Eigen Quaternion::_transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv
inline void rotate(const double* q, const double* v, double* out) {
    double uv0 = q[1] * v[2] - q[2] * v[1];
    double uv1 = q[2] * v[0] - q[0] * v[2];
    double uv2 = q[0] * v[1] - q[1] * v[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    const double c0 = q[1] * uv2 - q[2] * uv1;
    const double c1 = q[2] * uv0 - q[0] * uv2;
    const double c2 = q[0] * uv1 - q[1] * uv0;
    out[0] = v[0] + q[3] * uv0 + c0;
    out[1] = v[1] + q[3] * uv1 + c1;
    out[2] = v[2] + q[3] * uv2 + c2;
}

// SE3d * SE3d: t = tA + qA tB; q = qA qB renormalised by 2 / (1 + |q|^2) when |q|^2 != 1 (SO3::operator*=)
inline SE3 mul(const SE3& A, const SE3& B) {
    const double* a = A.d;
    const double* b = B.d;
    double r[3];
    rotate(a, b + 4, r);
    SE3 o;
    const double t0 = a[4] + r[0], t1 = a[5] + r[1], t2 = a[6] + r[2];
    const double ax = a[0], ay = a[1], az = a[2], aw = a[3], bx = b[0], by = b[1], bz = b[2], bw = b[3];
    double q[4];
    q[3] = aw * bw - ax * bx - ay * by - az * bz;
    q[0] = aw * bx + ax * bw + ay * bz - az * by;
    q[1] = aw * by + ay * bw + az * bx - ax * bz;
    q[2] = aw * bz + az * bw + ax * by - ay * bx;
    const double sn = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    if (sn != 1.0) {
        const double sc = 2.0 / (1.0 + sn);
        for (int i = 0; i < 4; ++i) q[i] *= sc;
    }
    for (int i = 0; i < 4; ++i) o.d[i] = q[i];
    o.d[4] = t0; o.d[5] = t1; o.d[6] = t2;
    return o;
}

// SE3d::inverse: invR = SO3(q.conjugate()) (normalised by |q|, Eigen's packet order (x^2 + z^2) + (y^2 + w^2)),
// t' = invR * (t * -1)
inline SE3 inverse(const SE3& T) {
    double q[4] = {-T.d[0], -T.d[1], -T.d[2], T.d[3]};
    const double len = std::sqrt((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
    for (int i = 0; i < 4; ++i) q[i] = q[i] / len;
    const double mt[3] = {T.d[4] * -1.0, T.d[5] * -1.0, T.d[6] * -1.0};
    double r[3];
    rotate(q, mt, r);
    SE3 o;
    for (int i = 0; i < 4; ++i) o.d[i] = q[i];
    o.d[4] = r[0]; o.d[5] = r[1]; o.d[6] = r[2];
    return o;
}

// SE3d(Matrix3d R, Vector3d t): Eigen's Quaternion from a rotation matrix (quaternion_assign_impl<3,3>), R row-major
inline SE3 from_Rt(const double* R, const double* t) {
    auto M = [R](int i, int j) { return R[3 * i + j]; };
    double q[4];  // x, y, z, w
    double tr = (M(0, 0) + M(1, 1)) + M(2, 2);
    if (tr > 0.0) {
        tr = std::sqrt(tr + 1.0);
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
        tr = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        q[i] = 0.5 * tr;
        tr = 0.5 / tr;
        q[3] = (M(k, j) - M(j, k)) * tr;
        q[j] = (M(j, i) + M(i, j)) * tr;
        q[k] = (M(k, i) + M(i, k)) * tr;
    }
    SE3 o;
    for (int i = 0; i < 4; ++i) o.d[i] = q[i];
    o.d[4] = t[0]; o.d[5] = t[1]; o.d[6] = t[2];
    return o;
}

}  // namespace se3
}  // namespace yavo_fe
