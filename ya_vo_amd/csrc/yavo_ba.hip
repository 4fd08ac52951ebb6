// yavo_ba.hip -- gfx950 kernels for the sliding-window bundle adjustment (BASELINE.json config 5):
// g2o's Levenberg-Marquardt over BlockSolver_6_3 with the reference's projection edge (include/Optimizer.hpp:64-126)
// extended to pose-landmark edges, restated like oracle/yavo_oracle_ba.c, expression for expression, in its
// summation orders (built with -ffp-contract=off):
//
//   ba_reduce_kernel      the iteration's linearisation and blocks: H_pp (21) + b_p (6) per free pose in tree4096
//                         order (16 workgroups per pose, each edge's e and J_pose formed on the fly), and one lane per
//                         landmark that linearises its edges -- e, J_pose (the reference's linearizeOplus), J_point =
//                         J_pose[:, :3] R, stored for the later kernels (H_pl = J_pose^T J_point is formed from them
//                         where it is read) -- for H_ll, b_l (sequential over its edges); its last workgroup starts
//                         the iteration's trial loop (device control). (Until round 5 a separate linearisation
//                         kernel stored e / J first: 10.5 us per iteration on a configs[2] window.)
//   ba_schur_kernel       per trial: the reduced pose system S = H_pp + lambda I - sum W H_pl^T and b_schur in tree4096
//                         order (16 workgroups per upper 6 x 6 block or b_schur row), W = H_pl (H_ll + lambda I)^-1
//                         formed per co-visible pair
//   ba_ldlt_reg_kernel    one workgroup: Eigen's LDLT (diagonal pivoting) on the reduced pose system, the matrix in
//                         registers, column pairs handed between waves through LDS (n <= 128; ba_ldlt_kernel on
//                         global memory above), then the solve
//   ba_step_kernel        the trial state: T <- exp(x_p) T, x_l = Dinv (b_l - sum_e H_pl^T x_p), X <- X + x_l (into
//                         the other state buffer), and the trial's chi2 and LM scale x.(lambda x + b) in the
//                         landmark-block order (one lane per landmark); its last workgroup decides the trial (device
//                         control) or leaves both for the host
//   ba_chi2_kernel        the solve's first chi2 in the same order
// The LM control (lambda, rho, accept / reject) runs on the device by default (ba_ctl_*), in the host loop's
// arithmetic; yv_ba_set_control(b, 0) runs it on the host.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/yavo/yavo.h"
#include "../../include/yavo/yavo_geom.h"
#include "../../include/yavo/yavo_map.h"
#include "yavo_internal.h"
#include "yavo_se3.h"

namespace yavo {
namespace ba {

using se3::quat_to_R;
using se3::se3_act;
using se3::se3_exp;
using se3::se3_mul;

constexpr int kNT = 256;

__device__ __forceinline__ void ba_error(const double* T, const double* K, const double* X, const double* meas,
                                         double* e) {
    double pc[3];
    se3_act(T, X, pc);
    const double u0 = K[0] * pc[0] + K[1] * pc[1] + K[2] * pc[2];
    const double u1 = K[3] * pc[0] + K[4] * pc[1] + K[5] * pc[2];
    const double u2 = K[6] * pc[0] + K[7] * pc[1] + K[8] * pc[2];
    e[0] = meas[0] - u0 / u2;
    e[1] = meas[1] - u1 / u2;
}

// the state (poses, landmarks) the current estimate is in: 0 = P.poses / P.X, 1 = P.poses2 / P.X2
__device__ __forceinline__ int ba_cur(const BaParams& P) { return P.cur ? *P.cur : 0; }

// One edge's linearisation at pose T, point X: the error e = meas - proj(T X), J_pose (the reference's
// linearizeOplus) and J_point = J_pose[:, :3] R. Every reader that needs them forms them with this function, so
// they are the same bits wherever they are formed.
__device__ __forceinline__ void edge_linearize(const double* T, const double* K, const double* X, const double* meas,
                                               double* err, double* Jp, double* Jl) {
    ba_error(T, K, X, meas, err);
    double pc[3];
    se3_act(T, X, pc);
    const double fx = K[0], fy = K[4];
    const double x = pc[0], y = pc[1], z = pc[2];
    const double zinv = 1.0 / (z + 1e-18);
    const double zinv2 = zinv * zinv;
    Jp[0] = -fx * zinv; Jp[1] = 0; Jp[2] = fx * x * zinv2; Jp[3] = fx * x * y * zinv2;
    Jp[4] = -fx - fx * x * x * zinv2; Jp[5] = fx * y * zinv;
    Jp[6] = 0; Jp[7] = -fy * zinv; Jp[8] = fy * y * zinv2; Jp[9] = fy + fy * y * y * zinv2;
    Jp[10] = -fy * x * y * zinv2; Jp[11] = -fy * x * zinv;
    if (Jl) {
        double R[9];
        quat_to_R(T, R);
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                Jl[r * 3 + c] =
                    Jp[r * 6 + 0] * R[0 * 3 + c] + Jp[r * 6 + 1] * R[1 * 3 + c] + Jp[r * 6 + 2] * R[2 * 3 + c];
    }
}

// H_pl(e) = J_pose^T J_point, the expression of the oracle's buildSystem, from the edge's stored Jacobians
__device__ __forceinline__ void hpl_load(const BaParams& P, int64_t e, double* h) {
    double J[12], L[6];
    const double2* jp = reinterpret_cast<const double2*>(P.Jp + 12 * e);
    const double2* jl = reinterpret_cast<const double2*>(P.Jl + 6 * e);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double2 v = jp[i];
        J[2 * i] = v.x;
        J[2 * i + 1] = v.y;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double2 v = jl[i];
        L[2 * i] = v.x;
        L[2 * i + 1] = v.y;
    }
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c) h[3 * a + c] = J[a] * L[c] + J[6 + a] * L[3 + c];
}

// last-block-done: every workgroup of the launch arrives once; true in the workgroup that arrived last. What the
// last workgroup reads from the others is published write-through (agent-scope atomic stores, or atomics), drained
// (s_waitcnt vmcnt(0) in every storing wave) before the workgroup's barrier and ticket, and read back with agent-scope
// atomic loads: no cache maintenance fences (MI355X guide, Guideline 16's sc1 form). The counter is left at 0 for the
// next launch. Every thread of the workgroup must call it.
__device__ bool ba_last_block(unsigned* ticket) {
    __shared__ unsigned s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned tk = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = tk == gridDim.x - 1;
        if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last ? 1u : 0u;
    }
    __syncthreads();
    return s_last != 0;
}

// the same over a large grid: consecutive workgroups in groups of gs = max(16, ceil(grid / 64)), counted per group
// (groups[0 .. 63]); the last of a group counts at *top. Same-address atomics serialise at the cache (a 512-way
// single counter cost ~10 us), so no counter takes more than 64 arrivals.
constexpr int kTicketGroups = 64;
__device__ bool ba_last_block_h(unsigned* top, unsigned* groups) {
    __shared__ unsigned s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned G = gridDim.x;
        const unsigned gs = max(16u, (G + kTicketGroups - 1) / kTicketGroups);
        const unsigned gi = blockIdx.x / gs, ng = (G + gs - 1) / gs, gsize = min(gs, G - gi * gs);
        bool last = false;
        if (__hip_atomic_fetch_add(&groups[gi], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
            __hip_atomic_store(&groups[gi], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1) {
                __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = true;
            }
        }
        s_last = last ? 1u : 0u;
    }
    __syncthreads();
    return s_last != 0;
}

// last of `count` workgroups to arrive at a per-task counter (see ba_last_block)
__device__ bool ba_last_of(unsigned* ticket, unsigned count) {
    __shared__ unsigned s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned tk = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = tk == count - 1;
        if (last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = last ? 1u : 0u;
    }
    __syncthreads();
    return s_last != 0;
}

__device__ __forceinline__ double ld_agent(const double* p) {
    return __longlong_as_double(
        __hip_atomic_load(reinterpret_cast<const long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// an iteration's trial loop starts (after its linearisation); the first one sets lambda = tau max|H_ii|
__device__ void ba_ctl_iter_begin(BaCtl* c, const unsigned long long* maxdiag) {
    if (maxdiag) {
        const double maxd = __longlong_as_double(
            (long long)__hip_atomic_load(maxdiag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        c->lambda = 1e-5 * maxd;
        c->ni = 2;
    }
    c->q = 0;
    c->iter_done = 0;
    c->skip_trial = 0;
}

// tree4096 (the oracle's order for H_pp / b_p, the Schur blocks and b_schur): leaf t sums items k = t mod 4096 in
// ascending k from 0.0, then p[t] += p[t + off], off = 2048 .. 1. A sum runs on kWG workgroups of kWLanes lanes:
// lane u of workgroup g holds leaf g + kWG u. Levels off = 2048 .. kWG add leaves of one residue class mod kWG, so
// each workgroup runs them on its own leaves (off / kWG lanes apart, nv trees at once) and publishes its class totals;
// the last workgroup runs levels kWG / 2 .. 1 over the kWG totals.
constexpr int kWLeaves = 4096;
// 16 workgroups of 256 lanes per sum (32 x 128 until c49: the reduce kernel 19.4 -> 17.3 us, the Schur kernel the same;
// 8 x 512: Schur 33 us, profiles/r05/c49)
constexpr int kWG = 16;
constexpr int kWLanes = kWLeaves / kWG;  // 256

template <int NV>
__device__ __forceinline__ void wide_local_tree(double* red) {  // red[q * kWLanes + u]; totals end in red[q * kWLanes]
    const int t = threadIdx.x;
    __syncthreads();
    for (int off = kWLanes / 2; off > 0; off >>= 1) {
        for (int idx = t; idx < NV * off; idx += kWLanes) {
            const int q = idx / off, u = idx - q * off;
            red[q * kWLanes + u] = red[q * kWLanes + u] + red[q * kWLanes + u + off];
        }
        __syncthreads();
    }
}

// levels kWG / 2 .. 1 over the class totals part[u * stride], u < kWG (published write-through)
__device__ __forceinline__ double wide_top_tree(const double* part, int stride) {
    double v[kWG];
#pragma unroll
    for (int u = 0; u < kWG; ++u) v[u] = ld_agent(&part[u * stride]);
#pragma unroll
    for (int off = kWG / 2; off > 0; off >>= 1)
#pragma unroll
        for (int i = 0; i < off; ++i) v[i] = v[i] + v[i + off];
    return v[0];
}

__device__ __forceinline__ void atomic_max_abs(unsigned long long* m, double v) {
    if (v > 0.0)  // NaN never, as fmax ignores it
        __hip_atomic_fetch_max(m, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One launch for the iteration's blocks of H and b (kWLanes threads per workgroup):
//  blocks [0, np kWG)  kWG per free pose: 21 upper H_pp entries + 6 b_p entries in tree4096 order over the pose's
//                      edges (a lane's items k = leaf + 4096 m: one per lane up to 4096 edges, all loads in flight),
//                      the 27 local trees at once, class totals published; the pose's last workgroup writes H_pp, b_p
//  blocks beyond:      one lane per landmark: H_ll, b_l sequential over its edges
// first: the largest |diagonal| (free poses and landmarks) into *P.maxdiag (uint64 bits of a non-negative double).
// Device control: the last workgroup starts the iteration's trial loop (lambda on the first iteration).
__global__ __launch_bounds__(kWLanes) void ba_reduce_kernel(BaParams P, BaMat3 K, int first) {
    __shared__ double red[27 * kWLanes];
    if (P.gate && *P.gate) return;  // a skipped phase of the device-driven LM
    const int t = threadIdx.x;
    const int cur = ba_cur(P);
    const double* Tc = cur ? P.poses2 : P.poses;
    const double* Xc = cur ? P.X2 : P.X;
    if ((int)blockIdx.x < P.np * kWG) {
        const int j = blockIdx.x / kWG, g = blockIdx.x - j * kWG, p = P.nf + j;
        const int k0 = P.pe_off[p], k1 = P.pe_off[p + 1];
        double T[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) T[i] = Tc[7 * p + i];
        double h[21], gv[6];
#pragma unroll
        for (int i = 0; i < 21; ++i) h[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) gv[i] = 0.0;
        // the pose's edges linearised here (the landmark lanes below store the same bits for the later kernels)
        for (int k = k0 + g + kWG * t; k < k1; k += kWLeaves) {
            const int e = P.pe[k];
            double J[12], ev[2];
            edge_linearize(T, K.v, Xc + 3 * (int64_t)P.el[e], P.meas + 2 * (int64_t)e, ev, J, nullptr);
            int q = 0;
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int b = a; b < 6; ++b, ++q) h[q] = h[q] + (J[a] * J[b] + J[6 + a] * J[6 + b]);
#pragma unroll
            for (int a = 0; a < 6; ++a) gv[a] = gv[a] + (J[a] * ev[0] + J[6 + a] * ev[1]);
        }
#pragma unroll
        for (int i = 0; i < 21; ++i) red[i * kWLanes + t] = h[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) red[(21 + i) * kWLanes + t] = gv[i];
        wide_local_tree<27>(red);
        double* part = P.rpart + (int64_t)j * kWG * 27;
        if (t < 27) st_agent(&part[g * 27 + t], red[t * kWLanes]);
        if (ba_last_of(P.rticket + j, kWG) && t < 27) {
            const double v = wide_top_tree(part + t, 27);
            double* H = P.Hpp + 36 * p;
            if (t < 21) {
                int a = 0, q = t;
                while (q >= 6 - a) {
                    q -= 6 - a;
                    ++a;
                }
                const int b = a + q;
                H[6 * a + b] = H[6 * b + a] = v;
                if (first && a == b) atomic_max_abs(P.maxdiag, fabs(v));
            } else {
                P.bp[6 * p + t - 21] = -v;
            }
        }
    } else {
        const int l = (blockIdx.x - P.np * kWG) * kWLanes + t;
        if (l < P.L) {
            double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
            const int k0 = P.le_off[l], k1 = P.le_off[l + 1];
            double X[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) X[c] = Xc[3 * (int64_t)l + c];
            // the landmark's edges two at a time: indices and poses, then both linearised (error, J_pose, J_point:
            // stored for the Schur and step kernels, 16-B stores) and added in edge order
            for (int kb = k0; kb < k1; kb += 2) {
                int eb[2], pb[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) eb[u] = kb + u < k1 ? P.le[kb + u] : 0;
#pragma unroll
                for (int u = 0; u < 2; ++u) pb[u] = kb + u < k1 ? P.ep[eb[u]] : 0;
                double jl[2][6], er[2][2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if (kb + u < k1) {
                        double Jp[12];
                        edge_linearize(Tc + 7 * (int64_t)pb[u], K.v, X, P.meas + 2 * (int64_t)eb[u], er[u], Jp, jl[u]);
                        reinterpret_cast<double2*>(P.err)[eb[u]] = make_double2(er[u][0], er[u][1]);
                        double2* jp2 = reinterpret_cast<double2*>(P.Jp + 12 * (int64_t)eb[u]);
#pragma unroll
                        for (int i = 0; i < 6; ++i) jp2[i] = make_double2(Jp[2 * i], Jp[2 * i + 1]);
                        double2* jl2 = reinterpret_cast<double2*>(P.Jl + 6 * (int64_t)eb[u]);
#pragma unroll
                        for (int i = 0; i < 3; ++i) jl2[i] = make_double2(jl[u][2 * i], jl[u][2 * i + 1]);
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if (kb + u >= k1) break;
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
#pragma unroll
                        for (int b = a; b < 3; ++b)
                            h[3 * a + b] = h[3 * a + b] + (jl[u][a] * jl[u][b] + jl[u][3 + a] * jl[u][3 + b]);
                        g[a] = g[a] + (jl[u][a] * er[u][0] + jl[u][3 + a] * er[u][1]);
                    }
                }
            }
            double m = 0.0;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
#pragma unroll
                for (int b = a; b < 3; ++b) {
                    P.Hll[9 * l + 3 * a + b] = h[3 * a + b];
                    P.Hll[9 * l + 3 * b + a] = h[3 * a + b];
                }
                P.bl[3 * l + a] = -g[a];
                m = fmax(m, fabs(h[4 * a]));
            }
            if (first) atomic_max_abs(P.maxdiag, m);
        }
    }
    if (P.ctl && ba_last_block_h(P.ticket + 0, P.ticket + 4) && t == 0)
        ba_ctl_iter_begin(P.ctl, first ? P.maxdiag : nullptr);
}

__device__ __forceinline__ void inv3(const double* a, double* o) {
    const double c00 = a[4] * a[8] - a[5] * a[7], c01 = a[5] * a[6] - a[3] * a[8], c02 = a[3] * a[7] - a[4] * a[6];
    const double det = a[0] * c00 + a[1] * c01 + a[2] * c02;
    const double id = 1.0 / det;
    o[0] = c00 * id; o[1] = (a[2] * a[7] - a[1] * a[8]) * id; o[2] = (a[1] * a[5] - a[2] * a[4]) * id;
    o[3] = c01 * id; o[4] = (a[0] * a[8] - a[2] * a[6]) * id; o[5] = (a[2] * a[3] - a[0] * a[5]) * id;
    o[6] = c02 * id; o[7] = (a[1] * a[6] - a[0] * a[7]) * id; o[8] = (a[0] * a[4] - a[1] * a[3]) * id;
}

// (H_ll + lambda I)^-1 of landmark l, the oracle's expressions (its Dinv)
__device__ __forceinline__ void landmark_dinv(const BaParams& P, int l, double lambda, double* Di) {
    double d[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) d[i] = P.Hll[9 * (int64_t)l + i];
#pragma unroll
    for (int a = 0; a < 3; ++a) d[4 * a] = d[4 * a] + lambda;
    inv3(d, Di);
}

// W_e = H_pl(e) Dinv (6 x 3), the oracle's expression
__device__ __forceinline__ void w_block(const double* h, const double* Di, double* w) {
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            w[3 * a + c] = h[3 * a + 0] * Di[0 * 3 + c] + h[3 * a + 1] * Di[1 * 3 + c] + h[3 * a + 2] * Di[2 * 3 + c];
}


// The Schur complement in the oracle's tree4096 order. Task = an upper block (p1 <= p2) of the free poses, or one
// pose's b_schur; kWG workgroups per task (see wide_local_tree). A lane's items (pair k = leaf + 4096 m) form what the
// oracle's trial step stores: Dinv of the pair's landmark from H_ll + lambda I, H_pl of both edges from their
// Jacobians, W_e1 = H_pl(e1) Dinv -- the same expressions, so the same bits, with no W / Dinv round trip through
// HBM and no trial kernel (216 B read per diagonal pair, 360 B per off-diagonal one). A configs[2] window has at most
// one item per lane, so a block's ~3,700 pairs are spread over 16 CUs with every load in flight at once.
// grid: (nb + np) kWG workgroups; task = blockIdx / kWG, g = blockIdx % kWG.
//  tasks [0, nb): S(a, b) = base - tree4096 over the co-visible pairs k of (W_e1(k)[a] . H_pl(e2(k))[b]); on a
//    diagonal block only a >= b is written, to both mirrored entries (the oracle's loop leaves that value)
//  tasks [nb, nb + np): b_schur(a) = b_p[a] - tree4096 over the pose's edges of W_e[a] . b_l(e)
__global__ __launch_bounds__(kWLanes) void ba_schur_kernel(BaParams P, double lambda) {
    __shared__ double red[36 * kWLanes];
    if (P.gate && *P.gate) return;  // a skipped phase of the device-driven LM
    if (P.lam) lambda = *P.lam;
    const int np = P.np, nb = np * (np + 1) / 2;
    const int task = blockIdx.x / kWG, g = blockIdx.x - task * kWG;
    const int t = threadIdx.x, leaf = g + kWG * t;
    if (task < nb) {
        int blk = task, i1 = 0;
        while (blk >= np - i1) {
            blk -= np - i1;
            ++i1;
        }
        const int i2 = i1 + blk;
        const int p1 = P.nf + i1, p2 = P.nf + i2;
        const int c0 = P.cv_off[p1 * P.P + p2], c1 = P.cv_off[p1 * P.P + p2 + 1];
        if (c1 == c0) {  // no shared landmark: base - (the tree of 0.0 leaves = 0.0)
            if (g == 0)
                for (int q = t; q < 36; q += kWLanes) {
                    const int a = q / 6, b = q % 6;
                    if (i1 == i2 && a < b) continue;
                    const double base = p1 == p2 ? P.Hpp[36 * p1 + 6 * a + b] + (a == b ? lambda : 0.0) : 0.0;
                    const double v = base - 0.0;
                    const int r = 6 * i1 + a, c = 6 * i2 + b, ns = P.ns;
                    P.S[(int64_t)r * ns + c] = v;
                    P.S[(int64_t)c * ns + r] = v;
                }
            return;
        }
        double acc[36];
#pragma unroll
        for (int i = 0; i < 36; ++i) acc[i] = 0.0;
        for (int i = c0 + leaf; i < c1; i += kWLeaves) {
            const int e1 = P.cv_e1[i], e2 = P.cv_e2[i];
            double Di[9], h[18], w[18];
            landmark_dinv(P, P.el[e1], lambda, Di);
            hpl_load(P, e1, h);
            w_block(h, Di, w);  // W_e1 = H_pl(e1) Dinv: the trial kernel's product, formed here
            if (e2 != e1) hpl_load(P, e2, h);
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int b = 0; b < 6; ++b)
                    acc[6 * a + b] = acc[6 * a + b] + (w[3 * a] * h[3 * b] + w[3 * a + 1] * h[3 * b + 1] + w[3 * a + 2] * h[3 * b + 2]);
        }
#pragma unroll
        for (int q = 0; q < 36; ++q) red[q * kWLanes + t] = acc[q];
        wide_local_tree<36>(red);
        double* part = P.spart + (int64_t)task * kWG * 36;
        if (t < 36) st_agent(&part[g * 36 + t], red[t * kWLanes]);
        if (!ba_last_of(P.sticket + task, kWG)) return;
        if (t < 36) {
            const int a = t / 6, b = t % 6;
            if (!(i1 == i2 && a < b)) {
                const double base = p1 == p2 ? P.Hpp[36 * p1 + 6 * a + b] + (a == b ? lambda : 0.0) : 0.0;
                const double v = base - wide_top_tree(part + t, 36);
                const int r = 6 * i1 + a, c = 6 * i2 + b, ns = P.ns;
                P.S[(int64_t)r * ns + c] = v;
                P.S[(int64_t)c * ns + r] = v;
            }
        }
    } else {
        const int j = task - nb, p = P.nf + j;
        const int k0 = P.pe_off[p], k1 = P.pe_off[p + 1];
        double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        for (int i = k0 + leaf; i < k1; i += kWLeaves) {
            const int e = P.pe[i], l = P.el[e];
            double Di[9], h[18], w[18];
            landmark_dinv(P, l, lambda, Di);
            hpl_load(P, e, h);
            w_block(h, Di, w);
            const double* gl = P.bl + 3 * l;
            const double g0 = gl[0], g1 = gl[1], g2 = gl[2];
#pragma unroll
            for (int a = 0; a < 6; ++a) acc[a] = acc[a] + (w[3 * a] * g0 + w[3 * a + 1] * g1 + w[3 * a + 2] * g2);
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) red[q * kWLanes + t] = acc[q];
        wide_local_tree<6>(red);
        double* part = P.spart + (int64_t)task * kWG * 36;
        if (t < 6) st_agent(&part[g * 36 + t], red[t * kWLanes]);
        if (!ba_last_of(P.sticket + task, kWG)) return;
        if (t < 6) P.bs[6 * j + t] = P.bp[6 * p + t] - wide_top_tree(part + t, 36);
    }
}

// Eigen LDLT on the reduced system (n <= kLdltRegN = 128), bit-identical to the oracle's left-looking
// or_ldlt_solve (diagonal pivoting), in one 512-thread workgroup with no workgroup barrier inside the factorisation:
//  1. The pivot sequence. At step k the oracle takes the first position of the largest |L(i, i)|, i >= k, and L(i, i)
//     for i >= k still holds an original diagonal entry (it is only updated at its own step), so the sequence follows
//     from the diagonal alone. Distinct values (the usual case): it is the descending order, by ranks. Any tie or NaN:
//     wave 0 replays the oracle's scan-and-swap step by step.
//  2. Pivoting commutes with the left-looking factorisation: the oracle swaps untouched original entries in the
//     trailing part and the finished rows of L, so its result equals the unpivoted factorisation of P S P^T (S is
//     bitwise symmetric: each Schur entry is stored to both halves from one value).
//  3. The unpivoted factorisation runs right-looking with the matrix in registers, two columns at a time. The oracle
//     forms column k as acc = L(i, k) - L(i, 0) t_0 - L(i, 1) t_1 - ... (t_j = D(j) L(k, j)) and D(k) = L(k, k) -
//     (L(k, 0) t_0 + ...); a term j applied to every such chain (L(i, c) -= L(i, j) t_j(c), t_j(c) = D(j) L(c, j);
//     dot_i += L(i, j) t_j(i)) in ascending j gives the same operations in the same order per entry. Wave w (of 8, two
//     per SIMD) holds the column pairs q = 8 j + w (columns 2q, 2q + 1) of P S P^T, lane l rows l and l + 64. The wave
//     that holds pair q + 1 finalises both its columns as soon as pair q is published: column 2q + 2 from terms 2q,
//     2q + 1 and its division, then column 2q + 3 with term 2q + 2 taken from its own lanes by v_readlane (no LDS
//     round trip inside the pair) -- at raised wave priority, before its share of the bulk update. A published pair
//     is L(., c) in the column store (kept for the solves), t_c(.) in a ring of kLdltRing pair slots and a per-slot
//     flag (workgroup-scope release / acquire). Every wave then applies the pair's two terms to its live pairs'
//     registers (a finalised pair's registers are dead). A slot is rewritten kLdltRing pairs later, which needs every
//     wave to have read it: a wave owns one of any eight consecutive pairs, so none runs more than eight ahead.
//     Wave 0 also runs the forward solve v(i) -= L(i, k) v(k), in the oracle's order.
//     (Round 4 kept the packed triangle in LDS with one workgroup barrier per column step: 139 us per factorisation
//     at n = 120 in the configs[2] sequence; one column per hand-off with four waves: 84 us.)
//  4. The diagonal and backward solves run on wave 0: the vector in registers (two entries per lane), broadcasts by
//     v_readlane, L read by row from the column store (stride 129 doubles: conflict-free by rows and by columns).
constexpr int kLdltRegN = 128;   // n <= 128: lane l holds rows l and l + 64
constexpr int kLdltWaves = 8;    // 512 threads: two waves per SIMD
constexpr int kLdltPairs = 8;    // column pairs per wave: pair 8 j + w holds columns 16 j + 2 w, 16 j + 2 w + 1
constexpr int kLdltLs = 129;     // column stride of the L store (doubles)
constexpr int kLdltRing = 8;     // published pairs in flight

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// makes one wave's LDS stores visible to its other lanes' later loads (wave-synchronous phases)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// t_c(r) of a ring slot's term h at [h][tq_index(r)] (row order: each wave loads them lane-distributed)
__device__ __forceinline__ int tq_index(int r) { return r; }

#ifdef YAVO_LM_PROFILE
// profiling builds: shader cycles of lane 0 of each wave in the phases of the LDLT, summed over launches
__device__ unsigned long long g_ldlt_prof[kLdltWaves][8];
#define LDP_DECL unsigned long long ldp_t = __builtin_readcyclecounter(), ldp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define LDP_MARK(q) do { const unsigned long long t_ = __builtin_readcyclecounter(); ldp_acc[q] += t_ - ldp_t; ldp_t = t_; } while (0)
#define LDP_STORE() do { if (l == 0) for (int q_ = 0; q_ < 8; ++q_) atomicAdd(&g_ldlt_prof[w][q_], ldp_acc[q_]); } while (0)
#else
#define LDP_DECL
#define LDP_MARK(q) do {} while (0)
#define LDP_STORE() do {} while (0)
#endif

// pair q + 1 = 8 J + w of this wave: both columns finalised and published (read-only on the registers)
#define LDLT_FIN(J)                                                                                            \
    case J: {                                                                                                  \
        constexpr int jl_ = (J) < kLdltPairs / 2 ? (J) : 0;                                                    \
        /* column an: terms ca, cb, then D(an) and the division */                                             \
        double aa0 = 0.0;                                                                                      \
        if ((J) < kLdltPairs / 2) aa0 = (Al[jl_][0] - lka0 * ta_a) - lkb0 * tb_a;                              \
        const double aa1 = (Ah[J][0] - lka1 * ta_a) - lkb1 * tb_a;                                             \
        const bool va = fabs(da) > 0;                                                                          \
        const double La0 = (J) < kLdltPairs / 2 ? (va ? aa0 / da : aa0) : 0.0;                                 \
        const double La1 = va ? aa1 / da : aa1;                                                                \
        const double ua0 = (J) < kLdltPairs / 2 ? da * La0 : 0.0, ua1 = da * La1;                              \
        if ((J) < kLdltPairs / 2) {                                                                            \
            Lc[an * kLdltLs + r0] = La0;                                                                       \
            tqn[tq0] = ua0;                                                                                    \
        }                                                                                                      \
        Lc[an * kLdltLs + r1] = La1;                                                                           \
        tqn[tq1] = ua1;                                                                                        \
        if (l == 0) Dv[an] = da;                                                                               \
        if (bn < n) {                                                                                          \
            /* column bn: terms ca, cb, an (t_an(bn) from row bn's lane), D(bn) = S(bn, bn) - (dot + L t) */   \
            const double ta_b = readlane_f64(bn < 64 ? ua0 : ua1, bn & 63);                                    \
            const double db = dorb - readlane_f64(bn < 64 ? dot0 + La0 * ua0 : dot1 + La1 * ua1, bn & 63);   \
            double ab0 = 0.0;                                                                                  \
            if ((J) < kLdltPairs / 2) ab0 = ((Al[jl_][1] - lka0 * tc_b) - lkb0 * td_b) - La0 * ta_b;           \
            const double ab1 = ((Ah[J][1] - lka1 * tc_b) - lkb1 * td_b) - La1 * ta_b;                          \
            const bool vb = fabs(db) > 0;                                                                      \
            const double Lb0 = (J) < kLdltPairs / 2 ? (vb ? ab0 / db : ab0) : 0.0;                             \
            const double Lb1 = vb ? ab1 / db : ab1;                                                            \
            if ((J) < kLdltPairs / 2) {                                                                        \
                Lc[bn * kLdltLs + r0] = Lb0;                                                                   \
                tqn[kLdltRegN + tq0] = db * Lb0;                                                               \
            }                                                                                                  \
            Lc[bn * kLdltLs + r1] = Lb1;                                                                       \
            tqn[kLdltRegN + tq1] = db * Lb1;                                                                   \
            if (l == 0) Dv[bn] = db;                                                                           \
        }                                                                                                      \
        __hip_atomic_store(&flag[qn & (kLdltRing - 1)], qn, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);   \
    } break;

__global__ __launch_bounds__(64 * kLdltWaves) void ba_ldlt_reg_kernel(BaParams P) {
    if (P.gate && *P.gate) return;  // a skipped phase of the device-driven LM
    __shared__ double Lc[kLdltRegN * kLdltLs];       // L(r, c) at Lc[c * 129 + r]
    __shared__ double tq[kLdltRing][2][kLdltRegN];   // pair q's t_2q(.), t_2q+1(.) in slot q % kLdltRing
    __shared__ double Dv[kLdltRegN];                 // D(k)
    __shared__ double dor[kLdltRegN];                // the diagonal of P S P^T
    __shared__ double dg[kLdltRegN];                 // |diagonal|, permuted as the pivots are taken
    __shared__ double dsv[kLdltRegN];                // the diagonal of S
    __shared__ int perm[kLdltRegN];                  // position -> original index: (P S P^T)(i, j) = S(perm[i], perm[j])
    __shared__ int flag[kLdltRing];                  // the pair a slot holds (-1: none yet)
    __shared__ int s_slow;
    const int n = P.ns, t = threadIdx.x, l = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int r0 = l, r1 = l + 64;
    LDP_DECL
    // S is read straight from global memory (L2-resident: the Schur kernel just wrote it): its diagonal here, the
    // registers' entries once the permutation is known (round 4 staged all of S in LDS first: ~4 us more)
    if (t < n) {
        const double d = P.S[(int64_t)t * n + t];
        dg[t] = fabs(d);
        dsv[t] = d;
    }
    if (t < kLdltRing) flag[t] = -1;
    if (t == 0) s_slow = 0;
    __syncthreads();
    // 1. ranks by (|d| descending, index ascending); a tie or a NaN sends the sequence to the replay
    if (t < n) {
        const double d = dg[t];
        int rank = 0;
        bool tie = isnan(d);
        int j = 0;
        for (; j + 8 <= n; j += 8) {
            double o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) o[u] = dg[j + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                rank += o[u] > d;
                tie |= (o[u] == d && j + u != t);
            }
        }
        for (; j < n; ++j) {
            const double o = dg[j];
            rank += o > d;
            tie |= (o == d && j != t);
        }
        perm[rank] = t;  // a permutation when there is no tie
        if (tie) s_slow = 1;
    }
    __syncthreads();
    if (s_slow) {
        if (t < 64) {
            for (int i = t; i < n; i += 64) perm[i] = i;
            wave_lds_sync();
            for (int k = 0; k < n; ++k) {
                double bv = -1.0;
                int bi = n;
                for (int i = k + t; i < n; i += 64) {
                    const double d = dg[i];
                    if (isnan(d)) continue;
                    if (bi == n || d > bv) {
                        bv = d;
                        bi = i;
                    }
                }
#pragma unroll
                for (int m = 1; m < 64; m <<= 1) {
                    const double ov = __shfl_xor(bv, m);
                    const int oi = __shfl_xor(bi, m);
                    if (oi < n && (bi == n || ov > bv || (ov == bv && oi < bi))) {
                        bv = ov;
                        bi = oi;
                    }
                }
                if (isnan(dg[k]) || bi == n) bi = k;
                wave_lds_sync();
                if (t == 0 && bi != k) {
                    const double q = dg[k];
                    dg[k] = dg[bi];
                    dg[bi] = q;
                    const int pq = perm[k];
                    perm[k] = perm[bi];
                    perm[bi] = pq;
                }
                wave_lds_sync();
            }
        }
        __syncthreads();
    }
    // the oracle's first step: a zero (or NaN) pivot ends the factorisation with only its own transposition applied
    // to the matrix and none to the vector
    const int big0 = perm[0];
    const double a00 = dsv[big0];
    const bool brk = !(fabs(a00) > 0);
    __syncthreads();
    if (brk) {
        if (t < n) perm[t] = t == 0 ? big0 : (t == big0 ? 0 : t);
        __syncthreads();
    }
    // 2. P S P^T into registers: Al[j][h] = entry (r0, 16 j + 2 w + h) for the columns below 64, Ah[j][h] = (r1, ...);
    // only the strict lower triangle is read (the rest is never used). S is bitwise symmetric, so entry (r, c) is read
    // as S(perm[c], perm[r]): one row of S per load instruction, all 24 loads of a lane in flight together
    double Al[kLdltPairs / 2][2], Ah[kLdltPairs][2];
    const int tq0 = tq_index(r0), tq1 = tq_index(r1);
    {
        const int p0 = r0 < n ? perm[r0] : 0, p1 = r1 < n ? perm[r1] : 0;
#pragma unroll
        for (int j = 0; j < kLdltPairs; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = 16 * j + 2 * w + h;
                const int pc = c < n ? perm[c] : 0;
                const double* row = P.S + (int64_t)pc * n;
                if (j < kLdltPairs / 2) Al[j < kLdltPairs / 2 ? j : 0][h] = (r0 > c && r0 < n) ? row[p0] : 0.0;
                Ah[j][h] = (r1 > c && r1 < n) ? row[p1] : 0.0;
            }
        if (t < n) dor[t] = dsv[perm[t]];
    }
    // the right-hand side, permuted (a zero first pivot: not permuted) -- wave 0 solves
    double v0 = 0.0, v1 = 0.0;
    if (w == 0) {
        v0 = r0 < n ? P.bs[brk ? r0 : perm[r0]] : 0.0;
        v1 = r1 < n ? P.bs[brk ? r1 : perm[r1]] : 0.0;
    }
    __syncthreads();
    int err = 0;
    if (brk) {
        // the solves read P S P^T as it stands
#pragma unroll
        for (int j = 0; j < kLdltPairs; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = 16 * j + 2 * w + h;
                if (c < n) {
                    if (j < kLdltPairs / 2) Lc[c * kLdltLs + r0] = Al[j < kLdltPairs / 2 ? j : 0][h];
                    Lc[c * kLdltLs + r1] = Ah[j][h];
                }
            }
        if (t < n) Dv[t] = dor[t];
        __syncthreads();
        if (w == 0)
            for (int j = 0; j < n; ++j) {
                const double vj = readlane_f64(j < 64 ? v0 : v1, j & 63);
                const double a0 = Lc[j * kLdltLs + r0], a1 = Lc[j * kLdltLs + r1];
                if (r0 > j && r0 < n) v0 = v0 - a0 * vj;
                if (r1 > j && r1 < n) v1 = v1 - a1 * vj;
            }
    } else {
        // 3. pair 0 (wave 0): column 0 with D(0) = a00 (nonzero here); column 1 from term 0 alone, dot_1 = L(1, 0) t_0(1)
        if (w == 0) {
            const double L00 = Al[0][0] / a00, L01 = Ah[0][0] / a00;
            const double u00 = a00 * L00, u01 = a00 * L01;
            Lc[r0] = L00;
            Lc[r1] = L01;
            tq[0][0][tq0] = u00;
            tq[0][0][tq1] = u01;
            if (l == 0) Dv[0] = a00;
            if (n > 1) {
                const double t01 = readlane_f64(u00, 1);
                const double d1 = dor[1] - readlane_f64(L00 * u00, 1);
                const bool v1ok = fabs(d1) > 0;
                const double b0 = Al[0][1] - L00 * t01, b1 = Ah[0][1] - L01 * t01;
                const double L10 = v1ok ? b0 / d1 : b0, L11 = v1ok ? b1 / d1 : b1;
                Lc[kLdltLs + r0] = L10;
                Lc[kLdltLs + r1] = L11;
                tq[0][1][tq0] = d1 * L10;
                tq[0][1][tq1] = d1 * L11;
                if (l == 0) Dv[1] = d1;
            }
            __hip_atomic_store(&flag[0], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        double dot0 = 0.0, dot1 = 0.0;  // rows r0, r1: L(r, 0) t_0(r) + L(r, 1) t_1(r) + ... (term 0 assigns)
        const int NP = (n + 1) >> 1;
        LDP_MARK(0);
        for (int q = 0; q < NP; ++q) {
            const int s = q & (kLdltRing - 1);
            for (int spin = 0; __hip_atomic_load(&flag[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q;) {
                if (++spin > (1 << 24)) {  // never expected: a bounded wait, reported as a failed solve
                    err = 1;
                    break;
                }
                // a short sleep between polls leaves the SIMD's issue slots to the wave finalising the pair
                // (60.2 vs 61 us per factorisation, +1% on the sequence leg: profiles/r05/c54)
                __builtin_amdgcn_s_sleep(1);
            }
            if (err) break;
            LDP_MARK(1);
            const int ca = 2 * q, cb = 2 * q + 1;  // this step's terms (cb == n: absent, odd n)
            const bool hb = cb < n;
            const int qn = q + 1, an = 2 * qn, bn = 2 * qn + 1;
            // the loads the critical path needs first: this wave's rows of columns ca, cb and their t values
            const double lka0 = Lc[ca * kLdltLs + r0], lka1 = Lc[ca * kLdltLs + r1];
            const double lkb0 = Lc[cb * kLdltLs + r0], lkb1 = Lc[cb * kLdltLs + r1];
            const double tka0 = tq[s][0][tq0], tka1 = tq[s][0][tq1];
            const double tkb0 = tq[s][1][tq0], tkb1 = tq[s][1][tq1];
            const double dora = dor[an < n ? an : 0], dorb = dor[bn < n ? bn : 0];
            dot0 = ca == 0 ? lka0 * tka0 : dot0 + lka0 * tka0;
            dot1 = ca == 0 ? lka1 * tka1 : dot1 + lka1 * tka1;
            if (hb) {
                dot0 = dot0 + lkb0 * tkb0;
                dot1 = dot1 + lkb1 * tkb1;
            }
            LDP_MARK(2);
            if (qn < NP && (qn & (kLdltWaves - 1)) == w) {  // this wave holds pair q + 1 (wave-uniform; hb holds)
                __builtin_amdgcn_s_setprio(3);
                double* const tqn = &tq[qn & (kLdltRing - 1)][0][0];
                const double ta_a = readlane_f64(an < 64 ? tka0 : tka1, an & 63);  // t_ca(an)
                const double tb_a = readlane_f64(an < 64 ? tkb0 : tkb1, an & 63);  // t_cb(an)
                const double tc_b = readlane_f64(bn < 64 ? tka0 : tka1, bn & 63);  // t_ca(bn)
                const double td_b = readlane_f64(bn < 64 ? tkb0 : tkb1, bn & 63);  // t_cb(bn)
                const double da = dora - readlane_f64(an < 64 ? dot0 : dot1, an & 63);
                switch (qn >> 3) {
                    LDLT_FIN(0) LDLT_FIN(1) LDLT_FIN(2) LDLT_FIN(3) LDLT_FIN(4) LDLT_FIN(5) LDLT_FIN(6) LDLT_FIN(7)
                    default: break;
                }
                __builtin_amdgcn_s_setprio(0);
                LDP_MARK(3);
            }
            // terms ca, cb on this wave's live pairs (pair 8 j + w > q). The t values of a pair's columns c are
            // v_readlane broadcasts of the lane-distributed t_ca(.), t_cb(.) loaded above (lane c & 63 of the half
            // holding c): LDS broadcast loads of them cost eight waves' worth of LDS return bandwidth every step
#pragma unroll
            for (int j = 0; j < kLdltPairs; ++j) {
                if (8 * j + w > q) {
                    const int cl = (16 * j + 2 * w) & 63;  // wave-uniform lane of this pair's first column
                    const double tax = readlane_f64(j < kLdltPairs / 2 ? tka0 : tka1, cl);
                    const double tay = readlane_f64(j < kLdltPairs / 2 ? tka0 : tka1, cl + 1);
                    if (j < kLdltPairs / 2) {
                        double (&a)[2] = Al[j < kLdltPairs / 2 ? j : 0];
                        a[0] = a[0] - lka0 * tax;
                        a[1] = a[1] - lka0 * tay;
                    }
                    Ah[j][0] = Ah[j][0] - lka1 * tax;
                    Ah[j][1] = Ah[j][1] - lka1 * tay;
                    if (hb) {
                        const double tbx = readlane_f64(j < kLdltPairs / 2 ? tkb0 : tkb1, cl);
                        const double tby = readlane_f64(j < kLdltPairs / 2 ? tkb0 : tkb1, cl + 1);
                        if (j < kLdltPairs / 2) {
                            double (&a)[2] = Al[j < kLdltPairs / 2 ? j : 0];
                            a[0] = a[0] - lkb0 * tbx;
                            a[1] = a[1] - lkb0 * tby;
                        }
                        Ah[j][0] = Ah[j][0] - lkb1 * tbx;
                        Ah[j][1] = Ah[j][1] - lkb1 * tby;
                    }
                }
            }
            if (w == 0) {  // the forward solve's terms ca, cb: rows below each
                const double va = readlane_f64(ca < 64 ? v0 : v1, ca & 63);
                if (r0 > ca && r0 < n) v0 = v0 - lka0 * va;
                if (r1 > ca && r1 < n) v1 = v1 - lka1 * va;
                if (hb) {
                    const double vb = readlane_f64(cb < 64 ? v0 : v1, cb & 63);
                    if (r0 > cb && r0 < n) v0 = v0 - lkb0 * vb;
                    if (r1 > cb && r1 < n) v1 = v1 - lkb1 * vb;
                }
            }
            LDP_MARK(4);
        }
    }
    __syncthreads();
    LDP_MARK(5);
    if (w != 0) {
        LDP_STORE();
        return;  // no barrier below
    }
    // 4. diagonal and backward solves on wave 0: lane l holds positions r0 and r1
    const double d0 = r0 < n ? Dv[r0] : 1.0, d1 = r1 < n ? Dv[r1] : 1.0;
    if (r0 < n) v0 = fabs(d0) > DBL_MIN ? v0 / d0 : 0.0;
    if (r1 < n) v1 = fabs(d1) > DBL_MIN ? v1 / d1 : 0.0;
    // backward, v(i) -= L(j, i) v(j) for j descending: while j >= 64 every row below 64 takes the term (v(j) in the
    // upper half), then only rows below j of the lower half; loads four columns ahead
    {
        int j = n - 1;
        for (; j >= 67; j -= 4) {
            double a0[4], a1[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a0[u] = Lc[r0 * kLdltLs + j - u];
                a1[u] = Lc[r1 * kLdltLs + j - u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double vj = readlane_f64(v1, (j - u) & 63);
                v0 = v0 - a0[u] * vj;
                if (r1 < j - u) v1 = v1 - a1[u] * vj;
            }
        }
        for (; j >= 64; --j) {
            const double vj = readlane_f64(v1, j & 63);
            v0 = v0 - Lc[r0 * kLdltLs + j] * vj;
            if (r1 < j) v1 = v1 - Lc[r1 * kLdltLs + j] * vj;
        }
        for (; j >= 3; j -= 4) {
            double a0[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) a0[u] = Lc[r0 * kLdltLs + j - u];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double vj = readlane_f64(v0, j - u);
                if (r0 < j - u) v0 = v0 - a0[u] * vj;
            }
        }
        for (; j >= 0; --j) {
            const double vj = readlane_f64(v0, j);
            if (r0 < j) v0 = v0 - Lc[r0 * kLdltLs + j] * vj;
        }
    }
    if (r0 < n) P.xp[brk ? r0 : perm[r0]] = v0;
    if (r1 < n) P.xp[brk ? r1 : perm[r1]] = v1;
    // isPositive: the oracle's sign state ends in {0, 1} exactly when no D(k) is negative (a zero first pivot: 0)
    const bool neg = !brk && ((r0 < n && d0 < 0) || (r1 < n && d1 < 0));
    const bool any_neg = __ballot(neg) != 0;
    if (l == 0) {
        P.scal[2] = (any_neg || err) ? 0.0 : 1.0;
        P.scal[3] = err ? 1.0 : 0.0;
    }
    LDP_MARK(6);
    LDP_STORE();
}
#undef LDLT_FIN


// larger systems: the same steps on S in global memory
__global__ __launch_bounds__(256) void ba_ldlt_kernel(BaParams P) {
    if (P.gate && *P.gate) return;  // a skipped phase of the device-driven LM
    extern __shared__ double s_dyn[];  // v [n], temp [n]
    __shared__ double s_pv[kNT];
    __shared__ int s_pi[kNT];
    __shared__ int s_sign, s_break;
    const int n = P.ns, t = threadIdx.x;
    double* S = P.S;
    int* tr = P.tr;
    double* v = s_dyn;
    double* temp = s_dyn + n;
#define LL(i, j) S[(int64_t)(i) * n + (j)]
    if (t == 0) {
        s_sign = 0;
        s_break = 0;
    }
    __syncthreads();
    for (int k = 0; k < n; ++k) {
        // pivot: the first index of the largest |L(i, i)|, i >= k (sequential strict '>' scan)
        double bv = -1.0;
        int bi = n;
        for (int i = k + t; i < n; i += kNT) {
            const double d = fabs(LL(i, i));
            if (bi == n || d > bv) {
                bv = d;
                bi = i;
            }
        }
        s_pv[t] = bv;
        s_pi[t] = bi;
        __syncthreads();
        for (int off = kNT / 2; off > 0; off >>= 1) {
            if (t < off) {
                const double ov = s_pv[t + off];
                const int oi = s_pi[t + off];
                if (oi < n && (s_pi[t] == n || ov > s_pv[t] || (ov == s_pv[t] && oi < s_pi[t]))) {
                    s_pv[t] = ov;
                    s_pi[t] = oi;
                }
            }
            __syncthreads();
        }
        // the sequential scan starts from bv = |L(k, k)| and only moves on a strict '>': ties keep the first index
        const int big = s_pi[0];
        __syncthreads();
        if (t == 0) tr[k] = big;
        if (k != big) {
            const int s = n - big - 1;
            for (int j = t; j < k; j += kNT) {
                const double q = LL(k, j);
                LL(k, j) = LL(big, j);
                LL(big, j) = q;
            }
            for (int j = t; j < s; j += kNT) {
                const double q = LL(big + 1 + j, k);
                LL(big + 1 + j, k) = LL(big + 1 + j, big);
                LL(big + 1 + j, big) = q;
            }
            if (t == 0) {
                const double q = LL(k, k);
                LL(k, k) = LL(big, big);
                LL(big, big) = q;
            }
            for (int i = k + 1 + t; i < big; i += kNT) {
                const double q = LL(i, k);
                LL(i, k) = LL(big, i);
                LL(big, i) = q;
            }
        }
        __syncthreads();
        if (k > 0) {
            for (int j = t; j < k; j += kNT) temp[j] = LL(j, j) * LL(k, j);
            __syncthreads();
            for (int i = k + 1 + t; i < n; i += kNT) {
                double acc = LL(i, k);
                for (int j = 0; j < k; ++j) acc = acc - LL(i, j) * temp[j];
                LL(i, k) = acc;
            }
            if (t == 0) {
                double dot = LL(k, 0) * temp[0];
                for (int j = 1; j < k; ++j) dot = dot + LL(k, j) * temp[j];
                LL(k, k) -= dot;
            }
            __syncthreads();
        }
        const double akk = LL(k, k);
        const bool valid = fabs(akk) > 0;
        if (k == 0 && !valid) {
            if (t == 0) s_break = 1;
            for (int j = t; j < n; j += kNT) tr[j] = j;
            __syncthreads();
            break;
        }
        if (n - k - 1 > 0 && valid)
            for (int i = k + 1 + t; i < n; i += kNT) LL(i, k) /= akk;
        if (t == 0) {
            int sign = s_sign;
            if (sign == 1) { if (akk < 0) sign = 3; }
            else if (sign == 2) { if (akk > 0) sign = 3; }
            else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
            s_sign = sign;
        }
        __syncthreads();
    }
    if (s_break && t == 0) s_sign = 0;
    for (int i = t; i < n; i += kNT) v[i] = P.bs[i];
    __syncthreads();
    if (t == 0)
        for (int k = 0; k < n; ++k) {
            const double q = v[k];
            v[k] = v[tr[k]];
            v[tr[k]] = q;
        }
    __syncthreads();
    for (int j = 0; j < n; ++j) {
        const double vj = v[j];
        for (int i = j + 1 + t; i < n; i += kNT) v[i] = v[i] - LL(i, j) * vj;
        __syncthreads();
    }
    for (int i = t; i < n; i += kNT) {
        const double d = LL(i, i);
        if (fabs(d) > DBL_MIN) v[i] /= d;
        else v[i] = 0;
    }
    __syncthreads();
    for (int j = n - 1; j >= 0; --j) {
        const double vj = v[j];
        for (int i = t; i < j; i += kNT) v[i] = v[i] - LL(j, i) * vj;
        __syncthreads();
    }
    if (t == 0)
        for (int k = n - 1; k >= 0; --k) {
            const double q = v[k];
            v[k] = v[tr[k]];
            v[tr[k]] = q;
        }
    __syncthreads();
    for (int i = t; i < n; i += kNT) P.xp[i] = v[i];
    if (t == 0) P.scal[2] = (s_sign == 1 || s_sign == 0) ? 1.0 : 0.0;
#undef LL
}

// ---- device-driven LM control (the host loop of yv_ba_solve's host form, operation for operation) ----
__device__ void ba_ctl_init(BaCtl* c, double chi2, double* log, unsigned long long* maxdiag) {
    c->currentChi = chi2;
    log[0] = chi2;
    c->lambda = 0;
    c->ni = 2;
    c->rho = 0;
    c->q = 0;
    c->it = 0;
    c->stop = 0;
    c->iters = 0;
    c->skip_iter = 0;
    c->skip_trial = 1;
    c->suspended = 0;
    c->iter_done = 0;
    *maxdiag = 0;
}

// after a trial: rho, accept (lambda *= max(1/3, min(2/3, 1 - (2 rho - 1)^3)), the trial state becomes current) or
// reject (lambda *= ni, ni *= 2); the trial loop ends when !(rho < 0 && q < 10). Then the iteration's end: its chi2
// is logged; stop on q == 10 / rho == 0 / non-finite lambda. A trial loop still running after the one trial slot the
// host enqueued per iteration suspends the solve (every later kernel skips) until the host resumes it.
__device__ void ba_ctl_decide(BaCtl* c, double tempChi, double scale, bool ok2, int* cur, double* log) {
    if (!ok2) tempChi = DBL_MAX;
    double rho = c->currentChi - tempChi;
    scale += 1e-3;
    rho /= scale;
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - cube_cr(2 * rho - 1);  // pow(2 rho - 1, 3), correctly rounded
        alpha = fmin(alpha, 2. / 3.);
        const double sf = fmax(1. / 3., alpha);
        c->lambda *= sf;
        c->ni = 2;
        c->currentChi = tempChi;
        *cur ^= 1;
    } else {
        c->lambda *= c->ni;
        c->ni *= 2;
    }
    c->rho = rho;
    c->q += 1;
    if (!(rho < 0 && c->q < 10)) {
        c->iter_done = 1;
        c->skip_trial = 1;
    }
    if (!c->iter_done) {
        c->suspended = 1;
        c->skip_iter = 1;
        c->skip_trial = 1;
        return;
    }
    log[c->it + 1] = c->currentChi;
    if (c->q == 10 || c->rho == 0 || !isfinite(c->lambda)) {
        c->stop = 1;
        c->iters = c->it + 1;
        c->skip_iter = 1;
        c->skip_trial = 1;
    } else {
        c->it += 1;
        c->iters = c->it;
    }
}

__global__ void ba_ctl_resume_kernel(BaCtl* c) {
    c->suspended = 0;
    c->skip_iter = 0;
    c->skip_trial = 0;
}

// chi2 and the LM scale in the oracle's landmark-block order (oracle/yavo_oracle_ba.c lblock_total): a workgroup of
// kNT lanes holds one block of 256 landmarks, lane t landmark 256 b + t (0.0 past L). Each workgroup runs the block's
// halving trees in LDS and publishes the totals write-through (P.part[1 + 2 b] chi2, [2 + 2 b] the landmarks' scale
// part; workgroup 0 also the free poses' scale part, tree256 over their items, at [0]); the last workgroup folds the
// block totals into 256 leaves (block b into leaf b mod 256, ascending b), runs the trees over the leaves and then
// decides the trial (device control), starts the solve (trial false), or leaves chi2 / scale in scal[0] / scal[1].
template <bool kTrial>
__device__ __forceinline__ void lblock_reduce(const BaParams& P, double chi, double sl, double sp) {
    __shared__ double red[3][kNT];
    const int t = threadIdx.x;
    red[0][t] = chi;
    red[1][t] = sl;
    red[2][t] = sp;
    __syncthreads();
    for (int off = kNT / 2; off > 0; off >>= 1) {
        if (t < off) {
            red[0][t] = red[0][t] + red[0][t + off];
            if (kTrial) {
                red[1][t] = red[1][t] + red[1][t + off];
                red[2][t] = red[2][t] + red[2][t + off];
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        st_agent(&P.part[1 + 2 * blockIdx.x], red[0][0]);
        if (kTrial) st_agent(&P.part[2 + 2 * blockIdx.x], red[1][0]);
        if (kTrial && blockIdx.x == 0) st_agent(&P.part[0], red[2][0]);
    }
    if (!ba_last_block_h(P.ticket + 1, P.ticket + 4 + kTicketGroups)) return;
    const int nb = (P.L + kNT - 1) / kNT;
    double lc = 0.0, ls = 0.0;
    for (int b = t; b < nb; b += kNT) {
        lc = lc + ld_agent(&P.part[1 + 2 * b]);
        if (kTrial) ls = ls + ld_agent(&P.part[2 + 2 * b]);
    }
    __syncthreads();  // this workgroup's own block trees are read
    red[0][t] = lc;
    red[1][t] = ls;
    __syncthreads();
    for (int off = kNT / 2; off > 0; off >>= 1) {
        if (t < off) {
            red[0][t] = red[0][t] + red[0][t + off];
            if (kTrial) red[1][t] = red[1][t] + red[1][t + off];
        }
        __syncthreads();
    }
    if (t != 0) return;
    const double chi2 = red[0][0];
    if (!kTrial) {
        if (!P.ctl) P.scal[0] = chi2;
        else ba_ctl_init(P.ctl, chi2, P.log, P.maxdiag);
        return;
    }
    const double scale = ld_agent(&P.part[0]) + red[1][0];
    if (!P.ctl) {
        P.scal[0] = chi2;
        P.scal[1] = scale;
    } else {
        ba_ctl_decide(P.ctl, chi2, scale, P.ns > 0 ? P.scal[2] != 0.0 : true, P.cur, P.log);
    }
}

// The trial step in one launch (g2o's back-substitution, oplus, the trial chi2 and the LM scale): every workgroup
// first forms all poses of the trial state in LDS (free: exp(x_p) T, fixed: T); one lane per landmark then runs
// x_l = Dinv (b_l - sum_e H_pl^T x_p) sequentially over its edges, writes X + x_l into the trial state, and sums |e|^2
// of its edges at the trial state and its three scale items x (lambda x + b) (each from 0.0, in order) for
// lblock_reduce, whose last workgroup decides the trial. The trial state is the other buffer: a rejected trial leaves
// the current one untouched (no backup / restore copies); an accepted one flips P.cur. (Until round 5 the per-edge
// |e|^2 and the scale items went through HBM to a separate tree4096 chi2 kernel: 11 us per trial.)
__global__ __launch_bounds__(kNT) void ba_step_kernel(BaParams P, BaMat3 K, double lambda) {
    extern __shared__ double sT[];  // [P][7]
    if (P.gate && *P.gate) return;  // a skipped phase of the device-driven LM
    if (P.lam) lambda = *P.lam;
    const int ns = P.ns;
    const int cur = ba_cur(P);
    const double* T0 = cur ? P.poses2 : P.poses;
    const double* X0 = cur ? P.X2 : P.X;
    double* T1 = cur ? P.poses : P.poses2;
    double* X1 = cur ? P.X : P.X2;
    const int t = threadIdx.x;
    for (int p = t; p < P.P; p += kNT) {
        double Tn[7];
        if (p < P.nf) {
#pragma unroll
            for (int i = 0; i < 7; ++i) Tn[i] = T0[7 * p + i];
        } else {
            double dT[7];
            se3_exp(P.xp + 6 * (p - P.nf), dT);
            se3_mul(dT, T0 + 7 * p, Tn);
        }
#pragma unroll
        for (int i = 0; i < 7; ++i) sT[7 * p + i] = Tn[i];
        if (blockIdx.x == 0) {
#pragma unroll
            for (int i = 0; i < 7; ++i) T1[7 * p + i] = Tn[i];
        }
    }
    // the free poses' scale items, leaf t = items k = t mod kNT in ascending k (workgroup 0)
    double sp = 0.0;
    if (blockIdx.x == 0)
        for (int k = t; k < ns; k += kNT) {
            const double x = P.xp[k];
            sp = sp + x * (lambda * x + P.bp[6 * P.nf + k]);
        }
    __syncthreads();
    const int l = blockIdx.x * kNT + t;
    double chi = 0.0, sl = 0.0;
    if (l < P.L) {
        const int k0 = P.le_off[l], k1 = P.le_off[l + 1];
        double tv[3] = {P.bl[3 * l], P.bl[3 * l + 1], P.bl[3 * l + 2]};
        double D[9];
        landmark_dinv(P, l, lambda, D);
        // the landmark's edges two at a time: indices and poses, then both edges' Jacobians and x_p loaded before
        // the subtractions (in edge order), one dependent load round per pair of edges
        for (int kb = k0; kb < k1; kb += 2) {
            int eb[2], pb[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) eb[u] = kb + u < k1 ? P.le[kb + u] : 0;
#pragma unroll
            for (int u = 0; u < 2; ++u) pb[u] = kb + u < k1 ? P.ep[eb[u]] : 0;
            double h[2][18], xv[2][6];
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (kb + u < k1 && pb[u] >= P.nf) {
                    hpl_load(P, eb[u], h[u]);
                    const double* xpp = P.xp + 6 * (pb[u] - P.nf);
#pragma unroll
                    for (int a = 0; a < 6; ++a) xv[u][a] = xpp[a];
                }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (kb + u >= k1 || pb[u] < P.nf) continue;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    double d = h[u][c] * xv[u][0];
#pragma unroll
                    for (int a = 1; a < 6; ++a) d = d + h[u][3 * a + c] * xv[u][a];
                    tv[c] = tv[c] - d;
                }
            }
        }
        double Xn[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double x = D[3 * c] * tv[0] + D[3 * c + 1] * tv[1] + D[3 * c + 2] * tv[2];
            P.xl[3 * l + c] = x;
            sl = sl + x * (lambda * x + P.bl[3 * l + c]);
            Xn[c] = X0[3 * l + c] + x;
            X1[3 * l + c] = Xn[c];
        }
        for (int kb = k0; kb < k1; kb += 2) {
            int eb[2], pb[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) eb[u] = kb + u < k1 ? P.le[kb + u] : 0;
#pragma unroll
            for (int u = 0; u < 2; ++u) pb[u] = kb + u < k1 ? P.ep[eb[u]] : 0;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (kb + u >= k1) break;
                double r[2];
                ba_error(sT + 7 * pb[u], K.v, Xn, P.meas + 2 * eb[u], r);
                chi = chi + (r[0] * r[0] + r[1] * r[1]);
            }
        }
    }
    lblock_reduce<true>(P, chi, sl, sp);
}

// the solve's first chi2 at the current estimate, in the same order: one lane per landmark over its edges. A solve
// starts in state 0 (P.poses / P.X); workgroup 0 also resets *P.cur for the kernels after it (no separate memset)
__global__ __launch_bounds__(kNT) void ba_chi2_kernel(BaParams P, BaMat3 K) {
    if (P.gate && *P.gate) return;  // a skipped phase of the device-driven LM
    if (P.cur && blockIdx.x == 0 && threadIdx.x == 0) *P.cur = 0;
    const double* T = P.poses;
    const double* X = P.X;
    const int l = blockIdx.x * kNT + threadIdx.x;
    double chi = 0.0;
    if (l < P.L) {
        const double Xl[3] = {X[3 * l], X[3 * l + 1], X[3 * l + 2]};
        for (int k = P.le_off[l]; k < P.le_off[l + 1]; ++k) {
            const int e = P.le[k];
            double r[2];
            ba_error(T + 7 * P.ep[e], K.v, Xl, P.meas + 2 * e, r);
            chi = chi + (r[0] * r[0] + r[1] * r[1]);
        }
    }
    lblock_reduce<false>(P, chi, 0.0, 0.0);
}

// after the solve: the estimate into P.poses / P.X when it ended in the other buffer
__global__ __launch_bounds__(256) void ba_finish_kernel(BaParams P) {
    if (P.gate && *P.gate) return;  // enqueued with the solve: skipped when it was suspended (the host reruns it)
    if (!P.cur || !*P.cur) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 7 * P.P) P.poses[i] = P.poses2[i];
    if (i < 3 * P.L) P.X[i] = P.X2[i];
}

}  // namespace ba

void launch_ba_ctl_resume(BaCtl* c, hipStream_t s) {
    hipLaunchKernelGGL(ba::ba_ctl_resume_kernel, dim3(1), dim3(1), 0, s, c);
}

void launch_ba_linearize(const BaParams& P, const BaMat3& K, int first, hipStream_t s) {
    const int nb = std::max(1, P.np * ba::kWG + (P.L + ba::kWLanes - 1) / ba::kWLanes);
    hipLaunchKernelGGL(ba::ba_reduce_kernel, dim3(nb), dim3(ba::kWLanes), 0, s, P, K, first);
}

void launch_ba_ldlt(const BaParams& P, hipStream_t s) {
    if (P.ns > 0 && P.ns <= ba::kLdltRegN)
        hipLaunchKernelGGL(ba::ba_ldlt_reg_kernel, dim3(1), dim3(64 * ba::kLdltWaves), 0, s, P);
    else if (P.ns > 0)
        hipLaunchKernelGGL(ba::ba_ldlt_kernel, dim3(1), dim3(256), sizeof(double) * 2 * P.ns, s, P);
}

void launch_ba_trial(const BaParams& P, const BaMat3& K, double lambda, hipStream_t s) {
    const int nb = P.np * (P.np + 1) / 2;
    if (nb > 0)
        hipLaunchKernelGGL(ba::ba_schur_kernel, dim3((nb + P.np) * ba::kWG), dim3(ba::kWLanes), 0, s, P, lambda);
    launch_ba_ldlt(P, s);
    hipLaunchKernelGGL(ba::ba_step_kernel, dim3(std::max(1, (P.L + 255) / 256)), dim3(256),
                       sizeof(double) * 7 * P.P, s, P, K, lambda);
}

void launch_ba_chi2(const BaParams& P, const BaMat3& K, hipStream_t s) {
    hipLaunchKernelGGL(ba::ba_chi2_kernel, dim3(std::max(1, (P.L + ba::kNT - 1) / ba::kNT)), dim3(ba::kNT), 0, s, P, K);
}

void launch_ba_finish(const BaParams& P, hipStream_t s) {
    const int n = std::max(7 * P.P, 3 * P.L);
    if (n > 0) hipLaunchKernelGGL(ba::ba_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, s, P);
}

}  // namespace yavo

// ---- C ABI (include/yavo/yavo_geom.h) ----

struct yv_ba {
    yv_ctx* ctx = nullptr;
    int dev = 0;
    hipStream_t st = nullptr;
    hipStream_t ctx_st = nullptr;  // the context's stream (yv_ba_set_stream(b, NULL) returns to it)
    int max_poses = 0, max_landmarks = 0, max_edges = 0;
    int64_t cv_cap = 0;
    yavo::BaParams P;
    yavo::BaMat3 K{};
    std::vector<void*> owned;
    int32_t *d_ep = nullptr, *d_el = nullptr, *d_pe_off = nullptr, *d_pe = nullptr, *d_le_off = nullptr,
            *d_le = nullptr, *d_cv_off = nullptr, *d_cv_e1 = nullptr, *d_cv_e2 = nullptr;
    double* d_meas = nullptr;
    int* d_cur = nullptr;          // the state the estimate is in (BaParams::cur)
    unsigned* d_ticket = nullptr;  // last-workgroup counters [kBaTickets]
    int64_t schur_cap = 0;         // Schur tasks P.spart / P.sticket hold
    unsigned long long* d_maxdiag = nullptr;
    double* h_scal = nullptr;  // pinned [4]
    yavo::BaCtl* d_ctl = nullptr;  // the device-driven LM's control block
    yavo::BaCtl* h_ctl = nullptr;  // pinned copy
    double* h_log = nullptr;       // pinned copy of d_log [log_cap]
    bool resumed = false;          // the last ba_solve_wait resumed a suspended solve
    int resumes = 0;               // suspended trial loops resumed since creation (yv_ba_debug_resumes)
    double* d_log = nullptr;       // [log_cap] chi2 per iteration
    int log_cap = 0;
    int device_control = 1;        // yv_ba_set_control
    bool ready = false;
};

namespace {

// [0] reduce, [1] chi2 (the last-workgroup tops); [4, 68) the reduce's groups, [68, 132) chi2's
constexpr int kBaTickets = 4 + 2 * yavo::ba::kTicketGroups;
// the global-memory LDLT keeps 2 x 6 np doubles in dynamic LDS beside ~3 KB of its own: 6 x 640 rows fit 64 KB
constexpr int kBaMaxPoses = 640;

template <class T>
int ba_alloc(yv_ba* b, T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)) != hipSuccess) {
        std::fprintf(stderr, "yavo: hipMalloc(%zu B) failed in yv_ba\n", count * sizeof(T));
        return YV_ERR_HIP;
    }
    b->owned.push_back(*p);
    return YV_OK;
}

void ba_free_one(yv_ba* b, void* p) {
    if (!p) return;
    (void)hipFree(p);
    b->owned.erase(std::remove(b->owned.begin(), b->owned.end(), p), b->owned.end());
}

// the tree4096 class totals and per-sum counters of np free poses: P.spart / P.sticket for the Schur tasks (nb upper
// blocks + np b_schur rows), P.rpart / P.rticket for the pose reduce; grown on demand
int ba_ensure_schur(yv_ba* b, int np, hipStream_t st) {
    const int64_t tasks = (int64_t)np * (np + 1) / 2 + np;
    if (tasks <= b->schur_cap) return YV_OK;
    if (hipStreamSynchronize(st) != hipSuccess) return YV_ERR_HIP;
    yavo::BaParams& Q = b->P;
    ba_free_one(b, Q.spart);
    ba_free_one(b, Q.sticket);
    ba_free_one(b, Q.rpart);
    ba_free_one(b, Q.rticket);
    Q.spart = Q.rpart = nullptr;
    Q.sticket = Q.rticket = nullptr;
    b->schur_cap = 0;
    if (ba_alloc(b, &Q.spart, (size_t)tasks * yavo::ba::kWG * 36) != YV_OK ||
        ba_alloc(b, &Q.sticket, (size_t)tasks) != YV_OK ||
        ba_alloc(b, &Q.rpart, (size_t)np * yavo::ba::kWG * 27) != YV_OK ||
        ba_alloc(b, &Q.rticket, (size_t)np) != YV_OK ||
        hipMemsetAsync(Q.sticket, 0, sizeof(unsigned) * tasks, st) != hipSuccess ||
        hipMemsetAsync(Q.rticket, 0, sizeof(unsigned) * (np > 0 ? np : 1), st) != hipSuccess)
        return YV_ERR_HIP;
    b->schur_cap = tasks;
    return YV_OK;
}

// the last-workgroup counters return to 0 at the end of every launch that uses them; a launch that never finished
// (an error, a fault) could leave one non-zero, and every later solve would then skip that launch's last-workgroup
// work silently -- so a new problem, and every failed enqueue, starts from zeroed counters (a few hundred bytes)
int ba_reset_tickets(yv_ba* b, hipStream_t st) {
    const yavo::BaParams& Q = b->P;
    if (hipMemsetAsync(b->d_ticket, 0, kBaTickets * sizeof(unsigned), st) != hipSuccess) return YV_ERR_HIP;
    if (b->schur_cap > 0 && (hipMemsetAsync(Q.sticket, 0, sizeof(unsigned) * b->schur_cap, st) != hipSuccess ||
                             hipMemsetAsync(Q.rticket, 0, sizeof(unsigned) * std::max(1, Q.np), st) != hipSuccess))
        return YV_ERR_HIP;
    return YV_OK;
}

int ba_sync_scal(yv_ba* b, int n) {
    if (hipMemcpyAsync(b->h_scal, b->P.scal, sizeof(double) * n, hipMemcpyDeviceToHost, b->st) != hipSuccess ||
        hipStreamSynchronize(b->st) != hipSuccess)
        return YV_ERR_HIP;
    return YV_OK;
}

}  // namespace

extern "C" int yv_ba_create(yv_ctx* ctx, int max_poses, int max_landmarks, int max_edges, yv_ba** out) {
    if (!out) return YV_ERR_INVALID;
    *out = nullptr;
    // the reduced pose system (6 max_poses)^2 doubles is factorised by one workgroup with its vectors in LDS
    if (!ctx || max_poses < 1 || max_poses > kBaMaxPoses || max_landmarks < 0 || max_edges < 0) return YV_ERR_INVALID;
    yv_ba* b = new yv_ba();
    b->ctx = ctx;
    b->dev = yavo::ctx_device(ctx);
    b->st = yavo::ctx_stream(ctx);
    b->ctx_st = b->st;
    b->max_poses = max_poses;
    b->max_landmarks = max_landmarks;
    b->max_edges = max_edges;
    if (hipSetDevice(b->dev) != hipSuccess) {
        delete b;
        return YV_ERR_HIP;
    }
    const size_t P = max_poses, L = max_landmarks, E = max_edges, ns = 6 * P;
    yavo::BaParams& Q = b->P;
    int rc = YV_OK;
    rc |= ba_alloc(b, &b->d_ep, E);
    rc |= ba_alloc(b, &b->d_el, E);
    rc |= ba_alloc(b, &b->d_meas, 2 * E);
    rc |= ba_alloc(b, &b->d_pe_off, P + 1);
    rc |= ba_alloc(b, &b->d_pe, E);
    rc |= ba_alloc(b, &b->d_le_off, L + 1);
    rc |= ba_alloc(b, &b->d_le, E);
    rc |= ba_alloc(b, &b->d_cv_off, P * P + 1);
    rc |= ba_alloc(b, &Q.poses, 7 * P);
    rc |= ba_alloc(b, &Q.X, 3 * L);
    rc |= ba_alloc(b, &Q.poses2, 7 * P);
    rc |= ba_alloc(b, &Q.X2, 3 * L);
    rc |= ba_alloc(b, &b->d_cur, 1);
    rc |= ba_alloc(b, &b->d_ticket, kBaTickets);
    rc |= ba_alloc(b, &Q.part, 1 + 2 * std::max<size_t>(1, (L + yavo::ba::kNT - 1) / yavo::ba::kNT));
    rc |= ba_alloc(b, &Q.err, 2 * E);
    rc |= ba_alloc(b, &Q.Jp, 12 * E);
    rc |= ba_alloc(b, &Q.Jl, 6 * E);
    rc |= ba_alloc(b, &Q.Hpp, 36 * P);
    rc |= ba_alloc(b, &Q.bp, 6 * P);
    rc |= ba_alloc(b, &Q.Hll, 9 * L);
    rc |= ba_alloc(b, &Q.bl, 3 * L);
    rc |= ba_alloc(b, &Q.S, ns * ns);
    rc |= ba_alloc(b, &Q.bs, ns);
    rc |= ba_alloc(b, &Q.xp, ns);
    rc |= ba_alloc(b, &Q.xl, 3 * L);
    rc |= ba_alloc(b, &Q.tr, ns);
    rc |= ba_alloc(b, &Q.scal, 16);
    rc |= ba_alloc(b, &b->d_maxdiag, 1);
    rc |= ba_alloc(b, &b->d_ctl, 1);
    if (rc == YV_OK && hipHostMalloc(reinterpret_cast<void**>(&b->h_scal), 4 * sizeof(double)) != hipSuccess)
        rc = YV_ERR_HIP;
    if (rc == YV_OK && hipHostMalloc(reinterpret_cast<void**>(&b->h_ctl), sizeof(yavo::BaCtl)) != hipSuccess)
        rc = YV_ERR_HIP;
    if (rc == YV_OK && hipHostMalloc(reinterpret_cast<void**>(&b->h_log), sizeof(double) * 65) != hipSuccess)
        rc = YV_ERR_HIP;
    // sized up front where that is small, so a solve loop's first iterations do not allocate (each growth
    // synchronises the stream and frees device memory, which synchronises the device): the Schur partials of up to 64
    // free poses, the window graph's co-visibility lists (3 per landmark) and a 64-iteration chi2 log
    if (rc == YV_OK && max_poses <= 64) rc |= ba_ensure_schur(b, max_poses, b->st);
    if (rc == YV_OK && max_landmarks > 0) {
        rc |= ba_alloc(b, &b->d_cv_e1, 3 * L);
        rc |= ba_alloc(b, &b->d_cv_e2, 3 * L);
        if (rc == YV_OK) b->cv_cap = 3 * (int64_t)L;
    }
    if (rc == YV_OK) {
        rc |= ba_alloc(b, &b->d_log, 65);
        if (rc == YV_OK) b->log_cap = 65;
    }
    if (rc == YV_OK && (hipMemsetAsync(b->d_ticket, 0, kBaTickets * sizeof(unsigned), b->st) != hipSuccess ||
                        hipMemsetAsync(b->d_cur, 0, sizeof(int), b->st) != hipSuccess ||
                        hipStreamSynchronize(b->st) != hipSuccess))
        rc = YV_ERR_HIP;
    if (rc != YV_OK) {
        yv_ba_destroy(b);
        return YV_ERR_HIP;
    }
    Q.cur = b->d_cur;
    Q.ticket = b->d_ticket;
    Q.maxdiag = b->d_maxdiag;
    *out = b;
    return YV_OK;
}

extern "C" void yv_ba_destroy(yv_ba* b) {
    if (!b) return;
    (void)hipSetDevice(b->dev);
    (void)hipStreamSynchronize(b->st);
    for (void* p : b->owned) (void)hipFree(p);
    if (b->h_scal) (void)hipHostFree(b->h_scal);
    if (b->h_ctl) (void)hipHostFree(b->h_ctl);
    if (b->h_log) (void)hipHostFree(b->h_log);
    delete b;
}

extern "C" int yv_ba_set_stream(yv_ba* b, void* stream) {
    if (!b) return YV_ERR_INVALID;
    if (hipSetDevice(b->dev) != hipSuccess || hipStreamSynchronize(b->st) != hipSuccess) return YV_ERR_HIP;
    b->st = stream ? reinterpret_cast<hipStream_t>(stream) : b->ctx_st;
    return YV_OK;
}

extern "C" int yv_ba_set_problem(yv_ba* b, int n_poses, int n_fixed, int n_landmarks, const int32_t* edge_pose,
                                 const int32_t* edge_landmark, const double* meas, int n_edges, const double K[9]) {
    if (!b || !K || n_poses < 1 || n_poses > b->max_poses || n_fixed < 0 || n_fixed > n_poses || n_landmarks < 0 ||
        n_landmarks > b->max_landmarks || n_edges < 0 || n_edges > b->max_edges ||
        (n_edges > 0 && (!edge_pose || !edge_landmark || !meas)))
        return YV_ERR_INVALID;
    for (int i = 0; i < 9; ++i)
        if (!std::isfinite(K[i])) return YV_ERR_INVALID;
    for (int e = 0; e < n_edges; ++e)
        if (edge_pose[e] < 0 || edge_pose[e] >= n_poses || edge_landmark[e] < 0 || edge_landmark[e] >= n_landmarks)
            return YV_ERR_INVALID;
    if (hipSetDevice(b->dev) != hipSuccess) return YV_ERR_HIP;
    b->ready = false;
    const int P = n_poses, L = n_landmarks, E = n_edges;
    // edges per pose / per landmark in edge order; co-visibility per pose pair (p1 <= p2), landmarks ascending
    std::vector<int32_t> pe_off(P + 1, 0), le_off(L + 1, 0), pe(std::max(E, 1)), le(std::max(E, 1));
    for (int e = 0; e < E; ++e) {
        pe_off[edge_pose[e] + 1]++;
        le_off[edge_landmark[e] + 1]++;
    }
    for (int p = 0; p < P; ++p) pe_off[p + 1] += pe_off[p];
    for (int l = 0; l < L; ++l) le_off[l + 1] += le_off[l];
    {
        std::vector<int32_t> fp(pe_off.begin(), pe_off.end() - 1), fl(le_off.begin(), le_off.end() - 1);
        for (int e = 0; e < E; ++e) {
            pe[fp[edge_pose[e]]++] = e;
            le[fl[edge_landmark[e]]++] = e;
        }
    }
    const int64_t NB = (int64_t)P * P;
    std::vector<int32_t> cv_off(NB + 1, 0);
    for (int l = 0; l < L; ++l)
        for (int a = le_off[l]; a < le_off[l + 1]; ++a)
            for (int c = le_off[l]; c < le_off[l + 1]; ++c) {
                const int p1 = edge_pose[le[a]], p2 = edge_pose[le[c]];
                if (p1 <= p2) cv_off[(int64_t)p1 * P + p2 + 1]++;
            }
    int64_t nc = 0;
    for (int64_t i = 0; i < NB; ++i) {
        nc += cv_off[i + 1];
        if (nc > INT32_MAX) return YV_ERR_CAPACITY;
        cv_off[i + 1] = (int32_t)nc;
    }
    std::vector<int32_t> cv_e1(std::max<int64_t>(nc, 1)), cv_e2(std::max<int64_t>(nc, 1));
    {
        std::vector<int32_t> fill(cv_off.begin(), cv_off.end() - 1);
        for (int l = 0; l < L; ++l)
            for (int a = le_off[l]; a < le_off[l + 1]; ++a)
                for (int c = le_off[l]; c < le_off[l + 1]; ++c) {
                    const int p1 = edge_pose[le[a]], p2 = edge_pose[le[c]];
                    if (p1 > p2) continue;
                    const int32_t k = fill[(int64_t)p1 * P + p2]++;
                    cv_e1[k] = le[a];
                    cv_e2[k] = le[c];
                }
    }
    if (nc > b->cv_cap) {
        ba_free_one(b, b->d_cv_e1);
        ba_free_one(b, b->d_cv_e2);
        b->d_cv_e1 = b->d_cv_e2 = nullptr;
        b->cv_cap = 0;
        if (ba_alloc(b, &b->d_cv_e1, nc) != YV_OK || ba_alloc(b, &b->d_cv_e2, nc) != YV_OK) return YV_ERR_HIP;
        b->cv_cap = nc;
    }
    auto h2d = [&](void* d, const void* h, size_t bytes) {
        return bytes == 0 || hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, b->st) == hipSuccess;
    };
    bool ok = h2d(b->d_ep, edge_pose, sizeof(int32_t) * E) && h2d(b->d_el, edge_landmark, sizeof(int32_t) * E) &&
              h2d(b->d_meas, meas, sizeof(double) * 2 * E) && h2d(b->d_pe_off, pe_off.data(), 4 * (P + 1)) &&
              h2d(b->d_pe, pe.data(), 4 * (size_t)E) && h2d(b->d_le_off, le_off.data(), 4 * (size_t)(L + 1)) &&
              h2d(b->d_le, le.data(), 4 * (size_t)E) && h2d(b->d_cv_off, cv_off.data(), 4 * (size_t)(NB + 1)) &&
              h2d(b->d_cv_e1, cv_e1.data(), 4 * (size_t)nc) && h2d(b->d_cv_e2, cv_e2.data(), 4 * (size_t)nc);
    // the pageable sources die with this call
    if (!ok || hipStreamSynchronize(b->st) != hipSuccess) return YV_ERR_HIP;
    yavo::BaParams& Q = b->P;
    Q.P = P;
    Q.nf = n_fixed;
    Q.np = P - n_fixed;
    Q.ns = 6 * Q.np;
    if (ba_ensure_schur(b, Q.np, b->st) != YV_OK || ba_reset_tickets(b, b->st) != YV_OK) return YV_ERR_HIP;
    Q.L = L;
    Q.E = E;
    Q.ep = b->d_ep;
    Q.el = b->d_el;
    Q.meas = b->d_meas;
    Q.pe_off = b->d_pe_off;
    Q.pe = b->d_pe;
    Q.le_off = b->d_le_off;
    Q.le = b->d_le;
    Q.cv_off = b->d_cv_off;
    Q.cv_e1 = b->d_cv_e1;
    Q.cv_e2 = b->d_cv_e2;
    std::memcpy(b->K.v, K, sizeof b->K.v);
    b->ready = true;
    return YV_OK;
}

// g2o OptimizationAlgorithmLevenberg::solve, as or_ba_lm: the host runs the damping control on the device's chi2
// and scale (bit-identical double arithmetic), the device everything per edge / landmark / pose
namespace {

// The LM of yv_ba_solve with its control on the device (default): the host enqueues every iteration's kernels
// without waiting -- linearise + H / b (whose last workgroup begins the iteration), one damping trial (Dinv / W,
// Schur, LDLT, step into the trial state, chi2 + scale, whose last workgroup decides and ends the iteration) -- and
// the control block (lambda, ni, currentChi, stop / accept) gates the kernels. g2o's trial loop usually accepts its
// first trial; an iteration that needs more suspends the solve (every later kernel skips) and the host resumes it.
// One read-back per solve, plus one per suspended trial loop.
// poses / landmarks: host in / out; both nullptr: the problem's poses and landmarks are already in Q.poses / Q.X on
// the device (yv_ba_window_solve) and stay there.
// the enqueue half: chi2 at the start, then every iteration with one trial slot, then the control block's read-back
// (asynchronous: ba_solve_wait collects it)
int ba_solve_enqueue_(yv_ba* b, const double* poses, const double* landmarks, int max_iters);

int ba_solve_enqueue(yv_ba* b, const double* poses, const double* landmarks, int max_iters) {
    const int rc = ba_solve_enqueue_(b, poses, landmarks, max_iters);
    if (rc != YV_OK) (void)ba_reset_tickets(b, b->st);
    return rc;
}

int ba_solve_enqueue_(yv_ba* b, const double* poses, const double* landmarks, int max_iters) {
    yavo::BaParams& Q = b->P;
    const size_t pb = sizeof(double) * 7 * Q.P, xb = sizeof(double) * 3 * Q.L;
    hipStream_t st = b->st;
    if (max_iters + 1 > b->log_cap) {
        if (hipStreamSynchronize(st) != hipSuccess) return YV_ERR_HIP;
        ba_free_one(b, b->d_log);
        b->d_log = nullptr;
        b->log_cap = 0;
        if (ba_alloc(b, &b->d_log, (size_t)max_iters + 1) != YV_OK) return YV_ERR_HIP;
        if (b->h_log) (void)hipHostFree(b->h_log);
        b->h_log = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&b->h_log), sizeof(double) * (max_iters + 1)) != hipSuccess)
            return YV_ERR_HIP;
        b->log_cap = max_iters + 1;
    }
    yavo::BaCtl* c = b->d_ctl;
    yavo::BaParams Pc = Q;
    Pc.ctl = c;
    Pc.log = b->d_log;
    yavo::BaParams Pit = Pc, Ptr = Pc;
    Pit.gate = &c->skip_iter;
    Ptr.gate = &c->skip_trial;
    Ptr.lam = &c->lambda;
    // (*Q.cur is reset by the first kernel, ba_chi2_kernel)
    if (poses && (hipMemcpyAsync(Q.poses, poses, pb, hipMemcpyHostToDevice, st) != hipSuccess ||
                  (xb && hipMemcpyAsync(Q.X, landmarks, xb, hipMemcpyHostToDevice, st) != hipSuccess)))
        return YV_ERR_HIP;
    yavo::launch_ba_chi2(Pc, b->K, st);
    for (int it = 0; it < max_iters; ++it) {
        yavo::launch_ba_linearize(Pit, b->K, it == 0 ? 1 : 0, st);
        yavo::launch_ba_trial(Ptr, b->K, 0.0, st);
    }
    // the end of the solve in the same submission (skipped on the device when it was suspended; ba_solve_wait then
    // resumes it and reruns these), so an unsuspended solve is collected with one wait
    yavo::BaParams Pf = Q;
    Pf.gate = &c->suspended;
    yavo::launch_ba_finish(Pf, st);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(b->h_log, b->d_log, sizeof(double) * (max_iters + 1), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(b->h_ctl, c, sizeof(yavo::BaCtl), hipMemcpyDeviceToHost, st) != hipSuccess)
        return YV_ERR_HIP;
    return YV_OK;
}

// the collecting half: waits for the control block, resumes a suspended trial loop (one read-back each) until the
// solve ends, then the estimate into Q.poses / Q.X (host copies when poses != nullptr) and the chi2 log
int ba_solve_wait(yv_ba* b, double* poses, double* landmarks, int max_iters, double* chi2_log, int* iters) {
    yavo::BaParams& Q = b->P;
    const size_t pb = sizeof(double) * 7 * Q.P, xb = sizeof(double) * 3 * Q.L;
    hipStream_t st = b->st;
    yavo::BaCtl* c = b->d_ctl;
    yavo::BaParams Pc = Q;
    Pc.ctl = c;
    Pc.log = b->d_log;
    yavo::BaParams Pit = Pc, Ptr = Pc;
    Pit.gate = &c->skip_iter;
    Ptr.gate = &c->skip_trial;
    Ptr.lam = &c->lambda;
    b->resumed = false;
    for (;;) {
        if (hipStreamSynchronize(st) != hipSuccess) return YV_ERR_HIP;
        if (!b->h_ctl->suspended) break;
        b->resumed = true;
        ++b->resumes;
        yavo::launch_ba_ctl_resume(c, st);  // the suspended iteration's trial loop continues at its trial q
        const int first = b->h_ctl->it;
        for (int it = first; it < max_iters; ++it) {
            if (it != first) yavo::launch_ba_linearize(Pit, b->K, 0, st);
            yavo::launch_ba_trial(Ptr, b->K, 0.0, st);
        }
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(b->h_ctl, c, sizeof(yavo::BaCtl), hipMemcpyDeviceToHost, st) != hipSuccess)
            return YV_ERR_HIP;
    }
    const int n_it = max_iters > 0 ? b->h_ctl->iters : 0;
    if (b->resumed) {
        yavo::launch_ba_finish(Q, st);
        if (hipMemcpyAsync(b->h_log, b->d_log, sizeof(double) * (max_iters + 1), hipMemcpyDeviceToHost, st) !=
            hipSuccess)
            return YV_ERR_HIP;
    }
    if (poses && (hipMemcpyAsync(poses, Q.poses, pb, hipMemcpyDeviceToHost, st) != hipSuccess ||
                  (xb && hipMemcpyAsync(landmarks, Q.X, xb, hipMemcpyDeviceToHost, st) != hipSuccess)))
        return YV_ERR_HIP;
    if ((b->resumed || poses) && hipStreamSynchronize(st) != hipSuccess) return YV_ERR_HIP;
    if (chi2_log) std::memcpy(chi2_log, b->h_log, sizeof(double) * (n_it + 1));
    if (iters) *iters = n_it;
    return YV_OK;
}

// The LM of yv_ba_solve with its control on the device (default): the host enqueues every iteration's kernels
// without waiting -- linearise + H / b (whose last workgroup begins the iteration), one damping trial (Schur, LDLT,
// step into the trial state, chi2 + scale, whose last workgroup decides and ends the iteration) -- and the control
// block (lambda, ni, currentChi, stop / accept) gates the kernels. g2o's trial loop usually accepts its first trial;
// an iteration that needs more suspends the solve (every later kernel skips) and the host resumes it. One read-back
// per solve, plus one per suspended trial loop.
// poses / landmarks: host in / out; both nullptr: the problem's poses and landmarks are already in Q.poses / Q.X on
// the device (yv_ba_window_solve) and stay there.
int ba_solve_device(yv_ba* b, double* poses, double* landmarks, int max_iters, double* chi2_log, int* iters) {
    const int rc = ba_solve_enqueue(b, poses, landmarks, max_iters);
    if (rc != YV_OK) return rc;
    return ba_solve_wait(b, poses, landmarks, max_iters, chi2_log, iters);
}

}  // namespace

extern "C" int yv_ba_set_control(yv_ba* b, int on_device) {
    if (!b || on_device < 0 || on_device > 1) return YV_ERR_INVALID;
    b->device_control = on_device;
    return YV_OK;
}

extern "C" int yv_ba_solve(yv_ba* b, double* poses, double* landmarks, int max_iters, double* chi2_log, int* iters) {
    if (!b || !b->ready || !poses || (b->P.L > 0 && !landmarks) || max_iters < 0) return YV_ERR_INVALID;
    if (hipSetDevice(b->dev) != hipSuccess) return YV_ERR_HIP;
    if (b->device_control) return ba_solve_device(b, poses, landmarks, max_iters, chi2_log, iters);
    yavo::BaParams& Q = b->P;
    const size_t pb = sizeof(double) * 7 * Q.P, xb = sizeof(double) * 3 * Q.L;
    hipStream_t st = b->st;
    int cur = 0;  // the state the estimate is in (the device's *Q.cur, which the host sets)
    if (hipMemsetAsync(b->d_cur, 0, sizeof(int), st) != hipSuccess ||
        hipMemcpyAsync(Q.poses, poses, pb, hipMemcpyHostToDevice, st) != hipSuccess ||
        (xb && hipMemcpyAsync(Q.X, landmarks, xb, hipMemcpyHostToDevice, st) != hipSuccess))
        return YV_ERR_HIP;
    yavo::launch_ba_chi2(Q, b->K, st);
    if (ba_sync_scal(b, 1) != YV_OK) return YV_ERR_HIP;
    double currentChi = b->h_scal[0];
    if (chi2_log) chi2_log[0] = currentChi;
    double lambda = 0, ni = 2;
    int it;
    for (it = 0; it < max_iters; ++it) {
        if (it == 0 && hipMemsetAsync(b->d_maxdiag, 0, sizeof(unsigned long long), st) != hipSuccess) return YV_ERR_HIP;
        yavo::launch_ba_linearize(Q, b->K, it == 0 ? 1 : 0, st);
        if (it == 0) {
            unsigned long long bits = 0;
            if (hipMemcpyAsync(&bits, b->d_maxdiag, sizeof bits, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return YV_ERR_HIP;
            double maxd;
            std::memcpy(&maxd, &bits, sizeof maxd);
            lambda = 1e-5 * maxd;
            ni = 2;
        }
        double rho = 0;
        int q = 0;
        do {
            yavo::launch_ba_trial(Q, b->K, lambda, st);
            if (hipGetLastError() != hipSuccess || ba_sync_scal(b, 3) != YV_OK) return YV_ERR_HIP;
            double tempChi = b->h_scal[0];
            const bool ok2 = Q.ns > 0 ? b->h_scal[2] != 0.0 : true;
            if (!ok2) tempChi = DBL_MAX;
            rho = currentChi - tempChi;
            double scale = b->h_scal[1];
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - yavo::cube_cr(2 * rho - 1);  // pow(2 rho - 1, 3), correctly rounded
                alpha = fmin(alpha, 2. / 3.);
                const double sf = fmax(1. / 3., alpha);
                lambda *= sf;
                ni = 2;
                currentChi = tempChi;
                cur ^= 1;  // the trial state becomes the estimate
                if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(b->d_cur), cur, 1, st) != hipSuccess)
                    return YV_ERR_HIP;
            } else {
                lambda *= ni;
                ni *= 2;
            }
            q++;
        } while (rho < 0 && q < 10);
        if (chi2_log) chi2_log[it + 1] = currentChi;
        if (q == 10 || rho == 0 || !std::isfinite(lambda)) {
            ++it;
            break;
        }
    }
    yavo::launch_ba_finish(Q, st);
    if (hipMemcpyAsync(poses, Q.poses, pb, hipMemcpyDeviceToHost, st) != hipSuccess ||
        (xb && hipMemcpyAsync(landmarks, Q.X, xb, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return YV_ERR_HIP;
    if (iters) *iters = it;
    return YV_OK;
}

// diagnostics: copy one of the workspace's device buffers (as left by the last yv_ba_solve) to the host
extern "C" int yv_ba_debug_resumes(yv_ba* b) { return b ? b->resumes : -1; }

extern "C" int yv_ba_debug_read(yv_ba* b, int which, double* dst, int64_t count) {
    if (!b || !b->ready || !dst || count < 0) return YV_ERR_INVALID;
    const yavo::BaParams& Q = b->P;
    // which = 3 (H_pl), 4 (W) and 9 (Dinv) are no longer stored (formed where they are read): YV_ERR_INVALID
    if (which == 3 || which == 4 || which == 9) return YV_ERR_INVALID;
    double* const bufs[] = {Q.err, Q.Jp, Q.Jl, nullptr, nullptr, Q.Hpp, Q.bp, Q.Hll, Q.bl, nullptr, Q.S, Q.bs, Q.xp, Q.xl,
                            Q.poses, Q.X, Q.scal};
    const int64_t sizes[] = {2LL * Q.E, 12LL * Q.E, 6LL * Q.E, 18LL * Q.E, 18LL * Q.E, 36LL * Q.P, 6LL * Q.P,
                             9LL * Q.L, 3LL * Q.L, 9LL * Q.L, (int64_t)Q.ns * Q.ns, Q.ns, Q.ns, 3LL * Q.L,
                             7LL * Q.P, 3LL * Q.L, 16};
    if (which < 0 || which >= (int)(sizeof sizes / sizeof sizes[0]) || count > sizes[which]) return YV_ERR_INVALID;
    if (hipSetDevice(b->dev) != hipSuccess || hipStreamSynchronize(b->st) != hipSuccess) return YV_ERR_HIP;
    if (count && hipMemcpy(dst, bufs[which], sizeof(double) * count, hipMemcpyDeviceToHost) != hipSuccess)
        return YV_ERR_HIP;
    return YV_OK;
}


#ifdef YAVO_LM_PROFILE
// profiling builds only (lib/libyavo_prof.so): LDLT phase cycles per wave [8][8], summed since the last call (reset)
extern "C" int yv_debug_ldlt_prof(unsigned long long* out) {
    unsigned long long z[yavo::ba::kLdltWaves * 8] = {};
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(out, HIP_SYMBOL(yavo::ba::g_ldlt_prof), sizeof z) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(yavo::ba::g_ldlt_prof), z, sizeof z) != hipSuccess)
        return -2;
    return 0;
}
#endif

extern "C" int yv_ba_debug_ldlt(yv_ctx* ctx, const double* S, int n, const double* b, double* x, int* ok) {
    if (!ctx || !S || !b || !x || !ok || n < 1 || n > 6 * kBaMaxPoses) return YV_ERR_INVALID;
    if (hipSetDevice(yavo::ctx_device(ctx)) != hipSuccess) return YV_ERR_HIP;
    hipStream_t st = yavo::ctx_stream(ctx);
    double *dS = nullptr, *db = nullptr, *dx = nullptr, *ds = nullptr;
    int32_t* dtr = nullptr;
    const size_t nn = (size_t)n * n;
    int rc = YV_OK;
    if (hipMalloc(reinterpret_cast<void**>(&dS), sizeof(double) * nn) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&db), sizeof(double) * n) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&dx), sizeof(double) * n) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&ds), sizeof(double) * 16) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&dtr), sizeof(int32_t) * n) != hipSuccess)
        rc = YV_ERR_HIP;
    double scal[4] = {0, 0, 0, 0};
    if (rc == YV_OK) {
        yavo::BaParams Q{};
        Q.ns = n;
        Q.S = dS;
        Q.bs = db;
        Q.xp = dx;
        Q.scal = ds;
        Q.tr = dtr;
        if (hipMemcpyAsync(dS, S, sizeof(double) * nn, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(db, b, sizeof(double) * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemsetAsync(ds, 0, sizeof(double) * 16, st) != hipSuccess)
            rc = YV_ERR_HIP;
        if (rc == YV_OK) {
            yavo::launch_ba_ldlt(Q, st);
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(x, dx, sizeof(double) * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(scal, ds, sizeof scal, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                rc = YV_ERR_HIP;
        }
    }
    for (void* p : {(void*)dS, (void*)db, (void*)dx, (void*)ds, (void*)dtr})
        if (p) (void)hipFree(p);
    if (rc == YV_OK) *ok = scal[2] != 0.0 ? 1 : 0;
    return rc;
}

// ------------------------------------------------------------------------------------------------
// The sliding BA window of the chained stereo front end, assembled on the device (ya_vo_amd/sequence.py
// window_problem / apply_window / frame_records_from_block, restated): frame records in HBM, the graph's index
// arrays from per-frame counts (every landmark is seen by its own frame and the one before), no host round trip.
// ------------------------------------------------------------------------------------------------
namespace {

// Sophus SE3d::inverse on data() = {qx, qy, qz, qw, tx, ty, tz}: SO3(q*) renormalised, -t rotated as Eigen's
// Quaternion * Vector3 (uv = 2 (q.vec x v); v + w uv + q.vec x uv): or_se3_inverse / ya_vo_amd/sequence.py
// se3_inverse, operation for operation (no contraction: -ffp-contract=off; sqrt and / correctly rounded)
__device__ void se3_inverse_dev(const double* T, double* o) {
    double x = -T[0], y = -T[1], z = -T[2], w = T[3];
    const double len = sqrt((x * x + z * z) + (y * y + w * w));  // the SO3 constructor's normalisation
    x = x / len;
    y = y / len;
    z = z / len;
    w = w / len;
    const double vx = T[4] * -1.0, vy = T[5] * -1.0, vz = T[6] * -1.0;
    double ux = y * vz - z * vy, uy = z * vx - x * vz, uz = x * vy - y * vx;
    ux += ux;
    uy += uy;
    uz += uz;
    const double cx = y * uz - z * uy, cy = z * ux - x * uz, cz = x * uy - y * ux;
    o[0] = x;
    o[1] = y;
    o[2] = z;
    o[3] = w;
    o[4] = vx + w * ux + cx;
    o[5] = vy + w * uy + cy;
    o[6] = vz + w * uz + cz;
}

constexpr int kWinMaxPoses = 128;

// one workgroup per keyframe of a placed block: its T_wc, landmarks and their two observations into the records
__global__ __launch_bounds__(256) void win_add_kernel(const uint8_t* __restrict__ block, const double* __restrict__ edge_uv,
                                                      const int32_t* __restrict__ edge_query,
                                                      const uint8_t* __restrict__ matches, int max_kp, int64_t g0,
                                                      int64_t cap, int max_lm, double* __restrict__ T, int32_t* __restrict__ cnt,
                                                      int32_t* __restrict__ edge, double* __restrict__ X,
                                                      double* __restrict__ uvo, double* __restrict__ uvp,
                                                      int64_t* __restrict__ info) {
    const yv_map_header* h = reinterpret_cast<const yv_map_header*>(block);
    const int j = blockIdx.x;
    if (j == 0 && threadIdx.x == 0) info[0] = h->n_kf;
    if (j >= h->n_kf) return;
    const yv_keyframe* kf = reinterpret_cast<const yv_keyframe*>(block + sizeof(yv_map_header)) + j;
    const int64_t lmo = ((int64_t)sizeof(yv_map_header) + (int64_t)h->max_kf * (int64_t)sizeof(yv_keyframe) + 255) & ~255ll;
    const yv_landmark* lm = reinterpret_cast<const yv_landmark*>(block + lmo) + (int64_t)j * h->lm_stride;
    const int64_t g = kf->frame_id, s = g - g0;
    const int64_t k64 = g - h->first_frame;
    if (s < 0 || s >= cap || k64 < 0 || k64 >= h->n_frames) return;  // not a frame of the reserved range
    const int k = (int)k64;
    const int n = min(kf->n_landmarks, max_lm);
    if (threadIdx.x < 7) T[s * 7 + threadIdx.x] = kf->T[threadIdx.x];
    if (threadIdx.x == 0) {
        cnt[s] = n;
        info[1 + 2 * j] = g;
        info[2 + 2 * j] = n;
    }
    for (int l = threadIdx.x; l < n; l += 256) {
        const int e = (int)(lm[l].id & 0xFFFF);
        const int64_t o = s * max_lm + l;
        edge[o] = e;
        X[3 * o] = lm[l].X[0];
        X[3 * o + 1] = lm[l].X[1];
        X[3 * o + 2] = lm[l].X[2];
        const int64_t ke = (int64_t)k * max_kp + e;
        uvp[2 * o] = edge_uv[2 * ke];
        uvp[2 * o + 1] = edge_uv[2 * ke + 1];
        const int q = edge_query[ke];
        const uint8_t* rec = matches + ((int64_t)(2 * k) * max_kp + q) * 100;  // the temporal pair's Matches
        int32_t px[2];
        __builtin_memcpy(px, rec + 48, 8);  // Matches::pt2 {x, y}
        uvo[2 * o] = (double)px[0];
        uvo[2 * o + 1] = (double)px[1];
    }
}

// one workgroup per exported frame: the record's T_wc and landmarks as a map block of a sequence shard (yavo_map.h
// placed = 2: the shard's own T_wc / X_w, placed after the shards before it by yv_map_place)
__global__ __launch_bounds__(256) void win_export_kernel(const double* __restrict__ T, const int32_t* __restrict__ cnt,
                                                         const int32_t* __restrict__ edge, const double* __restrict__ X,
                                                         int64_t s_first, int n, int64_t s_chunk, int64_t id0,
                                                         int max_lm, int max_kf, int lm_stride, uint8_t* __restrict__ block) {
    yv_map_header* h = reinterpret_cast<yv_map_header*>(block);
    const int j = blockIdx.x;
    if (j == 0 && threadIdx.x == 0) {
        for (int i = 0; i < 7; ++i) h->chunk[i] = T[7 * s_chunk + i];
        h->first_frame = id0;
        h->n_frames = n;
        h->n_kf = n;
        h->kf_every = 1;
        h->lm_stride = lm_stride;
        h->max_kf = max_kf;
        h->placed = 2;
        for (int i = 0; i < 5; ++i) h->pad[i] = 0.0;
    }
    if (j >= n) return;
    const int64_t s = s_first + j, g = id0 + j;
    yv_keyframe* kf = reinterpret_cast<yv_keyframe*>(block + sizeof(yv_map_header)) + j;
    const int64_t lmo = ((int64_t)sizeof(yv_map_header) + (int64_t)max_kf * (int64_t)sizeof(yv_keyframe) + 255) & ~255ll;
    yv_landmark* lm = reinterpret_cast<yv_landmark*>(block + lmo) + (int64_t)j * lm_stride;
    const int c = min(max(cnt[s], 0), lm_stride);
    if (threadIdx.x < 7) kf->T[threadIdx.x] = T[7 * s + threadIdx.x];
    if (threadIdx.x == 0) {
        kf->frame_id = g;
        kf->n_landmarks = c;
        kf->pad = 0;
    }
    for (int l = threadIdx.x; l < c; l += 256) {
        const int64_t o = s * max_lm + l;
        lm[l].id = (g << 16) | (int64_t)edge[o];
        lm[l].X[0] = X[3 * o];
        lm[l].X[1] = X[3 * o + 1];
        lm[l].X[2] = X[3 * o + 2];
    }
}

struct WinFrames {
    int P;
    int64_t s0;                   // store index of the window's first frame
    int32_t c[kWinMaxPoses];      // landmarks owned by pose i (0 for the first pose)
    int32_t base[kWinMaxPoses];   // their first landmark index
    int32_t pe0[kWinMaxPoses];    // pe_off of pose i
    int32_t row[kWinMaxPoses];    // first co-visibility entry of row p1 = i
};

// the graph of window_problem: poses (T_cw = inverse T_wc), landmarks, edges (own frame, then the frame before),
// edges per pose / landmark and the co-visibility lists, each entry written by its landmark's thread
__global__ __launch_bounds__(256) void win_build_kernel(WinFrames F, int L, int max_lm, const double* __restrict__ T,
                                                        const double* __restrict__ Xs, const double* __restrict__ uvo,
                                                        const double* __restrict__ uvp, double* __restrict__ poses,
                                                        double* __restrict__ X, int32_t* __restrict__ ep,
                                                        int32_t* __restrict__ el, double* __restrict__ meas,
                                                        int32_t* __restrict__ le_off, int32_t* __restrict__ le,
                                                        int32_t* __restrict__ pe, int32_t* __restrict__ cv1,
                                                        int32_t* __restrict__ cv2, int32_t* __restrict__ pe_off,
                                                        int32_t* __restrict__ cv_off) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int n = F.P;
    if (t < n) se3_inverse_dev(T + (F.s0 + t) * 7, poses + 7 * t);
    if (t == 0) le_off[L] = 2 * L;
    // the offsets (closed form in the counts): pose p's edges start at pe0[p]; the co-visibility lists of row p1 hold
    // (p1, p1): c[p1] + c[p1 + 1] entries and (p1, p1 + 1): c[p1 + 1], after F.row[p1]
    if (t <= n) pe_off[t] = t < n ? F.pe0[t] : 2 * L;
    for (int i = t; i <= n * n; i += gridDim.x * 256) {
        if (i == 0) {
            cv_off[0] = 0;
            continue;
        }
        const int p1 = (i - 1) / n, p2 = (i - 1) - p1 * n;
        const int cn = p1 + 1 < n ? F.c[p1 + 1] : 0;
        cv_off[i] = F.row[p1] + (p2 >= p1 ? F.c[p1] + cn : 0) + (p2 >= p1 + 1 ? cn : 0);
    }
    if (t >= L) return;
    int i = 1;  // the owning pose: base[i] <= t < base[i] + c[i]
    while (i + 1 < F.P && t >= F.base[i + 1]) ++i;
    while (F.c[i] == 0 || t >= F.base[i] + F.c[i]) ++i;
    const int j = t - F.base[i];
    const int64_t o = (F.s0 + i) * max_lm + j;
    X[3 * t] = Xs[3 * o];
    X[3 * t + 1] = Xs[3 * o + 1];
    X[3 * t + 2] = Xs[3 * o + 2];
    const int own = 2 * F.base[i] + j, prev = 2 * F.base[i] + F.c[i] + j;
    ep[own] = i;
    ep[prev] = i - 1;
    el[own] = t;
    el[prev] = t;
    meas[2 * own] = uvo[2 * o];
    meas[2 * own + 1] = uvo[2 * o + 1];
    meas[2 * prev] = uvp[2 * o];
    meas[2 * prev + 1] = uvp[2 * o + 1];
    le_off[t] = 2 * t;
    le[2 * t] = own;
    le[2 * t + 1] = prev;
    // pose i: its own edges first; pose i - 1: its own edges, then frame i's prev edges
    pe[F.pe0[i] + j] = own;
    pe[F.pe0[i - 1] + F.c[i - 1] + j] = prev;
    // (i, i): frame i's (own, own) first, frame i + 1's (prev, prev) after; (i - 1, i - 1) likewise;
    // (i - 1, i): frame i's (prev, own)
    cv1[F.row[i] + j] = own;
    cv2[F.row[i] + j] = own;
    const int r = F.row[i - 1] + F.c[i - 1];
    cv1[r + j] = prev;
    cv2[r + j] = prev;
    cv1[r + F.c[i] + j] = prev;
    cv2[r + F.c[i] + j] = own;
}

// apply_window: T_wc = inverse(T_cw) for every window frame, refined landmarks back to their frames, the anchor
__global__ __launch_bounds__(256) void win_scatter_kernel(WinFrames F, int L, int max_lm, const double* __restrict__ poses,
                                                          const double* __restrict__ X, double* __restrict__ T,
                                                          double* __restrict__ Xs, double* __restrict__ anchor,
                                                          const int* gate) {
    if (gate && *gate) return;  // enqueued with the solve: skipped when it was suspended (solve_end reruns it)
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t < F.P) {
        double o[7];
        se3_inverse_dev(poses + 7 * t, o);
        for (int k = 0; k < 7; ++k) T[(F.s0 + t) * 7 + k] = o[k];
        if (anchor && t == F.P - 1)
            for (int k = 0; k < 7; ++k) anchor[k] = o[k];
    }
    if (t >= L) return;
    int i = 1;
    while (i + 1 < F.P && t >= F.base[i + 1]) ++i;
    while (F.c[i] == 0 || t >= F.base[i] + F.c[i]) ++i;
    const int64_t o = (F.s0 + i) * max_lm + (t - F.base[i]);
    Xs[3 * o] = X[3 * t];
    Xs[3 * o + 1] = X[3 * t + 1];
    Xs[3 * o + 2] = X[3 * t + 2];
}

__global__ void win_anchor_kernel(const double* __restrict__ T, double* __restrict__ anchor) {
    if (threadIdx.x < 7) anchor[threadIdx.x] = T[threadIdx.x];
}

}  // namespace

struct yv_ba_window {
    yv_ba* ba = nullptr;
    int max_lm = 0, max_kf = 0;
    int64_t g0 = -1, cap = 0;  // store index 0 = frame g0; frames [g0, g0 + cap) fit
    int64_t hint = 0;          // yv_ba_window_reserve: frames the store is first sized for
    double *d_T = nullptr, *d_X = nullptr, *d_uvo = nullptr, *d_uvp = nullptr;
    int32_t *d_cnt = nullptr, *d_edge = nullptr;
    int64_t* d_info = nullptr;  // [1 + 2 max_kf]: n_kf, (frame, count) per keyframe of the last block
    int64_t* h_info = nullptr;  // pinned copy
    hipEvent_t added = nullptr;
    bool add_pending = false;
    std::vector<int32_t> h_cnt;  // per store index, -1 = not recorded
    // a solve enqueued by yv_ba_window_solve_begin, collected by yv_ba_window_solve_end
    bool solving = false;
    int solve_kind = 0;  // 1: the LM runs; 2: nothing to solve (only the anchor kernel)
    int solve_iters = 0, solve_nb = 0, solve_L = 0;
    double* solve_anchor = nullptr;
    WinFrames solve_F{};
};

namespace {

void win_free_store(yv_ba_window* w) {
    for (void* p : {(void*)w->d_T, (void*)w->d_X, (void*)w->d_uvo, (void*)w->d_uvp, (void*)w->d_cnt, (void*)w->d_edge})
        if (p) (void)hipFree(p);
    w->d_T = w->d_X = w->d_uvo = w->d_uvp = nullptr;
    w->d_cnt = w->d_edge = nullptr;
}

// the store covers frames [g0, end): grown by doubling, the recorded frames copied over (stream-ordered)
int win_reserve(yv_ba_window* w, int64_t first, int64_t end, hipStream_t st) {
    if (w->g0 < 0) w->g0 = first;
    if (first < w->g0) return YV_ERR_INVALID;
    if (end - w->g0 <= w->cap) return YV_OK;
    int64_t cap = std::max<int64_t>(std::max<int64_t>(64, w->hint), w->cap);
    while (cap < end - w->g0) cap *= 2;
    const int64_t M = w->max_lm;
    double *T = nullptr, *X = nullptr, *uvo = nullptr, *uvp = nullptr;
    int32_t *cnt = nullptr, *edge = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&T), sizeof(double) * 7 * cap) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&X), sizeof(double) * 3 * M * cap) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&uvo), sizeof(double) * 2 * M * cap) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&uvp), sizeof(double) * 2 * M * cap) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&cnt), sizeof(int32_t) * cap) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&edge), sizeof(int32_t) * M * cap) != hipSuccess) {
        for (void* p : {(void*)T, (void*)X, (void*)uvo, (void*)uvp, (void*)cnt, (void*)edge})
            if (p) (void)hipFree(p);
        return YV_ERR_HIP;
    }
    const int64_t c0 = w->cap;
    bool ok = true;
    if (c0 > 0) {
        ok = hipMemcpyAsync(T, w->d_T, sizeof(double) * 7 * c0, hipMemcpyDeviceToDevice, st) == hipSuccess &&
             hipMemcpyAsync(X, w->d_X, sizeof(double) * 3 * M * c0, hipMemcpyDeviceToDevice, st) == hipSuccess &&
             hipMemcpyAsync(uvo, w->d_uvo, sizeof(double) * 2 * M * c0, hipMemcpyDeviceToDevice, st) == hipSuccess &&
             hipMemcpyAsync(uvp, w->d_uvp, sizeof(double) * 2 * M * c0, hipMemcpyDeviceToDevice, st) == hipSuccess &&
             hipMemcpyAsync(cnt, w->d_cnt, sizeof(int32_t) * c0, hipMemcpyDeviceToDevice, st) == hipSuccess &&
             hipMemcpyAsync(edge, w->d_edge, sizeof(int32_t) * M * c0, hipMemcpyDeviceToDevice, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
    }
    win_free_store(w);
    w->d_T = T;
    w->d_X = X;
    w->d_uvo = uvo;
    w->d_uvp = uvp;
    w->d_cnt = cnt;
    w->d_edge = edge;
    w->cap = cap;
    w->h_cnt.resize((size_t)cap, -1);
    return ok ? YV_OK : YV_ERR_HIP;
}

// the last add's keyframe counts are on the host
int win_collect(yv_ba_window* w) {
    if (!w->add_pending) return YV_OK;
    if (hipEventSynchronize(w->added) != hipSuccess) return YV_ERR_HIP;
    w->add_pending = false;
    const int64_t n = std::min<int64_t>(w->h_info[0], w->max_kf);
    for (int64_t j = 0; j < n; ++j) {
        const int64_t s = w->h_info[1 + 2 * j] - w->g0;
        if (s >= 0 && s < w->cap) w->h_cnt[(size_t)s] = (int32_t)w->h_info[2 + 2 * j];
    }
    return YV_OK;
}

}  // namespace

extern "C" int yv_ba_window_create(yv_ba* ba, int max_lm, int max_kf, yv_ba_window** out) {
    if (!out) return YV_ERR_INVALID;
    *out = nullptr;
    if (!ba || max_lm < 1 || max_lm > 65536 || max_kf < 1) return YV_ERR_INVALID;
    if (hipSetDevice(ba->dev) != hipSuccess) return YV_ERR_HIP;
    yv_ba_window* w = new yv_ba_window();
    w->ba = ba;
    w->max_lm = max_lm;
    w->max_kf = max_kf;
    if (hipMalloc(reinterpret_cast<void**>(&w->d_info), sizeof(int64_t) * (1 + 2 * (size_t)max_kf)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&w->h_info), sizeof(int64_t) * (1 + 2 * (size_t)max_kf)) != hipSuccess ||
        hipEventCreateWithFlags(&w->added, hipEventDisableTiming) != hipSuccess) {
        yv_ba_window_destroy(w);
        return YV_ERR_HIP;
    }
    *out = w;
    return YV_OK;
}

extern "C" void yv_ba_window_destroy(yv_ba_window* w) {
    if (!w) return;
    (void)hipSetDevice(w->ba->dev);
    if (w->added) {
        (void)hipEventSynchronize(w->added);
        (void)hipEventDestroy(w->added);
    }
    (void)hipStreamSynchronize(w->ba->st);
    win_free_store(w);
    if (w->d_info) (void)hipFree(w->d_info);
    if (w->h_info) (void)hipHostFree(w->h_info);
    delete w;
}

extern "C" int yv_ba_window_reserve(yv_ba_window* w, int64_t n_frames) {
    if (!w || n_frames < 0 || n_frames > (int64_t)1 << 24 || w->solving) return YV_ERR_INVALID;
    w->hint = n_frames;
    if (n_frames <= w->cap) return YV_OK;
    if (hipSetDevice(w->ba->dev) != hipSuccess) return YV_ERR_HIP;
    if (w->g0 < 0) {
        // nothing recorded yet: allocate the store now, not at the first add_block, which runs inside the caller's
        // frame loop (the store is ~150 MB per 1000 frames at 2000 landmark slots); its origin stays unset
        w->g0 = 0;
        const int rc = win_reserve(w, 0, n_frames, yavo::ctx_stream(w->ba->ctx));
        w->g0 = -1;
        return rc;
    }
    return win_reserve(w, w->g0, w->g0 + n_frames, yavo::ctx_stream(w->ba->ctx));
}

extern "C" int yv_ba_window_add_block(yv_ba_window* w, const void* d_block, int64_t first_frame, int n_frames,
                                      const double* d_edge_uv, const int32_t* d_edge_query, const void* d_matches,
                                      int max_kp, void* stream) {
    if (!w || !d_block || !d_edge_uv || !d_edge_query || !d_matches || n_frames < 1 || first_frame < 0 ||
        max_kp < 1 || max_kp > 65536 || w->solving)  // a pending solve reads the store: collect it first
        return YV_ERR_INVALID;
    if (hipSetDevice(w->ba->dev) != hipSuccess) return YV_ERR_HIP;
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : yavo::ctx_stream(w->ba->ctx);
    if (win_collect(w) != YV_OK) return YV_ERR_HIP;  // one block in flight: its info buffer is reused
    const int rc = win_reserve(w, first_frame, first_frame + n_frames, st);
    if (rc != YV_OK) return rc;
    hipLaunchKernelGGL(win_add_kernel, dim3(w->max_kf), dim3(256), 0, st, reinterpret_cast<const uint8_t*>(d_block),
                       d_edge_uv, d_edge_query, reinterpret_cast<const uint8_t*>(d_matches), max_kp, w->g0, w->cap,
                       w->max_lm,
                       w->d_T, w->d_cnt, w->d_edge, w->d_X, w->d_uvo, w->d_uvp, w->d_info);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(w->h_info, w->d_info, sizeof(int64_t) * (1 + 2 * (size_t)w->max_kf), hipMemcpyDeviceToHost,
                       st) != hipSuccess ||
        hipEventRecord(w->added, st) != hipSuccess)
        return YV_ERR_HIP;
    w->add_pending = true;
    return YV_OK;
}

extern "C" int yv_ba_window_solve_begin(yv_ba_window* w, int64_t first, int n, int n_fixed, const double K[9],
                                        int max_iters, double* d_anchor) {
    if (!w || !K || n < 1 || n > kWinMaxPoses || n_fixed < 0 || max_iters < 0 || w->solving) return YV_ERR_INVALID;
    for (int i = 0; i < 9; ++i)
        if (!std::isfinite(K[i])) return YV_ERR_INVALID;
    yv_ba* b = w->ba;
    if (hipSetDevice(b->dev) != hipSuccess || win_collect(w) != YV_OK) return YV_ERR_HIP;
    if (first < w->g0 || first + n > w->g0 + w->cap) return YV_ERR_INVALID;
    WinFrames F{};
    F.P = n;
    F.s0 = first - w->g0;
    int L = 0;
    for (int i = 0; i < n; ++i) {
        const int32_t c = w->h_cnt[(size_t)(F.s0 + i)];
        if (c < 0) return YV_ERR_INVALID;  // frame not recorded
        F.c[i] = i == 0 ? 0 : c;           // the first frame's predecessor is outside the window
        F.base[i] = L;
        L += F.c[i];
    }
    hipStream_t st = b->st;
    if (n <= n_fixed || L == 0) {  // nothing to solve: the anchor is the last frame's pose as recorded
        if (d_anchor) {
            hipLaunchKernelGGL(win_anchor_kernel, dim3(1), dim3(64), 0, st, w->d_T + (F.s0 + n - 1) * 7, d_anchor);
            if (hipGetLastError() != hipSuccess) return YV_ERR_HIP;
        }
        w->solving = true;
        w->solve_kind = 2;
        return YV_OK;
    }
    const int E = 2 * L;
    const int64_t nc = 3 * (int64_t)L;
    if (n > b->max_poses || L > b->max_landmarks || E > b->max_edges) return YV_ERR_CAPACITY;
    // per pose: its edges start (own edges of frame p, then the prev edges of frame p + 1); per row p1 of the
    // co-visibility buckets: (p1, p1) = c[p1] + c[p1 + 1] entries, (p1, p1 + 1) = c[p1 + 1]. win_build_kernel writes
    // pe_off / cv_off from these (until c59 the host wrote them and copied them over: two copies per solve)
    int32_t acc = 0, racc = 0;
    for (int p = 0; p < n; ++p) {
        const int32_t cn = p + 1 < n ? F.c[p + 1] : 0;
        F.pe0[p] = acc;
        acc += F.c[p] + cn;
        F.row[p] = racc;
        racc += F.c[p] + 2 * cn;
    }
    if (nc > b->cv_cap) {
        if (hipStreamSynchronize(st) != hipSuccess) return YV_ERR_HIP;
        ba_free_one(b, b->d_cv_e1);
        ba_free_one(b, b->d_cv_e2);
        b->d_cv_e1 = b->d_cv_e2 = nullptr;
        b->cv_cap = 0;
        if (ba_alloc(b, &b->d_cv_e1, nc) != YV_OK || ba_alloc(b, &b->d_cv_e2, nc) != YV_OK) return YV_ERR_HIP;
        b->cv_cap = nc;
    }
    b->ready = false;
    yavo::BaParams& Q = b->P;
    const int nb = (std::max(L, n) + 255) / 256;
    hipLaunchKernelGGL(win_build_kernel, dim3(nb), dim3(256), 0, st, F, L, w->max_lm, w->d_T, w->d_X, w->d_uvo,
                       w->d_uvp, Q.poses, Q.X, b->d_ep, b->d_el, b->d_meas, b->d_le_off, b->d_le, b->d_pe, b->d_cv_e1,
                       b->d_cv_e2, b->d_pe_off, b->d_cv_off);
    if (hipGetLastError() != hipSuccess) return YV_ERR_HIP;
    Q.P = n;
    Q.nf = n_fixed;
    Q.np = n - n_fixed;
    Q.ns = 6 * Q.np;
    if (ba_ensure_schur(b, Q.np, st) != YV_OK) return YV_ERR_HIP;
    Q.L = L;
    Q.E = E;
    Q.ep = b->d_ep;
    Q.el = b->d_el;
    Q.meas = b->d_meas;
    Q.pe_off = b->d_pe_off;
    Q.pe = b->d_pe;
    Q.le_off = b->d_le_off;
    Q.le = b->d_le;
    Q.cv_off = b->d_cv_off;
    Q.cv_e1 = b->d_cv_e1;
    Q.cv_e2 = b->d_cv_e2;
    std::memcpy(b->K.v, K, sizeof b->K.v);
    b->ready = true;
    const int rc = ba_solve_enqueue(b, nullptr, nullptr, max_iters);
    if (rc != YV_OK) return rc;
    // the write-back in the same submission (skipped on the device if the solve suspends; _end reruns it then)
    hipLaunchKernelGGL(win_scatter_kernel, dim3(nb), dim3(256), 0, st, F, L, w->max_lm, Q.poses, Q.X, w->d_T, w->d_X,
                       d_anchor, static_cast<const int*>(&b->d_ctl->suspended));
    if (hipGetLastError() != hipSuccess) return YV_ERR_HIP;
    w->solving = true;
    w->solve_kind = 1;
    w->solve_iters = max_iters;
    w->solve_nb = nb;
    w->solve_L = L;
    w->solve_anchor = d_anchor;
    w->solve_F = F;
    return YV_OK;
}

extern "C" int yv_ba_window_solve_end(yv_ba_window* w, double* chi2_log, int* iters, int* solved) {
    if (!w || !w->solving) return YV_ERR_INVALID;
    yv_ba* b = w->ba;
    if (hipSetDevice(b->dev) != hipSuccess) return YV_ERR_HIP;
    hipStream_t st = b->st;
    const int kind = w->solve_kind;
    w->solving = false;
    w->solve_kind = 0;
    if (iters) *iters = 0;
    if (solved) *solved = 0;
    if (kind == 2) return hipStreamSynchronize(st) == hipSuccess ? YV_OK : YV_ERR_HIP;
    int it = 0;
    const int rc = ba_solve_wait(b, nullptr, nullptr, w->solve_iters, chi2_log, &it);
    if (rc != YV_OK) return rc;
    if (b->resumed) {  // the write-back enqueued by _begin was skipped: the solve finished only now
        yavo::BaParams& Q = b->P;
        hipLaunchKernelGGL(win_scatter_kernel, dim3(w->solve_nb), dim3(256), 0, st, w->solve_F, w->solve_L, w->max_lm,
                           Q.poses, Q.X, w->d_T, w->d_X, w->solve_anchor, static_cast<const int*>(nullptr));
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return YV_ERR_HIP;
    }
    if (iters) *iters = it;
    if (solved) *solved = 1;
    return YV_OK;
}

extern "C" int yv_ba_window_solve(yv_ba_window* w, int64_t first, int n, int n_fixed, const double K[9], int max_iters,
                                  double* d_anchor, double* chi2_log, int* iters, int* solved) {
    const int rc = yv_ba_window_solve_begin(w, first, n, n_fixed, K, max_iters, d_anchor);
    if (rc != YV_OK) return rc;
    return yv_ba_window_solve_end(w, chi2_log, iters, solved);
}

extern "C" int yv_ba_window_read(yv_ba_window* w, int64_t frame, double* T_wc, int* n, int32_t* edge, double* X,
                                 double* uv_own, double* uv_prev, int cap) {
    if (!w || !n || w->solving) return YV_ERR_INVALID;
    if (hipSetDevice(w->ba->dev) != hipSuccess || win_collect(w) != YV_OK) return YV_ERR_HIP;
    const int64_t s = frame - w->g0;
    if (w->g0 < 0 || s < 0 || s >= w->cap || w->h_cnt[(size_t)s] < 0) return YV_ERR_INVALID;
    hipStream_t st = w->ba->st;
    const int m = w->h_cnt[(size_t)s];
    *n = m;
    if (hipStreamSynchronize(yavo::ctx_stream(w->ba->ctx)) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return YV_ERR_HIP;
    const int k = std::min(m, cap);
    const int64_t o = s * w->max_lm;
    if ((T_wc && hipMemcpy(T_wc, w->d_T + 7 * s, sizeof(double) * 7, hipMemcpyDeviceToHost) != hipSuccess) ||
        (edge && k && hipMemcpy(edge, w->d_edge + o, sizeof(int32_t) * k, hipMemcpyDeviceToHost) != hipSuccess) ||
        (X && k && hipMemcpy(X, w->d_X + 3 * o, sizeof(double) * 3 * k, hipMemcpyDeviceToHost) != hipSuccess) ||
        (uv_own && k && hipMemcpy(uv_own, w->d_uvo + 2 * o, sizeof(double) * 2 * k, hipMemcpyDeviceToHost) != hipSuccess) ||
        (uv_prev && k && hipMemcpy(uv_prev, w->d_uvp + 2 * o, sizeof(double) * 2 * k, hipMemcpyDeviceToHost) != hipSuccess))
        return YV_ERR_HIP;
    return YV_OK;
}

extern "C" int yv_ba_window_export_block(yv_ba_window* w, int64_t first, int n, int64_t chunk_frame,
                                         int64_t frame_id_offset, void* d_block, int max_kf, int lm_stride,
                                         void* stream) {
    if (!w || !d_block || n < 0 || n > max_kf || max_kf < 1 || lm_stride < w->max_lm || w->solving ||
        frame_id_offset < 0 || first + frame_id_offset < 0 || first + frame_id_offset + n > ((int64_t)1 << 47))
        return YV_ERR_INVALID;
    if (hipSetDevice(w->ba->dev) != hipSuccess || win_collect(w) != YV_OK) return YV_ERR_HIP;
    if ((n > 0 && (first < w->g0 || first + n > w->g0 + w->cap)) || chunk_frame < w->g0 ||
        chunk_frame >= w->g0 + w->cap)
        return YV_ERR_INVALID;
    for (int64_t g = first; g < first + n; ++g)
        if (w->h_cnt[(size_t)(g - w->g0)] < 0) return YV_ERR_INVALID;  // not recorded
    if (w->h_cnt[(size_t)(chunk_frame - w->g0)] < 0) return YV_ERR_INVALID;
    // the records' last writers (add_block on its stream, the window write-back on the BA stream) are finished
    if (hipStreamSynchronize(yavo::ctx_stream(w->ba->ctx)) != hipSuccess ||
        hipStreamSynchronize(w->ba->st) != hipSuccess)
        return YV_ERR_HIP;
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : yavo::ctx_stream(w->ba->ctx);
    hipLaunchKernelGGL(win_export_kernel, dim3(std::max(n, 1)), dim3(256), 0, st, w->d_T, w->d_cnt,
                       w->d_edge, w->d_X, first - w->g0, n, chunk_frame - w->g0, first + frame_id_offset, w->max_lm,
                       max_kf, lm_stride, static_cast<uint8_t*>(d_block));
    return hipGetLastError() == hipSuccess ? YV_OK : YV_ERR_HIP;
}

extern "C" int yv_ba_window_trajectory(yv_ba_window* w, int64_t first, int n, double* T_wc) {
    if (!w || !T_wc || n < 0 || w->solving) return YV_ERR_INVALID;
    if (hipSetDevice(w->ba->dev) != hipSuccess || win_collect(w) != YV_OK) return YV_ERR_HIP;
    if (n == 0) return YV_OK;
    if (first < w->g0 || first + n > w->g0 + w->cap) return YV_ERR_INVALID;
    if (hipStreamSynchronize(yavo::ctx_stream(w->ba->ctx)) != hipSuccess ||
        hipStreamSynchronize(w->ba->st) != hipSuccess ||
        hipMemcpy(T_wc, w->d_T + 7 * (first - w->g0), sizeof(double) * 7 * n, hipMemcpyDeviceToHost) != hipSuccess)
        return YV_ERR_HIP;
    return YV_OK;
}
