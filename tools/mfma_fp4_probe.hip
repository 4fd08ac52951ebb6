// FP4 MFMA rate probe (the matcher's instruction): what v_mfma_scale_f32_16x16x128_f8f6f4 and _32x32x64_ with FP4
// operands sustain on gfx950, alone and with the matcher's running-maximum VALU beside them, at 1-3 waves per SIMD.
//
// Each wave runs R rounds of independent accumulator chains (8 for 16x16x128, 4 for 32x32x64: the same MACs per
// round); the "+max" forms fold every accumulator element into a running maximum with v_max3_u32 as the matcher
// does (1 per 16x16x128 MFMA, 2 per 32x32x64 MFMA).  Workgroups of 256 threads, grid 256 * W.  Reported:
//   TOP/s = 2 * MACs / kernel time (HIP events), and the fraction of the 10 POP/s dense FP4 peak.
//
// Build + run (GPU box; accumulators in VGPRs as in the matcher's build):
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -o gpurun_out/mfma_fp4_probe tools/mfma_fp4_probe.hip &&
//                         gpurun_out/mfma_fp4_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <bool MAX>
__global__ __launch_bounds__(256) void k16(int rounds, uint32_t seed, uint32_t* sink) {
    const uint32_t t = threadIdx.x + seed;
    v8i a = {(int)(t & 0x22222222u), (int)(t * 3u & 0x22222222u), (int)(t * 5u & 0x22222222u),
             (int)(t * 7u & 0x22222222u), 0, 0, 0, 0};
    v8i b = {(int)(t * 11u & 0x22222222u), (int)(t * 13u & 0x22222222u), (int)(t * 17u & 0x22222222u),
             (int)(t * 19u & 0x22222222u), 0, 0, 0, 0};
    v4f acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = v4f{(float)i, 0.f, 0.f, 0.f};
    uint32_t best[4] = {0, 0, 0, 0};
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[i], 4, 4, 0, 133, 0, 133);
        if (MAX) {
#pragma unroll
            for (int i = 0; i < 8; i += 2)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    best[e] = max(best[e], max(__float_as_uint(acc[i][e]), __float_as_uint(acc[i + 1][e])));
        }
    }
    uint32_t s = best[0] ^ best[1] ^ best[2] ^ best[3];
    for (int i = 0; i < 8; ++i) s ^= __float_as_uint(acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3]);
    if (s == 0x12345678u) sink[threadIdx.x] = s;
}

template <bool MAX>
__global__ __launch_bounds__(256) void k32(int rounds, uint32_t seed, uint32_t* sink) {
    const uint32_t t = threadIdx.x + seed;
    v8i a = {(int)(t & 0x22222222u), (int)(t * 3u & 0x22222222u), (int)(t * 5u & 0x22222222u),
             (int)(t * 7u & 0x22222222u), 0, 0, 0, 0};
    v8i b = {(int)(t * 11u & 0x22222222u), (int)(t * 13u & 0x22222222u), (int)(t * 17u & 0x22222222u),
             (int)(t * 19u & 0x22222222u), 0, 0, 0, 0};
    v16f acc[4];
    for (int i = 0; i < 4; ++i) {
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
        acc[i][0] = (float)i;
    }
    uint32_t best = 0;
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[i], 4, 4, 0, 133, 0, 133);
        if (MAX) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 16; e += 2)
                    best = max(best, max(__float_as_uint(acc[i][e]), __float_as_uint(acc[i][e + 1])));
        }
    }
    uint32_t s = best;
    for (int i = 0; i < 4; ++i) s ^= __float_as_uint(acc[i][0] + acc[i][5]);
    if (s == 0x12345678u) sink[threadIdx.x] = s;
}

// the x32 matcher's inner loop without LDS: per round 4 query tiles x 4 K-steps (two chains at a time from one C),
// then each chain's 16 keys folded into its tile's running maximum (max16: a depth-3 tree of v_max3)
__device__ __forceinline__ uint32_t max16_u32(uint32_t best, const v16f& a) {
    auto u = [&](int i) { return __float_as_uint(a[i]); };
    const uint32_t m0 = max(u(0), max(u(1), u(2))), m1 = max(u(3), max(u(4), u(5)));
    const uint32_t m2 = max(u(6), max(u(7), u(8))), m3 = max(u(9), max(u(10), u(11)));
    const uint32_t m4 = max(u(12), max(u(13), u(14)));
    const uint32_t m5 = max(m0, max(m1, m2)), m6 = max(m3, max(m4, u(15)));
    return max(best, max(m5, m6));
}

template <int QT>
__global__ __launch_bounds__(256) void k32chain(int rounds, uint32_t seed, uint32_t* sink) {
    const uint32_t t = threadIdx.x + seed;
    v8i A[4], B[QT][4];
    for (int s = 0; s < 4; ++s) {
        A[s] = v8i{(int)(t * (3u + s) & 0x22222222u), (int)(t * (5u + s) & 0x22222222u), (int)(t * (7u + s) & 0x22222222u),
                   (int)(t * (9u + s) & 0x22222222u), 0, 0, 0, 0};
        for (int q = 0; q < QT; ++q)
            B[q][s] = v8i{(int)(t * (11u + s + q) & 0x22222222u), (int)(t * (13u + s) & 0x22222222u),
                          (int)(t * (17u + q) & 0x22222222u), (int)(t * (19u + s) & 0x22222222u), 0, 0, 0, 0};
    }
    v16f C;
    for (int e = 0; e < 16; ++e) C[e] = (float)(e + t);
    uint32_t best[QT];
    for (int q = 0; q < QT; ++q) best[q] = 0;
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int q = 0; q < QT; q += 2) {
            v16f a0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A[0], B[q][0], C, 4, 4, 0, 133, 0, 133);
            v16f a1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A[0], B[q + 1][0], C, 4, 4, 0, 133, 0, 133);
#pragma unroll
            for (int s = 1; s < 4; ++s) {
                a0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A[s], B[q][s], a0, 4, 4, 0, 133, 0, 133);
                a1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A[s], B[q + 1][s], a1, 4, 4, 0, 133, 0, 133);
            }
            best[q] = max16_u32(best[q], a0);
            best[q + 1] = max16_u32(best[q + 1], a1);
        }
        C[r & 15] += 1.0f;  // keep C live and varying
    }
    uint32_t s = 0;
    for (int q = 0; q < QT; ++q) s ^= best[q];
    if (s == 0x12345678u) sink[threadIdx.x] = s;
}

// the production 16x16x128 matcher's inner loop without LDS: QT query tiles x two 16-train tiles x 2 K-steps, then
// one v_max3 per MFMA into the tiles' running maxima
template <int QT>
__global__ __launch_bounds__(256) void k16chain(int rounds, uint32_t seed, uint32_t* sink) {
    const uint32_t t = threadIdx.x + seed;
    v8i A[QT][2], Ba[2], Bb[2];
    for (int s = 0; s < 2; ++s) {
        Ba[s] = v8i{(int)(t * (3u + s) & 0x22222222u), (int)(t * (5u + s) & 0x22222222u), (int)(t * (7u + s) & 0x22222222u),
                    (int)(t * (9u + s) & 0x22222222u), 0, 0, 0, 0};
        Bb[s] = v8i{(int)(t * (23u + s) & 0x22222222u), (int)(t * (29u + s) & 0x22222222u), (int)(t * (7u + s) & 0x22222222u),
                    (int)(t * (31u + s) & 0x22222222u), 0, 0, 0, 0};
        for (int q = 0; q < QT; ++q)
            A[q][s] = v8i{(int)(t * (11u + s + q) & 0x22222222u), (int)(t * (13u + s) & 0x22222222u),
                          (int)(t * (17u + q) & 0x22222222u), (int)(t * (19u + s) & 0x22222222u), 0, 0, 0, 0};
    }
    v4f Ca = {(float)t, (float)t, (float)t, (float)t}, Cb = {(float)(t + 1), (float)(t + 1), (float)(t + 1), (float)(t + 1)};
    uint32_t best[QT][4];
    for (int q = 0; q < QT; ++q)
        for (int r = 0; r < 4; ++r) best[q][r] = 0;
    for (int rr = 0; rr < rounds; ++rr) {
#pragma unroll
        for (int q = 0; q < QT; q += 2) {
            v4f a0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q][0], Ba[0], Ca, 4, 4, 0, 133, 0, 133);
            v4f b0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q][0], Bb[0], Cb, 4, 4, 0, 133, 0, 133);
            v4f a1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q + 1][0], Ba[0], Ca, 4, 4, 0, 133, 0, 133);
            v4f b1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q + 1][0], Bb[0], Cb, 4, 4, 0, 133, 0, 133);
            a0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q][1], Ba[1], a0, 4, 4, 0, 133, 0, 133);
            b0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q][1], Bb[1], b0, 4, 4, 0, 133, 0, 133);
            a1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q + 1][1], Ba[1], a1, 4, 4, 0, 133, 0, 133);
            b1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[q + 1][1], Bb[1], b1, 4, 4, 0, 133, 0, 133);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                best[q][r] = max(best[q][r], max(__float_as_uint(a0[r]), __float_as_uint(b0[r])));
                best[q + 1][r] = max(best[q + 1][r], max(__float_as_uint(a1[r]), __float_as_uint(b1[r])));
            }
        }
        Ca[rr & 3] += 1.0f;
    }
    uint32_t s = 0;
    for (int q = 0; q < QT; ++q)
        for (int r = 0; r < 4; ++r) s ^= best[q][r];
    if (s == 0x12345678u) sink[threadIdx.x] = s;
}

template <typename K>
static int run(const char* name, K kern, int rounds, double macs_per_wave_round) {
    uint32_t* sink;
    CK(hipMalloc(&sink, 1024 * sizeof(uint32_t)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int W = 1; W <= 3; ++W) {
        const int grid = 256 * W;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, 16, 1u, sink);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, rounds, 1u, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double ops = 2.0 * macs_per_wave_round * rounds * grid * 4;
        printf("%-22s W=%d  %.3f ms  %.1f TOP/s  %.3f of 10 POP/s\n", name, W, ms, ops / ms / 1e9,
               ops / ms / 1e9 / 10000.0);
    }
    CK(hipFree(sink));
    return 0;
}

int main() {
    const int R = 20000;
    // MACs per wave per round: 8 * 16*16*128 = 4 * 32*32*64 = 262144
    if (run("16x16x128", k16<false>, R, 262144.0)) return 1;
    if (run("16x16x128 + max3", k16<true>, R, 262144.0)) return 1;
    if (run("32x32x64", k32<false>, R, 262144.0)) return 1;
    if (run("32x32x64 + max3", k32<true>, R, 262144.0)) return 1;
    // per round QT * 4 MFMAs of 65536 MACs
    if (run("x32 loop QT=4", k32chain<4>, R / 4, 4 * 4 * 65536.0)) return 1;
    if (run("x32 loop QT=2", k32chain<2>, R / 2, 2 * 4 * 65536.0)) return 1;
    // per round QT * 4 MFMAs of 32768 MACs
    if (run("x16 loop QT=8", k16chain<8>, R / 4, 8 * 4 * 32768.0)) return 1;
    return 0;
}
