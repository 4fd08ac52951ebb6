// Issue-rate probe for the VALU / LDS instructions the image kernels are built from (VERDICT r02 "next" #1):
// is a wave64 integer op such as v_sad_u8 issued every 2 or every 4 cycles per SIMD on gfx950, and how does the
// rate change with 1, 2, 4, 8 waves per SIMD?
//
// Each wave runs R rounds of 8 independent accumulator chains (8 instructions per round, inline asm so the
// compiler neither folds nor reorders them), stamps s_memtime (shader clock) before and after, and lane 0 writes
// the stamps with a vector store.  Workgroups of 256 threads = one wave per SIMD; W workgroups per CU are forced
// by dynamic LDS of 160 KB / W each (so exactly W waves share each SIMD).  Reported per op and W:
//   cyc/inst/SIMD = median over waves of (t_end - t_start) / (W * 8 * R)   (every wave of a SIMD overlaps)
//   wall cyc/inst = kernel wall (HIP events) * clock / (instructions per SIMD), clock from s_memtime / s_memrealtime
//
// Build + run (GPU box):  hipcc -O3 --offload-arch=gfx950 -o gpurun_out/valu_probe tools/valu_probe.hip &&
//                         gpurun_out/valu_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

enum Op {
    OP_ADD_U32, OP_FMA_F32, OP_SAD_U8, OP_ALIGNBIT, OP_ALIGNBYTE, OP_DOT4_U8, OP_DOT2_U16, OP_PERM, OP_MUL_U24,
    OP_OR3, OP_FMA_F64, OP_ADD_F64, OP_PK_ADD_U16, OP_MIX_SAD_ALIGNBIT, OP_DS_READ_U8, OP_DS_READ_B32, OP_N
};
static const char* kOpName[OP_N] = {
    "v_add_u32", "v_fma_f32", "v_sad_u8", "v_alignbit_b32", "v_alignbyte_b32", "v_dot4_u32_u8", "v_dot2_u32_u16",
    "v_perm_b32", "v_mul_u32_u24", "v_or3_b32", "v_fma_f64", "v_add_f64", "v_pk_add_u16", "sad+alignbit (1:1)",
    "ds_read_u8", "ds_read_b32"};

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(1024) void probe(int rounds, uint32_t seed, unsigned long long* stamps, uint32_t* sink) {
    extern __shared__ uint32_t lds[];
    const uint32_t t = threadIdx.x;
    uint32_t a0 = seed ^ t, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 11u, a5 = a0 * 13u, a6 = a0 * 17u,
             a7 = a0 * 19u;
    const uint32_t b = seed * 0x9E3779B9u + t, c = 0x05040302u;
    float f0 = (float)a0, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    const float fb = 1.0000001f;
    double d0 = a0, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
    const double db = 1.0000000001;
    // lane l reads byte / dword l (+ a per-chain row): conflict-free
    const uint32_t lbase = (OP == OP_DS_READ_U8 ? (t & 63) : 4 * (t & 63));
    if (OP == OP_DS_READ_U8 || OP == OP_DS_READ_B32) {
        for (int i = t; i < 4096; i += blockDim.x) lds[i] = i * 2654435761u;
        __syncthreads();
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < rounds; ++r) {
#define A(i) a##i
#define F(i) f##i
#define D(i) d##i
        if (OP == OP_ADD_U32) {
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_FMA_F32) {
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(F(i)) : "v"(fb));
            R8(X)
#undef X
        } else if (OP == OP_SAD_U8) {
#define X(i) asm volatile("v_sad_u8 %0, %0, %1, %0" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_ALIGNBIT) {
#define X(i) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_ALIGNBYTE) {
#define X(i) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_DOT4_U8) {
#define X(i) asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_DOT2_U16) {
#define X(i) asm volatile("v_dot2_u32_u16 %0, %0, %1, %0" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_PERM) {
#define X(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(A(i)) : "v"(b), "v"(c));
            R8(X)
#undef X
        } else if (OP == OP_MUL_U24) {
#define X(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_OR3) {
#define X(i) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(A(i)) : "v"(b), "v"(c));
            R8(X)
#undef X
        } else if (OP == OP_FMA_F64) {
#define X(i) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(D(i)) : "v"(db));
            R8(X)
#undef X
        } else if (OP == OP_ADD_F64) {
#define X(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(D(i)) : "v"(db));
            R8(X)
#undef X
        } else if (OP == OP_PK_ADD_U16) {
#define X(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_MIX_SAD_ALIGNBIT) {
            // the phase-1 / phase-2 pattern of detect_kernel: sad then alignbit on alternating chains
#define X(i) if ((i) & 1) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(A(i)) : "v"(b)); \
             else asm volatile("v_sad_u8 %0, %0, %1, %0" : "+v"(A(i)) : "v"(b));
            R8(X)
#undef X
        } else if (OP == OP_DS_READ_U8) {
            // 8 independent byte reads in flight, then one wait (the loop carries no dependence through LDS)
#define X(i) asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(A(i)) : "v"(lbase), "i"(64 * (i)));
            R8(X)
#undef X
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (OP == OP_DS_READ_B32) {
#define X(i) asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(A(i)) : "v"(lbase), "i"(256 * (i)));
            R8(X)
#undef X
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
#undef A
#undef F
#undef D
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t acc = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ __float_as_uint(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7) ^
                         (uint32_t)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
    if (acc == 0x12345678u) sink[0] = acc;  // keeps every chain live
    if ((t & 63) == 0) {
        const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (t >> 6);
        stamps[4 * w + 0] = t0;
        stamps[4 * w + 1] = t1;
        stamps[4 * w + 2] = rt0;
        stamps[4 * w + 3] = rt1;
    }
}

typedef void (*ProbeFn)(int, uint32_t, unsigned long long*, uint32_t*);
static ProbeFn kFn[OP_N] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>,
                            probe<8>, probe<9>, probe<10>, probe<11>, probe<12>, probe<13>, probe<14>, probe<15>};

int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    const size_t lds_cu = 160 * 1024;
    printf("device %s, %d CUs, LDS/CU %zu\n", prop.name, ncu, lds_cu);
    unsigned long long* stamps;
    uint32_t* sink;
    const int max_blocks = ncu * 8;
    CK(hipMalloc(&stamps, (size_t)max_blocks * 16 * 4 * sizeof(unsigned long long)));
    CK(hipMalloc(&sink, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned long long> h((size_t)max_blocks * 64);
    printf("%-20s %3s %12s %12s %10s %8s\n", "op", "W", "cyc/inst/SIMD", "wall cyc/in", "clock GHz", "ms");
    for (int op = 0; op < OP_N; ++op) {
        const bool f64 = (op == OP_FMA_F64 || op == OP_ADD_F64);
        const bool lds = (op == OP_DS_READ_U8 || op == OP_DS_READ_B32);
        for (int W : {1, 2, 4, 8}) {
            const int rounds = (f64 || lds ? 2000 : 4000) / W;
            const int blocks = ncu * W;
            const size_t dyn = lds_cu / W - 1024;  // exactly W workgroups per CU
            CK(hipFuncSetAttribute((const void*)kFn[op], hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
            hipLaunchKernelGGL(kFn[op], dim3(blocks), dim3(256), dyn, 0, rounds, 7u, stamps, sink);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kFn[op], dim3(blocks), dim3(256), dyn, 0, rounds, 7u, stamps, sink);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(h.data(), stamps, (size_t)blocks * 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            std::vector<double> cyc, clk;
            for (int w = 0; w < blocks * 4; ++w) {
                const double dc = (double)(h[4 * w + 1] - h[4 * w + 0]);
                const double dr = (double)(h[4 * w + 3] - h[4 * w + 2]);
                cyc.push_back(dc);
                if (dr > 0) clk.push_back(dc / dr * 0.1);  // s_memrealtime ticks at 100 MHz
            }
            std::sort(cyc.begin(), cyc.end());
            std::sort(clk.begin(), clk.end());
            const double inst = 8.0 * rounds;  // per wave
            const double med = cyc[cyc.size() / 2];
            const double ghz = clk.empty() ? 0 : clk[clk.size() / 2];
            const double per_simd = med / (W * inst);
            const double wall = ms * 1e-3 * ghz * 1e9 / (W * inst);
            printf("%-20s %3d %12.2f %12.2f %10.3f %8.3f\n", kOpName[op], W, per_simd, wall, ghz, ms);
        }
    }
    // Mode 2: ONE workgroup of 256 W threads per CU (W waves on each SIMD, dispatched together), long runs; per CU the
    // window max(end) - min(start) over its waves: cycles per instruction per SIMD = window / (W * inst)
    printf("\nmode 2: one %s per CU\n", "256 W-thread workgroup");
    printf("%-20s %3s %14s %10s %8s\n", "op", "W", "cyc/inst/SIMD", "clock GHz", "ms");
    for (int op = 0; op < OP_N; ++op) {
        const bool f64 = (op == OP_FMA_F64 || op == OP_ADD_F64);
        const bool lds = (op == OP_DS_READ_U8 || op == OP_DS_READ_B32);
        for (int W : {1, 2, 4}) {
            const int rounds = (f64 || lds ? 8000 : 16000) / W;
            const int nt = 256 * W;
            const size_t dyn = 100 * 1024;  // one workgroup per CU
            CK(hipFuncSetAttribute((const void*)kFn[op], hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
            hipLaunchKernelGGL(kFn[op], dim3(ncu), dim3(nt), dyn, 0, rounds, 7u, stamps, sink);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kFn[op], dim3(ncu), dim3(nt), dyn, 0, rounds, 7u, stamps, sink);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const int nw = ncu * 4 * W;
            CK(hipMemcpy(h.data(), stamps, (size_t)nw * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            std::vector<double> win, clk;
            for (int b = 0; b < ncu; ++b) {
                unsigned long long lo = ~0ull, hi = 0, rlo = ~0ull, rhi = 0;
                for (int w = 0; w < 4 * W; ++w) {
                    const unsigned long long* q = &h[4 * (size_t)(b * 4 * W + w)];
                    lo = std::min(lo, q[0]); hi = std::max(hi, q[1]);
                    rlo = std::min(rlo, q[2]); rhi = std::max(rhi, q[3]);
                }
                win.push_back((double)(hi - lo));
                if (rhi > rlo) clk.push_back((double)(hi - lo) / (double)(rhi - rlo) * 0.1);
            }
            std::sort(win.begin(), win.end());
            std::sort(clk.begin(), clk.end());
            const double inst = 8.0 * rounds;
            printf("%-20s %3d %14.2f %10.3f %8.3f\n", kOpName[op], W, win[win.size() / 2] / (W * inst),
                   clk.empty() ? 0 : clk[clk.size() / 2], ms);
        }
    }
    return 0;
}
