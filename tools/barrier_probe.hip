#include <hip/hip_runtime.h>
#include <cstdio>
template <int NT>
__global__ __launch_bounds__(NT) void bar_only(int steps, double* out) {
    __shared__ double x[128];
    double acc = threadIdx.x;
    for (int k = 0; k < steps; ++k) {
        if (threadIdx.x == (k & 127)) x[k & 127] = acc;
        __syncthreads();
        acc = acc + x[k & 127];
        __syncthreads();
    }
    if (acc == 12345.0) out[0] = acc;
}
template <int NT>
__global__ __launch_bounds__(NT) void div_chain(int steps, double* out) {
    __shared__ double x[128];
    double acc = threadIdx.x + 1.0;
    for (int k = 0; k < steps; ++k) {
        if (threadIdx.x == (k & 127)) x[k & 127] = 1.0 / acc;
        __syncthreads();
        acc = acc + x[k & 127];
        __syncthreads();
    }
    if (acc == 12345.0) out[0] = acc;
}
int main() {
    double* d; hipMalloc(&d, 8);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto run = [&](const char* name, auto kern, int nt) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(1), dim3(nt), 0, 0, 114, d);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("%s nt=%d: %.1f us (%.0f ns per step)\n", name, nt, ms * 1e3, ms * 1e6 / 114);
        }
    };
    run("bar_only", bar_only<64>, 64);
    run("bar_only", bar_only<256>, 256);
    run("bar_only", bar_only<512>, 512);
    run("bar_only", bar_only<1024>, 1024);
    run("div_chain", div_chain<512>, 512);
    return 0;
}
