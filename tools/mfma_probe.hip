// Microbenchmark: sustained rate of v_mfma_f64_16x16x4_f64 and v_fma_f64 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void mfma_f64(double* out, int iters) {
    d4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    double s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void fma_f64(double* out, int iters) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    const double a = 0.999999, b = 1e-7;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fma(x[i], a, b);
    double s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    int blocks = 256 * 8, iters = 2000;
    double* out; hipMalloc(&out, sizeof(double) * blocks * 256);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(mfma_f64, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(a); hipLaunchKernelGGL(mfma_f64, dim3(blocks), dim3(256), 0, 0, out, iters); hipEventRecord(b);
        hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
        double flops = (double)blocks * 4 /*waves*/ * iters * 8 * 2048.0;
        printf("mfma_f64_16x16x4: %.1f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
        hipLaunchKernelGGL(fma_f64, dim3(blocks), dim3(256), 0, 0, out, iters * 8);
        hipEventRecord(a); hipLaunchKernelGGL(fma_f64, dim3(blocks), dim3(256), 0, 0, out, iters * 8); hipEventRecord(b);
        hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
        flops = (double)blocks * 256 * iters * 8 * 8 * 2.0;
        printf("v_fma_f64: %.1f TFLOP/s (%.3f ms)\n", flops / ms / 1e9, ms);
    }
    return 0;
}
