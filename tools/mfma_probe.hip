// Microbenchmark: sustained f64 rate of v_mfma_f64_16x16x4_f64, v_fma_f64, and
// both at once (half the waves of each workgroup on each pipe), on gfx950.
// Question it answers: do the f64 matrix and f64 vector pipes overlap, i.e. is
// there f64 throughput beyond either pipe alone?
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__device__ __forceinline__ double mfma_loop(int iters) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    return s;
}
__device__ __forceinline__ double fma_loop(int iters) {
    double x[16];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x + i;
    const double a = 0.999999, b = 1e-7;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = fma(x[i], a, b);
    double s = 0;
    for (int i = 0; i < 16; ++i) s += x[i];
    return s;
}
// mode 0: all waves MFMA; 1: all waves VALU FMA; 2: even waves MFMA, odd waves FMA
template <int NACC>
__global__ __launch_bounds__(256) void probe(double* out, int mode, int mi, int fi) {
    const int w = threadIdx.x >> 6;
    double s;
    if (mode == 0 || (mode == 2 && (w & 1) == 0)) s = mfma_loop<NACC>(mi);
    else s = fma_loop(fi);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    const int blocks = 256 * 8, mi = 2000, fi = mi * 8 * 2048 / (16 * 64 * 2);  // equal FLOPs per wave at nacc = 8
    double* out;
    hipMalloc(&out, sizeof(double) * blocks * 256);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // flops per wave: MFMA wave mi*NACC*2048, FMA wave fi*16*64*2
    auto run = [&](auto kern, int nacc, int mode, const char* what) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, mode, mi, fi);
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, mode, mi, fi);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double waves = blocks * 4.0, fm = (double)mi * nacc * 2048.0, ff = (double)fi * 16 * 64 * 2.0;
        const double flops = mode == 0 ? waves * fm : mode == 1 ? waves * ff : waves / 2 * (fm + ff);
        printf("%-28s nacc=%2d: %6.1f TFLOP/s (%.3f ms)\n", what, nacc, flops / ms / 1e9, ms);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run(probe<8>, 8, 0, "mfma_f64_16x16x4 only");
        run(probe<16>, 16, 0, "mfma_f64_16x16x4 only");
        run(probe<8>, 8, 1, "v_fma_f64 only");
        run(probe<8>, 8, 2, "mfma + v_fma (split waves)");
        run(probe<16>, 16, 2, "mfma + v_fma (split waves)");
    }
    return 0;
}
