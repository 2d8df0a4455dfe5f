// PMC calibration probe (round 4): kernels with an exactly known number of
// MFMAs, to check what rocprofv3's MFMA counters report on gfx950 before any
// profile of the GEMM kernels quotes them:
//   SQ_INSTS_VALU_MFMA_MOPS_{F64,BF16} should equal FLOPs / 512;
//   SQ_VALU_MFMA_BUSY_CYCLES should scale with the MFMA count (the round-1..3
//   profiles read exact powers of two regardless of the kernel).
// Each wave issues ITERS x NACC MFMAs on independent accumulators; grid of
// 2048 workgroups x 4 waves.  Prints the expected FLOPs and MFMA counts per
// dispatch and the event-timed duration of each.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

constexpr int NACC = 8, WAVES = 4, BLOCKS = 2048;

__global__ __launch_bounds__(256) void mfma_f64(double* out, int iters) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
    const double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void mfma_bf16(float* out, int iters) {
    f4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
    bf8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(threadIdx.x * 1e-3f + j);
        b[j] = (__bf16)(1.0f - j * 1e-2f);
    }
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
    const int base = argc > 1 ? atoi(argv[1]) : 1000;
    double* o64;
    float* o32;
    if (hipMalloc(&o64, sizeof(double) * BLOCKS * 256) != hipSuccess) return 1;
    if (hipMalloc(&o32, sizeof(float) * BLOCKS * 256) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double waves = double(BLOCKS) * WAVES;
    // dispatch order: f64 x1, f64 x2, bf16 x1, bf16 x2 (x = iteration multiplier)
    for (int kind = 0; kind < 2; ++kind)
        for (int mul = 1; mul <= 2; ++mul) {
            const int iters = base * mul;
            hipEventRecord(e0, 0);
            if (kind == 0) hipLaunchKernelGGL(mfma_f64, dim3(BLOCKS), dim3(256), 0, 0, o64, iters);
            else hipLaunchKernelGGL(mfma_bf16, dim3(BLOCKS), dim3(256), 0, 0, o32, iters);
            hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess) return 2;
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double nmfma = waves * iters * NACC;
            const double flop_per = kind == 0 ? 2.0 * 16 * 16 * 4 : 2.0 * 16 * 16 * 32;
            const double flops = nmfma * flop_per;
            std::printf("dispatch %s iters %d: mfma %.6e flops %.6e mops_expected %.6e ms %.3f TF %.1f\n",
                        kind == 0 ? "f64_16x16x4" : "bf16_16x16x32", iters, nmfma, flops, flops / 512.0, ms,
                        flops / (ms * 1e-3) / 1e12);
        }
    return 0;
}
