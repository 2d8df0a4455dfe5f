// Probe: does buffer_load_dwordx4 ... lds (raw_ptr_buffer_load_lds) place data in
// LDS like global_load_lds_dwordx4?  One wave stages 1 KiB both ways and dumps LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((address_space(3))) char lds_char;

__global__ void probe(const double* src, double* out, int mode) {
    __shared__ __attribute__((aligned(1024))) char lds_raw[2048];
    lds_char* lds = (lds_char*)lds_raw;
    const int l = threadIdx.x;
    for (int i = l; i < 256; i += 64) ((double*)lds_raw)[i] = -1.0;
    __syncthreads();
    if (mode == 0) {
        __builtin_amdgcn_global_load_lds((const void*)(src + 2 * l), (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
    } else {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 4096 * 8, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, l * 16, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = l; i < 256; i += 64) out[i] = ((double*)lds_raw)[i];
}

int main() {
    std::vector<double> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = i;
    double *d, *o;
    hipMalloc(&d, 4096 * 8);
    hipMalloc(&o, 256 * 8);
    hipMemcpy(d, h.data(), 4096 * 8, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, mode);
        std::vector<double> r(256);
        hipMemcpy(r.data(), o, 256 * 8, hipMemcpyDeviceToHost);
        printf("mode %d:", mode);
        for (int i = 0; i < 20; ++i) printf(" %g", r[i]);
        printf(" ... [126..129] %g %g %g %g\n", r[126], r[127], r[128], r[129]);
    }
    return 0;
}
