// HBM -> LDS staging sources shared by the LDS-DMA GEMM kernels.
//
// A slab image is loaded by 1-KiB wave-instructions of 16 B per lane that the
// hardware writes lane-linearly into LDS (M0 + 16 * lane).  The per-lane source
// is an element offset from a wave-uniform slab base; two ways to issue it:
//   GlobalSrc: global_load_lds_dwordx4 with a 64-bit VGPR address per lane;
//   BufferSrc: buffer_load_dwordx4 ... lds with the base in a buffer descriptor
//              (SGPRs) and a 32-bit byte offset per lane.  Measured faster for
//              the fp64 kernel (profiles/r01_f64_buf.log); usable when every
//              offset of an image fits 31 bits (dma_fits).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

namespace elx {
namespace kern {

typedef __attribute__((address_space(3))) char lds_char;

template <typename T>
struct GlobalSrc {
    const T* base;
    __device__ __forceinline__ GlobalSrc(const T* b, int64_t) : base(b) {}
    __device__ __forceinline__ void load(int64_t off, lds_char* dst) const {
        __builtin_amdgcn_global_load_lds((const void*)(base + off), (__attribute__((address_space(3))) void*)dst, 16,
                                         0, 0);
    }
};

template <typename T>
struct BufferSrc {
    __amdgpu_buffer_rsrc_t rs;
    // bytes: the extent every offset of this image stays below (<= 2^31 - 1)
    __device__ __forceinline__ BufferSrc(const T* b, int64_t bytes)
        : rs(__builtin_amdgcn_make_buffer_rsrc((void*)b, 0, (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff),
                                               0x00020000)) {}
    __device__ __forceinline__ void load(int64_t off, lds_char* dst) const {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16,
                                                 (int)(off * (int64_t)sizeof(T)), 0, 0, 0);
    }
};

template <bool BUF, typename T>
using DmaSrc = typename std::conditional<BUF, BufferSrc<T>, GlobalSrc<T>>::type;

// Can an image of `span` k-rows or operand rows (each ld elements apart) be
// addressed with 31-bit byte offsets from its base?
inline bool dma_fits(int64_t span, int64_t ld, int64_t es) { return span * ld * es + 16 < (1ll << 31); }

}  // namespace kern
}  // namespace elx
