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

// s_waitcnt through the builtin, not inline asm: hipcc's waitcnt pass sees a
// builtin wait and drops the conservative waits it would otherwise add for
// fragment registers whose LDS reads an opaque asm wait already retired (at
// bf16 TN the asm form left 72 spurious "s_waitcnt lgkmcnt(7)" among the MFMAs
// of every five K-tiles; removing them: +0.5-2.4 %, bf16 NN 32768^3 1394-1413 ->
// 1428 TF in one process, profiles/r04_h16_waitcnt_ab.log).  gfx9 encoding: vmcnt [3:0] and [15:14], expcnt
// [6:4], lgkmcnt [11:8]; the fields not waited on are at their maxima.
template <int VM, int LGKM>
__device__ __forceinline__ void wait_cnt() {
    static_assert(VM >= 0 && VM <= 63 && LGKM >= 0 && LGKM <= 15, "waitcnt field range");
    __builtin_amdgcn_s_waitcnt((VM & 15) | ((VM >> 4) << 14) | (7 << 4) | (LGKM << 8));
}
constexpr int NOWAIT_VM = 63, NOWAIT_LGKM = 15;

// Workgroup barrier without __syncthreads' release fence (which waits for every
// outstanding vector-memory op, in-flight LDS DMA of later slabs included): the
// caller's wait_cnt states what must have landed.
__device__ __forceinline__ void dma_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

}  // namespace kern
}  // namespace elx
