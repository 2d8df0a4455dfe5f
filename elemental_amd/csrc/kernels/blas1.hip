// BLAS-1 / data-movement kernels for gfx950 (HBM-bound).
//
// Replace the reference's per-op device kernels and rocBLAS geam fallbacks:
//   copy2d_batch : Copy_GPU_impl copy_1d/copy_2d (src/hydrogen/blas/gpu/Copy.cu:13-205),
//                  Transpose_GPU_impl (src/hydrogen/blas/gpu/Transpose.cu:17-127),
//                  Axpy_GPU_impl incl. the transpose-tiled form (src/hydrogen/blas/gpu/Axpy.cu:20-189),
//                  and every hipMemcpy2DAsync pack/unpack of Copy/util.hpp:233-355 —
//                  ONE launch moves all r or c portions of a redistribution.
//   fill2d       : Fill_GPU_impl (src/hydrogen/blas/gpu/Fill.cu:20-76)
//   scale2d      : Scale_GPU_impl (src/hydrogen/blas/gpu/Scale.cu:17-81)
//   hadamard2d   : Hadamard_GPU_impl (src/hydrogen/blas/gpu/Hadamard.cu:16-117)
//   entrywise_map: EntrywiseMapImpl (include/hydrogen/blas/gpu/EntrywiseMapImpl.hpp:46-104)
//
// Every kernel is a 256-thread (4-wave) workgroup; lanes always walk the
// unit-stride dimension of whatever they read or write (64 lanes x elem = one
// or more full cache lines); a transposing move stages a 64x64 tile in LDS
// (pitch 65: conflict-free both ways).
#include <hip/hip_runtime.h>
#include "kernels.hpp"
#include "elem.hpp"
#include "../../../include/elemental_amd.h"

namespace elx {
namespace kern {

namespace {

constexpr int TILE = 64;
constexpr int NT = 256;

struct CopyBatch {
    Copy2D d[kMaxCopyBatch];
};

template <typename T, bool AXPY>
__global__ __launch_bounds__(NT) void copy2d_kernel(CopyBatch b, double alpha) {
    using E = Elem<T>;
    using S = typename E::storage;
    using Cmp = typename E::compute;
    __shared__ S tile[TILE][TILE + 1];  // [j][i]
    const Copy2D& d = b.d[blockIdx.y];
    const i64 tiles_i = (d.m + TILE - 1) / TILE, tiles_j = (d.n + TILE - 1) / TILE;
    const i64 ntiles = tiles_i * tiles_j;
    const S* src = static_cast<const S*>(d.src);
    S* dst = static_cast<S*>(d.dst);
    const bool src_i = (d.scs == 1) || (d.srs != 1);
    const bool dst_i = (d.dcs == 1) || (d.drs != 1);
    const int t = threadIdx.x, fast = t & (TILE - 1), slow = t >> 6;
    const Cmp a = (Cmp)alpha;
    for (i64 tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
        const i64 i0 = (tile_id % tiles_i) * TILE, j0 = (tile_id / tiles_i) * TILE;
        if (src_i == dst_i) {
            // both sides walk the same dimension: no staging needed
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const i64 i = i0 + (src_i ? fast : slow + 4 * e);
                const i64 j = j0 + (src_i ? slow + 4 * e : fast);
                if (i < d.m && j < d.n) {
                    const S v = src[i * d.scs + j * d.srs];
                    S* o = dst + i * d.dcs + j * d.drs;
                    if (AXPY) *o = E::store(E::load(*o) + a * E::load(v));
                    else *o = v;
                }
            }
        } else {
            __syncthreads();
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const int li = src_i ? fast : slow + 4 * e;
                const int lj = src_i ? slow + 4 * e : fast;
                const i64 i = i0 + li, j = j0 + lj;
                if (i < d.m && j < d.n) tile[lj][li] = src[i * d.scs + j * d.srs];
            }
            __syncthreads();
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const int li = dst_i ? fast : slow + 4 * e;
                const int lj = dst_i ? slow + 4 * e : fast;
                const i64 i = i0 + li, j = j0 + lj;
                if (i < d.m && j < d.n) {
                    S* o = dst + i * d.dcs + j * d.drs;
                    if (AXPY) *o = E::store(E::load(*o) + a * E::load(tile[lj][li]));
                    else *o = tile[lj][li];
                }
            }
        }
    }
}

// 2-D elementwise driver: columns over gridDim.y, rows over gridDim.x*NT.
template <typename F>
__device__ __forceinline__ void for_each_2d(i64 m, i64 n, F&& f) {
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        for (i64 i = (i64)blockIdx.x * NT + threadIdx.x; i < m; i += (i64)gridDim.x * NT) f(i, j);
}

template <typename T>
__global__ __launch_bounds__(NT) void fill_kernel(i64 m, i64 n, double v, typename Elem<T>::storage* A, i64 lda) {
    using E = Elem<T>;
    const auto s = E::store((typename E::compute)v);
    for_each_2d(m, n, [&](i64 i, i64 j) { A[i + j * lda] = s; });
}

template <typename T>
__global__ __launch_bounds__(NT) void scale_kernel(i64 m, i64 n, double alpha, typename Elem<T>::storage* A, i64 lda) {
    using E = Elem<T>;
    const auto a = (typename E::compute)alpha;
    for_each_2d(m, n, [&](i64 i, i64 j) { auto& x = A[i + j * lda]; x = E::store(a * E::load(x)); });
}

template <typename T>
__global__ __launch_bounds__(NT) void hadamard_kernel(i64 m, i64 n, const typename Elem<T>::storage* A, i64 lda,
                                                      const typename Elem<T>::storage* B, i64 ldb,
                                                      typename Elem<T>::storage* C, i64 ldc) {
    using E = Elem<T>;
    // in-place aliasing (C==A or C==B) is safe: each element is read before its own write
    for_each_2d(m, n, [&](i64 i, i64 j) {
        C[i + j * ldc] = E::store(E::load(A[i + j * lda]) * E::load(B[i + j * ldb]));
    });
}

template <typename C>
__device__ __forceinline__ C apply_map(int fn, C x) {
    switch (fn) {
    case ELX_MAP_IDENTITY: return x;
    case ELX_MAP_NEGATE: return -x;
    case ELX_MAP_ABS: return x < C(0) ? -x : x;
    case ELX_MAP_SQUARE: return x * x;
    case ELX_MAP_SQRT: return sqrt(x);
    case ELX_MAP_EXP: return exp(x);
    case ELX_MAP_LOG: return log(x);
    case ELX_MAP_RELU: return x > C(0) ? x : C(0);
    case ELX_MAP_SIGMOID: return C(1) / (C(1) + exp(-x));
    case ELX_MAP_RECIP: return C(1) / x;
    case ELX_MAP_TANH: return tanh(x);
    default: return x;
    }
}

template <typename T, int FN>
__global__ __launch_bounds__(NT) void map_kernel(i64 m, i64 n, const typename Elem<T>::storage* A, i64 lda,
                                                 typename Elem<T>::storage* B, i64 ldb) {
    using E = Elem<T>;
    for_each_2d(m, n, [&](i64 i, i64 j) { B[i + j * ldb] = E::store(apply_map(FN, E::load(A[i + j * lda]))); });
}

template <typename T>
__global__ __launch_bounds__(NT) void hash_kernel(i64 m, i64 n, typename Elem<T>::storage* A, i64 lda, i64 i0,
                                                  i64 istride, i64 j0, i64 jstride, uint64_t seed,
                                                  double center, double radius) {
    using E = Elem<T>;
    for_each_2d(m, n, [&](i64 i, i64 j) {
#pragma clang fp contract(off)
        const double u = hash_unit(seed, i0 + i * istride, j0 + j * jstride);
        // explicit roundings: no FMA contraction, so host and device agree bit for bit
        // plain operators under `contract(off)`: the instructions are created in
        // this scope, so no fused multiply-add can merge them (host == device)
        const double v = center + radius * (2.0 * u - 1.0);
        A[i + j * lda] = E::store((typename E::compute)v);  // double -> compute (RNE) -> storage (RNE)
    });
}

dim3 grid2d(i64 m, i64 n) {
    i64 gx = (m + NT - 1) / NT;
    if (gx > 64) gx = 64;
    if (gx < 1) gx = 1;
    i64 gy = n < 1 ? 1 : n;
    if (gy > 4096) gy = 4096;
    return dim3((unsigned)gx, (unsigned)gy);
}

#define ELX_DTYPE_SWITCH(dtype, T, ...)                 \
    switch (dtype) {                                    \
    case ELX_F64: { using T = double; __VA_ARGS__; break; } \
    case ELX_F32: { using T = float; __VA_ARGS__; break; }  \
    case ELX_F16: { using T = f16_t; __VA_ARGS__; break; }  \
    case ELX_BF16: { using T = bf16_t; __VA_ARGS__; break; } \
    default: return hipErrorInvalidValue;               \
    }

}  // namespace

hipError_t copy2d_batch(int dtype, const Copy2D* d, int nd, bool axpy, double alpha, hipStream_t s) {
    for (int base = 0; base < nd; base += kMaxCopyBatch) {
        CopyBatch b{};
        const int cnt = (nd - base) < kMaxCopyBatch ? (nd - base) : kMaxCopyBatch;
        i64 maxtiles = 0;
        int used = 0;
        for (int q = 0; q < cnt; ++q) {
            const Copy2D& x = d[base + q];
            if (x.m <= 0 || x.n <= 0) continue;
            b.d[used++] = x;
            const i64 t = ((x.m + TILE - 1) / TILE) * ((x.n + TILE - 1) / TILE);
            if (t > maxtiles) maxtiles = t;
        }
        if (used == 0) continue;
        const unsigned gx = (unsigned)(maxtiles > 4096 ? 4096 : maxtiles);
        dim3 grid(gx, used);
        ELX_DTYPE_SWITCH(dtype, T,
            if (axpy) hipLaunchKernelGGL((copy2d_kernel<T, true>), grid, dim3(NT), 0, s, b, alpha);
            else hipLaunchKernelGGL((copy2d_kernel<T, false>), grid, dim3(NT), 0, s, b, alpha));
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t fill2d(int dtype, i64 m, i64 n, double v, void* A, i64 lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T,
        hipLaunchKernelGGL((fill_kernel<T>), grid2d(m, n), dim3(NT), 0, s, m, n, v,
                           static_cast<typename Elem<T>::storage*>(A), lda));
    return hipGetLastError();
}

hipError_t scale2d(int dtype, i64 m, i64 n, double alpha, void* A, i64 lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T,
        hipLaunchKernelGGL((scale_kernel<T>), grid2d(m, n), dim3(NT), 0, s, m, n, alpha,
                           static_cast<typename Elem<T>::storage*>(A), lda));
    return hipGetLastError();
}

hipError_t hadamard2d(int dtype, i64 m, i64 n, const void* A, i64 lda, const void* B, i64 ldb, void* C,
                      i64 ldc, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T, {
        using S = typename Elem<T>::storage;
        hipLaunchKernelGGL((hadamard_kernel<T>), grid2d(m, n), dim3(NT), 0, s, m, n,
                           static_cast<const S*>(A), lda, static_cast<const S*>(B), ldb,
                           static_cast<S*>(C), ldc);
    });
    return hipGetLastError();
}

template <typename T, int FN>
static void launch_map(dim3 g, hipStream_t s, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb) {
    using S = typename Elem<T>::storage;
    hipLaunchKernelGGL((map_kernel<T, FN>), g, dim3(NT), 0, s, m, n, static_cast<const S*>(A), lda,
                       static_cast<S*>(B), ldb);
}

hipError_t entrywise_map(int dtype, int fn, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb,
                         hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    const dim3 g = grid2d(m, n);
#define ELX_MAP_CASE(F) case F: launch_map<T, F>(g, s, m, n, A, lda, B, ldb); break;
    ELX_DTYPE_SWITCH(dtype, T, switch (fn) {
        ELX_MAP_CASE(ELX_MAP_IDENTITY) ELX_MAP_CASE(ELX_MAP_NEGATE) ELX_MAP_CASE(ELX_MAP_ABS)
        ELX_MAP_CASE(ELX_MAP_SQUARE) ELX_MAP_CASE(ELX_MAP_SQRT) ELX_MAP_CASE(ELX_MAP_EXP)
        ELX_MAP_CASE(ELX_MAP_LOG) ELX_MAP_CASE(ELX_MAP_RELU) ELX_MAP_CASE(ELX_MAP_SIGMOID)
        ELX_MAP_CASE(ELX_MAP_RECIP) ELX_MAP_CASE(ELX_MAP_TANH)
        default: return hipErrorInvalidValue;
    });
#undef ELX_MAP_CASE
    return hipGetLastError();
}

hipError_t fill_hash(int dtype, i64 m, i64 n, void* A, i64 lda, i64 i0, i64 istride, i64 j0, i64 jstride,
                     uint64_t seed, double center, double radius, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T,
        hipLaunchKernelGGL((hash_kernel<T>), grid2d(m, n), dim3(NT), 0, s, m, n,
                           static_cast<typename Elem<T>::storage*>(A), lda, i0, istride, j0, jstride,
                           seed, center, radius));
    return hipGetLastError();
}

}  // namespace kern
}  // namespace elx
