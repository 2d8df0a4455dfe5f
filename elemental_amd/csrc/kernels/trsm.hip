// Local triangular solve with many right-hand sides: the diagonal-block solve
// of the distributed Trsm (LocalTrsm on L11[*,*] and X1[*,VR], Trsm/LLN.hpp:53-59;
// the reference's GPU build calls rocblas_{s,d}trsm through gpu_blas::Trsm).
//
// Solve op(A) X = B in place, A m x m (only its uplo triangle is read; unit
// diagonal when `unit`), B m x n column-major.  One wavefront owns 64 right-hand
// sides: its columns are staged once into LDS as x[row][lane] (each lane's
// column stays in LDS for the whole substitution; op(A) entries are wave-uniform
// loads that hit the L1/L2), then written back.  Column-oriented substitution:
// x_i /= a_ii, then x_r -= a_ri x_i for the rows r still to come.  m is the
// distributed block size (<= MAXM rows per LDS pass; larger m falls back to the
// same loop on global memory).  The substitution is a dependent chain per lane,
// so with many right-hand sides exec::Trsm instead inverts the block (IDENT: the
// identity as right-hand sides, m lanes) and applies op(A)^-1 as one MFMA GEMM.
#include "kernels.hpp"
#include "../common.hpp"

namespace elx {
namespace kern {
namespace {

constexpr int WAVE = 64;

// IDENT: the right-hand sides are the identity (B is output only): B := op(A)^-1
template <typename T, bool LDS, bool IDENT>
__device__ __forceinline__ void trsm_body(bool lower, bool trans, bool unit, i64 m, i64 n, const T* A, i64 lda, T* B,
                                          i64 ldb) {
    extern __shared__ unsigned char smem[];
    T* x = reinterpret_cast<T*>(smem);
    const i64 col = (i64)blockIdx.x * WAVE + threadIdx.x;
    const bool live = col < n;
    T* bcol = B + (live ? col : 0) * ldb;
    // element (r) of this lane's right-hand side
    auto X = [&](i64 r) -> T& { return LDS ? x[r * WAVE + threadIdx.x] : bcol[r]; };
    if (live) {
        if (IDENT)
            for (i64 r = 0; r < m; ++r) X(r) = r == col ? T(1) : T(0);
        else if (LDS)
            for (i64 r = 0; r < m; ++r) x[r * WAVE + threadIdx.x] = bcol[r];
    }
    auto opA = [&](i64 r, i64 c) { return trans ? A[c + r * lda] : A[r + c * lda]; };
    const bool forward = lower != trans;  // op(A) lower triangular
    // LDS mode: column i of op(A) is staged into LDS by the whole wave before
    // the step (independent loads, one latency per step instead of one per row)
    T* acol = x + m * WAVE;
    for (i64 s = 0; s < m; ++s) {
        const i64 i = forward ? s : m - 1 - s;
        const i64 lo = forward ? i : 0, hi = forward ? m : i + 1;  // rows touched by step i
        if (LDS) {
            __syncthreads();
            for (i64 r = lo + threadIdx.x; r < hi; r += WAVE) acol[r] = opA(r, i);
            __syncthreads();
        }
        if (!live) continue;
        T xi = X(i);
        if (!unit) xi = xi / (LDS ? acol[i] : opA(i, i));
        X(i) = xi;
        // rows [r0, r1) -= op(A)(r, i) x_i, eight rows per batch: all sixteen
        // loads issued before the first FMA (one LDS latency per batch, not per row)
        const i64 r0 = forward ? i + 1 : 0, r1 = forward ? m : i;
        i64 r = r0;
        if (LDS) {
            for (; r + 8 <= r1; r += 8) {
                T xv[8], av[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    xv[u] = X(r + u);
                    av[u] = acol[r + u];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) X(r + u) = xv[u] - av[u] * xi;
            }
        }
        for (; r < r1; ++r) X(r) = X(r) - (LDS ? acol[r] : opA(r, i)) * xi;
    }
    if (LDS && live)
        for (i64 r = 0; r < m; ++r) bcol[r] = x[r * WAVE + threadIdx.x];
}

template <typename T, bool LDS, bool IDENT>
__global__ __launch_bounds__(WAVE) void trsm_kernel(bool lower, bool trans, bool unit, i64 m, i64 n, const T* A,
                                                    i64 lda, T* B, i64 ldb) {
    trsm_body<T, LDS, IDENT>(lower, trans, unit, m, n, A, lda, B, ldb);
}

// Every diagonal block of A at once: blockIdx.y = block b (rows/cols [b*nb,
// min(m, (b+1)*nb))), W_b = op(A_bb)^-1 at W + b*nb*nb with leading dimension nb.
template <typename T>
__global__ __launch_bounds__(WAVE) void tri_inverse_batched_kernel(bool lower, bool trans, bool unit, i64 nb, i64 m,
                                                                   const T* A, i64 lda, T* W) {
    const i64 b = blockIdx.y, r0 = b * nb;
    const i64 sz = (m - r0) < nb ? (m - r0) : nb;
    trsm_body<T, true, true>(lower, trans, unit, sz, sz, A + r0 + r0 * lda, lda, W + b * nb * nb, nb);
}

template <typename T>
hipError_t launch_trsm(bool ident, bool lower, bool trans, bool unit, i64 m, i64 n, const T* A, i64 lda, T* B,
                       i64 ldb, hipStream_t s) {
    const dim3 grid((unsigned)((n + WAVE - 1) / WAVE));
    const size_t lds = (size_t)m * (WAVE + 1) * sizeof(T);
    if (lds <= 66 * 1024) {
        if (ident)
            hipLaunchKernelGGL((trsm_kernel<T, true, true>), grid, dim3(WAVE), lds, s, lower, trans, unit, m, n, A, lda, B, ldb);
        else
            hipLaunchKernelGGL((trsm_kernel<T, true, false>), grid, dim3(WAVE), lds, s, lower, trans, unit, m, n, A, lda, B, ldb);
    } else {
        if (ident)
            hipLaunchKernelGGL((trsm_kernel<T, false, true>), grid, dim3(WAVE), 0, s, lower, trans, unit, m, n, A, lda, B, ldb);
        else
            hipLaunchKernelGGL((trsm_kernel<T, false, false>), grid, dim3(WAVE), 0, s, lower, trans, unit, m, n, A, lda, B, ldb);
    }
    return hipGetLastError();
}

}  // namespace

bool tri_inverse_lds_ok(int dtype, i64 nb) {
    const int es = dtype == ELX_F64 ? 8 : 4;
    const size_t lds = (size_t)nb * (WAVE + 1) * es;
    if (lds > (size_t)kTriInverseLdsMax || (dtype != ELX_F64 && dtype != ELX_F32)) return false;
    if (lds <= 64 * 1024) return true;
    const void* f = dtype == ELX_F64 ? reinterpret_cast<const void*>(&tri_inverse_batched_kernel<double>)
                                     : reinterpret_cast<const void*>(&tri_inverse_batched_kernel<float>);
    return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
}

hipError_t tri_inverse_batched(int dtype, bool lower, bool trans, bool unit, i64 nb, i64 m, const void* A, i64 lda,
                               void* W, hipStream_t s) {
    if (m <= 0 || nb <= 0) return hipSuccess;
    const i64 nblk = (m + nb - 1) / nb;
    const int es = dtype == ELX_F64 ? 8 : 4;
    const size_t lds = (size_t)nb * (WAVE + 1) * es;
    if (lds > (size_t)kTriInverseLdsMax || nblk > 65535) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((nb + WAVE - 1) / WAVE), (unsigned)nblk);
    switch (dtype) {
    case ELX_F64:
        if (lds > 64 * 1024) {  // beyond the default dynamic-LDS limit (gfx950: 160 KiB per workgroup)
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&tri_inverse_batched_kernel<double>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((tri_inverse_batched_kernel<double>), grid, dim3(WAVE), lds, s, lower, trans, unit, nb, m,
                           static_cast<const double*>(A), lda, static_cast<double*>(W));
        break;
    case ELX_F32:
        if (lds > 64 * 1024) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&tri_inverse_batched_kernel<float>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((tri_inverse_batched_kernel<float>), grid, dim3(WAVE), lds, s, lower, trans, unit, nb, m,
                           static_cast<const float*>(A), lda, static_cast<float*>(W));
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t trsm_local(int dtype, bool ident, bool lower, bool trans, bool unit, i64 m, i64 n, const void* A, i64 lda,
                      void* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    if (n > (i64)WAVE * 0x7fffffff) return hipErrorInvalidValue;
    switch (dtype) {
    case ELX_F64:
        return launch_trsm(ident, lower, trans, unit, m, n, static_cast<const double*>(A), lda, static_cast<double*>(B), ldb, s);
    case ELX_F32:
        return launch_trsm(ident, lower, trans, unit, m, n, static_cast<const float*>(A), lda, static_cast<float*>(B), ldb, s);
    default:
        return hipErrorInvalidValue;
    }
}

}  // namespace kern
}  // namespace elx
