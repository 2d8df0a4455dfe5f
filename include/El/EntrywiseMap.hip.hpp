// El/EntrywiseMap.hip.hpp — functor-generic entrywise kernels for GPU matrices,
// header-only, compiled by the CALLER's hipcc (as the reference's device
// templates are: include/hydrogen/blas/gpu/EntrywiseMapImpl.hpp:36-211,
// CombineImpl.hpp:47-213, and the GPU overloads of
// include/El/blas_like/level1/EntrywiseMap.hpp:141-203).  Any device-callable
// functor works: a __device__ / __host__ __device__ lambda or a struct with a
// __device__ operator().  The library's C-ABI cannot carry such a functor, so
// these launch their own kernels on the target matrix's stream; the closed
// functor set behind elx_entrywise_map / elx_combine stays available for
// callers that do not compile HIP.
//
//   #include <El.hpp>      // (El.hpp pulls this header in under __HIPCC__)
//   El::EntrywiseMap(A.LockedMatrix(), B.Matrix(), [] __device__ (double x) { return x > 0 ? x : 0.1 * x; });
//   El::Combine(A.LockedMatrix(), B.Matrix(), [] __device__ (double a, double b) { return a * b + 1; });
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../El.hpp"

namespace El {
namespace device {

// One workgroup of 256 lanes walks a column chunk of 1024 rows per pass; each
// lane loads its four elements before computing, so four independent loads
// are in flight per lane (the op is HBM-bound: 64-wide wavefronts read 64
// consecutive elements per instruction, fully coalesced for column-major data).
constexpr int kMapThreads = 256;
constexpr int kMapUnroll = 4;
constexpr Int kMapRows = Int(kMapThreads) * kMapUnroll;

template <typename S, typename T, typename F>
__global__ __launch_bounds__(kMapThreads) void EntrywiseMapKernel(Int m, Int n, const S* __restrict__ A, Int lda,
                                                                   T* __restrict__ B, Int ldb, F f) {
    const Int chunks = (m + kMapRows - 1) / kMapRows;
    for (Int id = blockIdx.x; id < chunks * n; id += gridDim.x) {
        const Int j = id / chunks, i0 = (id - j * chunks) * kMapRows + threadIdx.x;
        S x[kMapUnroll];
#pragma unroll
        for (int u = 0; u < kMapUnroll; ++u) {
            const Int i = i0 + u * kMapThreads;
            if (i < m) x[u] = A[i + j * lda];
        }
#pragma unroll
        for (int u = 0; u < kMapUnroll; ++u) {
            const Int i = i0 + u * kMapThreads;
            if (i < m) B[i + j * ldb] = f(x[u]);
        }
    }
}

// B(i,j) := f(A(i,j), B(i,j))
template <typename S, typename T, typename F>
__global__ __launch_bounds__(kMapThreads) void CombineKernel(Int m, Int n, const S* __restrict__ A, Int lda,
                                                              T* __restrict__ B, Int ldb, F f) {
    const Int chunks = (m + kMapRows - 1) / kMapRows;
    for (Int id = blockIdx.x; id < chunks * n; id += gridDim.x) {
        const Int j = id / chunks, i0 = (id - j * chunks) * kMapRows + threadIdx.x;
        S x[kMapUnroll];
        T y[kMapUnroll];
#pragma unroll
        for (int u = 0; u < kMapUnroll; ++u) {
            const Int i = i0 + u * kMapThreads;
            if (i < m) {
                x[u] = A[i + j * lda];
                y[u] = B[i + j * ldb];
            }
        }
#pragma unroll
        for (int u = 0; u < kMapUnroll; ++u) {
            const Int i = i0 + u * kMapThreads;
            if (i < m) B[i + j * ldb] = f(x[u], y[u]);
        }
    }
}

inline void Check(hipError_t e, const char* what) {
    if (e != hipSuccess)
        throw hydrogen_errors::GPUError(std::string(what) + ": " + hipGetErrorString(e));
}

// MultiSync (include/hydrogen/MultiSync.hpp:33-78) for one read operand:
// `master` waits for `other`'s queued work now; `other` waits for master's on exit
struct PairSync {
    hipStream_t master, other;
    PairSync(void* m, void* o) : master(static_cast<hipStream_t>(m)), other(static_cast<hipStream_t>(o)) {
        Fence(other, master);
    }
    ~PairSync() {
        try { Fence(master, other); } catch (...) {}
    }
    static void Fence(hipStream_t from, hipStream_t to) {
        if (!from || !to || from == to) return;
        hipEvent_t ev;
        Check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreateWithFlags");
        Check(hipEventRecord(ev, from), "hipEventRecord");
        Check(hipStreamWaitEvent(to, ev, 0), "hipStreamWaitEvent");
        Check(hipEventDestroy(ev), "hipEventDestroy");
    }
};

inline unsigned GridFor(Int m, Int n) {
    const Int work = ((m + kMapRows - 1) / kMapRows) * n;
    return static_cast<unsigned>(std::max<Int>(1, std::min<Int>(work, 8192)));
}

// EntrywiseMapImpl (EntrywiseMapImpl.hpp:46-104): B := f(A) on an m x n block
template <typename S, typename T, typename F>
void EntrywiseMapImpl(Int m, Int n, const S* A, Int lda, T* B, Int ldb, F f, void* stream) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL((EntrywiseMapKernel<S, T, F>), dim3(GridFor(m, n)), dim3(kMapThreads), 0,
                       static_cast<hipStream_t>(stream), m, n, A, lda, B, ldb, f);
    Check(hipGetLastError(), "EntrywiseMapKernel launch");
}

// CombineImpl (CombineImpl.hpp:47-105): B := f(A, B)
template <typename S, typename T, typename F>
void CombineImpl(Int m, Int n, const S* A, Int lda, T* B, Int ldb, F f, void* stream) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL((CombineKernel<S, T, F>), dim3(GridFor(m, n)), dim3(kMapThreads), 0,
                       static_cast<hipStream_t>(stream), m, n, A, lda, B, ldb, f);
    Check(hipGetLastError(), "CombineKernel launch");
}

}  // namespace device

// EntrywiseMap(Matrix<S,GPU> const&, Matrix<T,GPU>&, FunctorT) (EntrywiseMap.hpp:154-168):
// B is resized to A's shape; the kernel runs on B's stream after A's queued work
template <typename S, typename T, typename FunctorT>
void EntrywiseMap(const Matrix<S, Device::GPU>& A, Matrix<T, Device::GPU>& B, FunctorT func) {
    B.Resize(A.Height(), A.Width());
    device::PairSync sync(B.Stream(), A.Stream());
    device::EntrywiseMapImpl(A.Height(), A.Width(), A.LockedBuffer(), A.LDim(), B.Buffer(), B.LDim(), func,
                             B.Stream());
}

// in place: A := f(A)
template <typename T, typename FunctorT>
void EntrywiseMap(Matrix<T, Device::GPU>& A, FunctorT func) {
    device::EntrywiseMapImpl(A.Height(), A.Width(), A.LockedBuffer(), A.LDim(), A.Buffer(), A.LDim(), func,
                             A.Stream());
}

// Combine(Matrix<S,GPU> const&, Matrix<T,GPU>&, FunctorT) (EntrywiseMap.hpp:187-202): B := f(A, B)
template <typename S, typename T, typename FunctorT>
void Combine(const Matrix<S, Device::GPU>& A, Matrix<T, Device::GPU>& B, FunctorT func) {
    if (A.Height() != B.Height() || A.Width() != B.Width())
        throw RuntimeError("A and B must be the same size for Combine.");
    device::PairSync sync(B.Stream(), A.Stream());
    device::CombineImpl(A.Height(), A.Width(), A.LockedBuffer(), A.LDim(), B.Buffer(), B.LDim(), func, B.Stream());
}

// DistMatrix forms (EntrywiseMap.hpp:90-137): with A in B's distribution the
// local blocks are mapped directly (B aligned with A); otherwise A is first
// redistributed into a temporary with B's distribution and alignment
// (EntrywiseMap_payload), then mapped
template <typename S, Dist U, Dist V, typename T, Dist X, Dist Y, typename FunctorT>
void EntrywiseMap(const DistMatrix<S, U, V, ELEMENT, Device::GPU>& A, DistMatrix<T, X, Y, ELEMENT, Device::GPU>& B,
                  FunctorT func) {
    if (U == X && V == Y) {
        B.AlignWith(A, false);
        B.Resize(A.Height(), A.Width());
        EntrywiseMap(A.LockedMatrix(), B.Matrix(), func);
        return;
    }
    B.Resize(A.Height(), A.Width());
    DistMatrix<S, X, Y, ELEMENT, Device::GPU> AProx(B.Grid());
    AProx.AlignWith(B, true);
    AProx.SetStream(B.Stream());
    AProx = A;
    EntrywiseMap(AProx.LockedMatrix(), B.Matrix(), func);
}

template <typename T, Dist U, Dist V, typename FunctorT>
void EntrywiseMap(DistMatrix<T, U, V, ELEMENT, Device::GPU>& A, FunctorT func) {
    EntrywiseMap(A.Matrix(), func);
}

// Combine on DistMatrices: same size, distribution and alignment, local blocks
template <typename S, typename T, Dist U, Dist V, typename FunctorT>
void Combine(const DistMatrix<S, U, V, ELEMENT, Device::GPU>& A, DistMatrix<T, U, V, ELEMENT, Device::GPU>& B,
             FunctorT func) {
    if (A.Height() != B.Height() || A.Width() != B.Width())
        throw RuntimeError("A and B must be the same size for Combine.");
    if (A.ColAlign() != B.ColAlign() || A.RowAlign() != B.RowAlign())
        throw LogicError("Combine: A and B must be aligned");
    Combine(A.LockedMatrix(), B.Matrix(), func);
}

}  // namespace El
