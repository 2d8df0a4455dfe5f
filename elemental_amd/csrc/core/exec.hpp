// Device-dispatched local primitives.  Device::GPU launches the gfx950 kernels
// (elemental_amd/csrc/kernels); Device::CPU runs the host loops that back the
// reference's Device::CPU DistMatrix path (used when a caller builds CPU
// matrices, e.g. the gloo multi-rank tests).  A GPU matrix never runs here on
// the host: there is no fallback between the two.
#pragma once
#include "../common.hpp"
#include "../runtime/runtime.hpp"
#include "../kernels/kernels.hpp"

namespace elx {
namespace exec {

using kern::Copy2D;

void Copy2DBatch(Device dev, DType t, const Copy2D* d, int nd, bool axpy, double alpha, hipStream_t s);
// dst(i,j) += alpha*src_q(i,j) for every q in order, each rounded to the storage
// type: the rank-ordered sum of AxpyContract in one pass over dst (any number of
// sources: groups of kern::kMaxContractSources, in order)
struct ContractSource { const void* p; Int cs, rs; };
void ContractSum(Device dev, DType t, Int m, Int n, void* dst, Int dcs, Int drs, const ContractSource* src,
                 int nsrc, double alpha, hipStream_t s);
// dst(i,j) = (dst type) src(i,j): Copy_GPU_impl<SrcT,DestT> (Copy.cu:93-205)
void Convert2D(Device dev, DType src_t, DType dst_t, const Copy2D& d, hipStream_t s);
void Gemm(Device dev, DType t, bool ta, bool tb, Int m, Int n, Int k, double alpha,
          const void* A, Int lda, const void* B, Int ldb, double beta, void* C, Int ldc, hipStream_t s);
void Fill(Device dev, DType t, Int m, Int n, double v, void* A, Int lda, hipStream_t s);
void Scale(Device dev, DType t, Int m, Int n, double alpha, void* A, Int lda, hipStream_t s);
// Frobenius-norm pieces: max |a| (NaN propagates) and sum (a / scale)^2, in double
double AbsMax(Device dev, DType t, Int m, Int n, const void* A, Int lda, hipStream_t s);
double ScaledSumSq(Device dev, DType t, Int m, Int n, const void* A, Int lda, double scale, hipStream_t s);
void Hadamard(Device dev, DType t, Int m, Int n, const void* A, Int lda, const void* B, Int ldb,
              void* C, Int ldc, hipStream_t s);
void Map(Device dev, DType t, int fn, Int m, Int n, const void* A, Int lda, void* B, Int ldb, hipStream_t s);
void Combine(Device dev, DType t, int fn, Int m, Int n, const void* A, Int lda, void* B, Int ldb, hipStream_t s);
// Y := beta*Y + alpha*X (X null: beta*Y) on the lower/upper trapezoid of the
// global index map (i0 + i*is, j0 + j*js) (ScaleTrapezoid.hpp, AxpyTrapezoid)
void Trapezoid(Device dev, DType t, bool lower, Int m, Int n, double alpha, const void* X, Int ldx, double beta,
               void* Y, Int ldy, Int i0, Int is, Int j0, Int js, Int offset, hipStream_t s);
// op(A) X = B in place, A m x m (LocalTrsm / blas::Trsm, Left side); f64/f32
void Trsm(Device dev, DType t, bool lower, bool trans, bool unit, Int m, Int n, const void* A, Int lda, void* B,
          Int ldb, hipStream_t s);
// GPU only: W_b := op(A_bb)^-1 for every nb x nb diagonal block of the m x m A
// (W_b at W + b*nb*nb, leading dimension nb), one launch
void TriInverseBatched(DType t, bool lower, bool trans, bool unit, Int nb, Int m, const void* A, Int lda, void* W,
                       hipStream_t s);
// B := W B (W m x m) through a workspace: one MFMA GEMM + one copy
void ApplyInverse(Device dev, DType t, Int m, Int n, const void* W, Int ldw, void* B, Int ldb, hipStream_t s);
void FillHash(Device dev, DType t, Int m, Int n, void* A, Int lda, Int i0, Int is, Int j0, Int js,
              uint64_t seed, double center, double radius, hipStream_t s);
// host-side scalar conversion of one element (for Get/Set and tests)
double LoadScalar(DType t, const void* p);
void StoreScalar(DType t, void* p, double v);

}  // namespace exec
}  // namespace elx
