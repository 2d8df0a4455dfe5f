// El::Gemm / El::LocalGemm on DistMatrices: the SUMMA drivers.
#pragma once
#include "distmatrix.hpp"

namespace elx {

enum Orientation { NORMAL = ELX_NORMAL, TRANSPOSE = ELX_TRANSPOSE, ADJOINT = ELX_ADJOINT };

// C := alpha op(A) op(B) + beta C  (src/blas_like/level3/Gemm.cpp:273-302)
void Gemm(int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, double beta, DistMatrix& C,
          int alg);
// local update on the local blocks, with the reference's conformance checks
void LocalGemm(int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, double beta, DistMatrix& C);
// beta-less form: aligns and resizes C, then beta = 0
void LocalGemmResize(int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, DistMatrix& C);

// A := alpha A on its lower/upper trapezoid (ScaleTrapezoid.hpp:47-88)
void ScaleTrapezoid(double alpha, int uplo, DistMatrix& A, Int offset);
// C := alpha op(A) op(A)^T + beta C on C's lower/upper triangle (Syrk.cpp:196-211; Herk for real T)
void Syrk(int uplo, int orient, double alpha, const DistMatrix& A, double beta, DistMatrix& C);
// C := alpha op(A) op(B) + beta C on C's uplo triangle (Trrk.cpp:100-117)
void Trrk(int uplo, int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, double beta,
          DistMatrix& C);
// C := alpha (op(A) op(B)^T + op(B) op(A)^T) + beta C on C's uplo triangle (Syr2k.cpp:78-93)
void Syr2k(int uplo, int orient, double alpha, const DistMatrix& A, const DistMatrix& B, double beta,
           DistMatrix& C);
// B := alpha op(A)^-1 B (LEFT) / alpha B op(A)^-1 (RIGHT)  (Trsm.cpp:129-420)
// checkIfSingular: SingularMatrixError when a NON_UNIT diagonal holds an exact zero (Trsm.cpp:60-68)
void Trsm(int side, int uplo, int orient, int diag, double alpha, const DistMatrix& A, DistMatrix& B,
          bool checkIfSingular = false);
// C := alpha A B + beta C (LEFT) / alpha B A + beta C (RIGHT), A symmetric (uplo stored)  (Symm.cpp:55-80)
void Symm(int side, int uplo, double alpha, const DistMatrix& A, const DistMatrix& B, double beta, DistMatrix& C);

void SetBlocksize(Int nb);
Int Blocksize();
void PushBlocksizeStack(Int nb);
void PopBlocksizeStack();
void EmptyBlocksizeStack();
void SetComputePanel(Int kc);
Int ComputePanel();
int LastGemmAlgorithm();
// stream pool of the multistream variants (hydrogen::SyncInfoPool); 0 = H_STREAMPOOL_SIZE
void SetStreamPoolSize(int n);
int StreamPoolSize();
void SetProfiling(bool on);
void ProfileStats(double& gemm_ms, int64_t& launches, double& flops, double& comm_ms, int64_t& bytes);
void CommProfileStats(double& transfer_ms, int64_t& bytes, int64_t& transfers);
void PipelineStats(double& gap_ms, int64_t& gaps);

}  // namespace elx
