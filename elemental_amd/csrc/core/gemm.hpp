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

void SetBlocksize(Int nb);
Int Blocksize();
void SetComputePanel(Int kc);
Int ComputePanel();
int LastGemmAlgorithm();
void SetProfiling(bool on);
void ProfileStats(double& gemm_ms, int64_t& launches, double& flops, double& comm_ms, int64_t& bytes);

}  // namespace elx
