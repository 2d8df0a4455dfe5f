// The DistMatrix redistribution engine and the distributed BLAS-1 front doors.
#pragma once
#include <utility>
#include <vector>
#include "distmatrix.hpp"

namespace elx {

// B := A (DistMatrix::operator=), any element-wise pair, any alignments.
void Copy(const DistMatrix& A, DistMatrix& B);
// Several Copy(A_i, B_i) whose exchanges share one grouped all-to-all (targets
// on one stream, same type and device on one grid; otherwise plain Copy each)
void CopyGroup(const std::vector<std::pair<const DistMatrix*, DistMatrix*>>& pairs);
// B := A^T (El::Transpose on DistMatrices; ADJOINT == TRANSPOSE for real types)
void Transpose(const DistMatrix& A, DistMatrix& B);
// B += alpha * (sum of A's redundant partial copies), redistributed to B (AxpyContract)
void AxpyContract(double alpha, const DistMatrix& A, DistMatrix& B);
// same, but B's data first comes from A^T (TransposeAxpyContract)
void TransposeAxpyContract(double alpha, const DistMatrix& A, DistMatrix& B);

void Axpy(double alpha, const DistMatrix& X, DistMatrix& Y);
void Scale(double alpha, DistMatrix& A);
void Zero(DistMatrix& A);
void Hadamard(const DistMatrix& A, const DistMatrix& B, DistMatrix& C);
void EntrywiseMap(int fn, const DistMatrix& A, DistMatrix& B);
// B := f(A, B) on the local blocks (Combine, EntrywiseMap.hpp:187-202): same
// size, distribution, alignment and device, else RuntimeError / LogicError
void Combine(int fn, const DistMatrix& A, DistMatrix& B);

// true iff A's local block already is B-with-B's-alignment's local block
// (same owner of every element): lets SUMMA use views instead of copies.
bool SameLocalLayout(const DistMatrix& A, Dist cd, Dist rd, int calign, int ralign);

// entry access (El::DistMatrix::Get is collective; Set/Update write the local copies)
double Get(const DistMatrix& A, Int i, Int j);
void Set(DistMatrix& A, Int i, Int j, double v);
void Update(DistMatrix& A, Int i, Int j, double v);
// El::Fill: every entry := v
void Fill(DistMatrix& A, double v);
// collective: is any diagonal entry exactly zero?  (Trsm's checkIfSingular)
bool DiagonalHasZero(const DistMatrix& A);
// El::FrobeniusNorm (src/lapack_like/norm/Frobenius.cpp): collective over the grid,
// each entry counted once however many ranks hold a copy of it
double FrobeniusNorm(const DistMatrix& A);
// grid-wide scalar sum / broadcast from VC rank `rootVC`
double GridAllReduceSum(const Grid& g, double v);
double GridAllReduceMax(const Grid& g, double v);
double GridBcast(const Grid& g, double v, int rootVC);

}  // namespace elx
