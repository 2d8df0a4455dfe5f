// El::InitializeRandom / Uniform / MakeUniform (the reference's test-input RNG).
#pragma once
#include "distmatrix.hpp"

namespace elx {

// seed the process-global generator: (secs << 16) | rank, secs = 21 if deterministic
void InitializeRandom(bool deterministic, int worldRank);
// A(i,j) ~ U[center - radius, center + radius) drawn as the reference draws it
void MakeUniform(DistMatrix& A, double center, double radius);
void Uniform(DistMatrix& A, Int m, Int n, double center, double radius);

}  // namespace elx
