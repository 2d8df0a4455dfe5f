/*
 * oracle.h — CPU restatement of the reference's El::Gemm path.  TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker.  Never linked into
 * libelemental_amd.so.  See oracle.c for the parity-pinning status.
 */
#ifndef ELX_ORACLE_H
#define ELX_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* include/El/core/indexing/impl.hpp:33-36,62-63,244-245 */
int64_t orc_shift(int64_t rank, int64_t align, int64_t stride);
int64_t orc_length(int64_t n, int64_t shift, int64_t stride);
int64_t orc_max_length(int64_t n, int64_t stride);
/* src/core/Grid.cpp:58-64 and :147-148 */
int orc_default_height(int p);
void orc_grid_coords(int r, int c, int order, int rank, int* mc, int* mr, int* vc, int* vr);
/* stride of / rank in a distribution (El::Dist ordinals); -1 = holds nothing */
void orc_md_coords(int r, int c, int vc, int* diag, int* pos);
int orc_dist_stride(int dist, int r, int c);
int orc_dist_rank(int dist, int r, int c, int vc, int root);
/* local block of global column-major G (es-byte elements) on VC rank vc,
 * for distribution [U,V] with alignments; returns local height/width */
void orc_local_block(const void* G, int64_t es, int64_t H, int64_t W, int64_t ldg, int U, int V, int r, int c,
                     int vc, int colAlign, int rowAlign, int root, void* out, int64_t ldo, int64_t* lh,
                     int64_t* lw);
/* inverse: scatter a local block back into global G */
void orc_place_block(void* G, int64_t es, int64_t H, int64_t W, int64_t ldg, int U, int V, int r, int c, int vc,
                     int colAlign, int rowAlign, int root, const void* loc, int64_t ldl);

/* grid-independent synthetic inputs (bit-identical to the library's fill) */
uint64_t orc_splitmix64(uint64_t z);
double orc_hash_unit(uint64_t seed, int64_t i, int64_t j);
void orc_hash_fill_f64(int64_t H, int64_t W, uint64_t seed, double center, double radius, double* G, int64_t ldg);
void orc_hash_fill_f32(int64_t H, int64_t W, uint64_t seed, double center, double radius, float* G, int64_t ldg);

/* BLAS GEMM semantics, restated from the reference's naive gemm
 * (src/core/imports/blas/Gemm.hpp:47-260; the same loop nest as netlib
 * DGEMM, which the reference calls through EL_BLAS(dgemm), :13-40).
 * ta/tb: 'N' or 'T'. */
void orc_gemm_f64(char ta, char tb, int64_t m, int64_t n, int64_t k, double alpha, const double* A, int64_t lda,
                  const double* B, int64_t ldb, double beta, double* C, int64_t ldc);
void orc_gemm_f32(char ta, char tb, int64_t m, int64_t n, int64_t k, float alpha, const float* A, int64_t lda,
                  const float* B, int64_t ldb, float beta, float* C, int64_t ldc);

/* SUMMA C-stationary over a simulated r x c grid, every rank's local update
 * done panel by panel exactly as SUMMA_NNC_impl (src/blas_like/level3/Gemm/NN.hpp:341-385):
 * C := alpha A B + beta C on global column-major matrices, nb = Blocksize(). */
void orc_summa_nnc_f64(int r, int c, int64_t m, int64_t n, int64_t k, int64_t nb, double alpha, const double* A,
                       int64_t lda, const double* B, int64_t ldb, double beta, double* C, int64_t ldc);

/* bench.py's CPU baseline (cpu_gemm.c): blocked, packed, OpenMP-parallel
 * BLAS-semantics dgemm standing in for the reference's multi-threaded BLAS
 * call (src/core/imports/blas/Gemm.hpp:13-40) */
void orc_cpu_gemm_f64(char ta, char tb, int64_t m, int64_t n, int64_t k, double alpha, const double* A, int64_t lda,
                      const double* B, int64_t ldb, double beta, double* C, int64_t ldc);
int orc_cpu_threads(void);
void orc_cpu_set_threads(int n);

/* parity metric of the north_star: ||C - Cref||_F / (||A||_F ||B||_F k eps) */
double orc_fro(int64_t m, int64_t n, const double* X, int64_t ldx);

#ifdef __cplusplus
}
#endif
#endif
