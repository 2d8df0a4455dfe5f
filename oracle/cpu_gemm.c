/*
 * cpu_gemm.c — the CPU baseline leg of bench.py.  TEST INFRASTRUCTURE: only
 * bench.py's cpu_baseline (and tests/ as a checker of it) call this.
 *
 * The reference's CPU path for the local panel update is a multi-threaded BLAS
 * dgemm (EL_BLAS(dgemm), src/core/imports/blas/Gemm.hpp:13-40; MKL in the
 * survey's measurement).  This is a port of that role, not of
 * MKL: a cache-blocked, packed, OpenMP-parallel GEMM (GotoBLAS-style loop
 * order jc / pc / ic with an 8 x 6 register micro-kernel), so the baseline
 * reported next to the GPU number is a fair multi-core CPU GEMM on the GPU
 * box's own cores rather than the naive loop nest of oracle.c.
 * Semantics are BLAS: C := alpha op(A) op(B) + beta C, column-major; beta == 0
 * never reads C.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef double v4d __attribute__((vector_size(32)));

enum { MR = 8, NR = 6, MC = 96, KC = 256, NC = 96 };

static inline double opA(char ta, const double* A, int64_t lda, int64_t i, int64_t l) {
    return ta == 'N' ? A[i + l * lda] : A[l + i * lda];
}
static inline double opB(char tb, const double* B, int64_t ldb, int64_t l, int64_t j) {
    return tb == 'N' ? B[l + j * ldb] : B[j + l * ldb];
}

/* Ap[s][l][r] = alpha * op(A)(i0 + s*MR + r, l0 + l), zero-padded to MR rows */
static void pack_a(char ta, const double* A, int64_t lda, int64_t i0, int64_t mb, int64_t l0, int64_t kb,
                   double alpha, double* Ap) {
    for (int64_t s = 0; s < (mb + MR - 1) / MR; ++s)
        for (int64_t l = 0; l < kb; ++l)
            for (int r = 0; r < MR; ++r) {
                const int64_t i = s * MR + r;
                Ap[(s * kb + l) * MR + r] = i < mb ? alpha * opA(ta, A, lda, i0 + i, l0 + l) : 0.0;
            }
}
/* Bp[s][l][c] = op(B)(l0 + l, j0 + s*NR + c), zero-padded to NR columns */
static void pack_b(char tb, const double* B, int64_t ldb, int64_t l0, int64_t kb, int64_t j0, int64_t nb,
                   double* Bp) {
    for (int64_t s = 0; s < (nb + NR - 1) / NR; ++s)
        for (int64_t l = 0; l < kb; ++l)
            for (int c = 0; c < NR; ++c) {
                const int64_t j = s * NR + c;
                Bp[(s * kb + l) * NR + c] = j < nb ? opB(tb, B, ldb, l0 + l, j0 + j) : 0.0;
            }
}

/* C[0:mr, 0:nr] += Ap-sliver * Bp-sliver (kb deep) */
static void micro(int64_t kb, const double* a, const double* b, double* C, int64_t ldc, int mr, int nr) {
    v4d c0[NR], c1[NR];
    for (int j = 0; j < NR; ++j) {
        c0[j] = (v4d){0, 0, 0, 0};
        c1[j] = (v4d){0, 0, 0, 0};
    }
    for (int64_t l = 0; l < kb; ++l) {
        v4d a0, a1;
        memcpy(&a0, a + l * MR, sizeof a0);
        memcpy(&a1, a + l * MR + 4, sizeof a1);
        for (int j = 0; j < NR; ++j) {
            const double bj = b[l * NR + j];
            const v4d bv = {bj, bj, bj, bj};
            c0[j] += a0 * bv;
            c1[j] += a1 * bv;
        }
    }
    for (int j = 0; j < nr; ++j)
        for (int r = 0; r < mr; ++r) C[r + j * ldc] += r < 4 ? c0[j][r] : c1[j][r - 4];
}

void orc_cpu_gemm_f64(char ta, char tb, int64_t m, int64_t n, int64_t k, double alpha, const double* A, int64_t lda,
                      const double* B, int64_t ldb, double beta, double* C, int64_t ldc) {
    if (m <= 0 || n <= 0) return;
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i) C[i + j * ldc] = beta == 0.0 ? 0.0 : beta * C[i + j * ldc];
    if (k <= 0 || alpha == 0.0) return;
    const int64_t ncb = (n + NC - 1) / NC;
#pragma omp parallel
    {
        double* Ap = (double*)malloc(sizeof(double) * (MC + MR) * KC);
        double* Bp = (double*)malloc(sizeof(double) * (NC + NR) * KC);
#pragma omp for schedule(dynamic, 1)
        for (int64_t jb = 0; jb < ncb; ++jb) {
            const int64_t j0 = jb * NC, nb = (n - j0) < NC ? (n - j0) : NC;
            for (int64_t l0 = 0; l0 < k; l0 += KC) {
                const int64_t kb = (k - l0) < KC ? (k - l0) : KC;
                pack_b(tb, B, ldb, l0, kb, j0, nb, Bp);
                for (int64_t i0 = 0; i0 < m; i0 += MC) {
                    const int64_t mb = (m - i0) < MC ? (m - i0) : MC;
                    pack_a(ta, A, lda, i0, mb, l0, kb, alpha, Ap);
                    for (int64_t js = 0; js < (nb + NR - 1) / NR; ++js)
                        for (int64_t is = 0; is < (mb + MR - 1) / MR; ++is) {
                            const int mr = (int)((mb - is * MR) < MR ? (mb - is * MR) : MR);
                            const int nr = (int)((nb - js * NR) < NR ? (nb - js * NR) : NR);
                            micro(kb, Ap + is * kb * MR, Bp + js * kb * NR, C + (i0 + is * MR) + (j0 + js * NR) * ldc,
                                  ldc, mr, nr);
                        }
                }
            }
        }
        free(Ap);
        free(Bp);
    }
}

int orc_cpu_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* threads of this process's later parallel regions (OMP_NUM_THREADS is read
 * once, when the OpenMP runtime loads, possibly before the caller could set it) */
void orc_cpu_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
