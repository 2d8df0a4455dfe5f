/*
 * oracle.c — CPU restatement of the reference (aj-prime/Elemental = LLNL
 * Hydrogen) El::Gemm path.  TEST INFRASTRUCTURE: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, always as
 * the checker / CPU baseline, never as the thing measured or shipped.
 *
 * Parity pinning:
 *  - The reference ships no golden vectors or fixture files for this path
 *    (SURVEY §4); its tests are self-consistency checks.  The reference itself
 *    needs its CMake build (generated El/config.h, hydrogen_config.h), MPI and
 *    BLAS, so under this round's rules it is treated as unbuildable here and is
 *    never compiled or run: no outputs of the reference pin this file.
 *  - What pins it instead: (1) the reference's own test procedures, restated in
 *    tests/ (associativity residual tests/blas_like/Gemm.cpp:15-49; GPU-vs-CPU
 *    elementwise check tests/blas_like/BasicGemm.cpp:84-94; redistribution
 *    round trip tests/core/DistMatrix.cpp:12-78), (2) known-answer inputs
 *    whose products are exact in binary floating point, (3) the published
 *    algorithm of the third-party BLAS the reference calls (netlib DGEMM loop
 *    nest == src/core/imports/blas/Gemm.hpp:47-260), and (4) the measured
 *    reference residuals recorded in BASELINE.md §2.  GEMM arithmetic parity is
 *    therefore "unpinned at the BLAS boundary" in the strict sense.
 */
#include "oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* El::Dist ordinals (include/El/core/types.hpp:207-217) */
enum { D_MC = 0, D_MD = 1, D_MR = 2, D_VC = 3, D_VR = 4, D_STAR = 5, D_CIRC = 6 };

/* Shift_(rank, align, stride) = mod(rank - align, stride): indexing/impl.hpp:244-245 */
int64_t orc_shift(int64_t rank, int64_t align, int64_t stride) {
    int64_t r = (rank - align) % stride;
    return r < 0 ? r + stride : r;
}
/* Length_(n, shift, stride): indexing/impl.hpp:33-36 */
int64_t orc_length(int64_t n, int64_t shift, int64_t stride) {
    return n > shift ? (n - shift - 1) / stride + 1 : 0;
}
/* MaxLength_: indexing/impl.hpp:62-63 */
int64_t orc_max_length(int64_t n, int64_t stride) { return n > 0 ? (n - 1) / stride + 1 : 0; }

/* Grid::DefaultHeight: src/core/Grid.cpp:58-64 */
int orc_default_height(int p) {
    int h = (int)sqrt((double)p);
    if (h < 1) h = 1;
    while (p % h != 0) ++h;
    return h;
}

/* Grid.cpp:125-148: column-major cart -> mc = rank % r, mr = rank / r;
 * vcRank = mc + r*mr, vrRank = mr + c*mc. */
void orc_grid_coords(int r, int c, int order, int rank, int* mc, int* mr, int* vc, int* vr) {
    if (order == 1) { *mc = rank % r; *mr = rank / r; }
    else { *mr = rank % c; *mc = rank / c; }
    *vc = *mc + r * *mr;
    *vr = *mr + c * *mc;
}

static int gcd_int(int a, int b) { while (b) { int t = a % b; a = b; b = t; } return a; }

/* Grid.cpp:105-107,157-185: diagonal index mod(mr - mc, gcd) and the position
 * along it, reached by walking (0, diag) -> (+1, +1) mod (r, c). */
void orc_md_coords(int r, int c, int vc, int* diag, int* pos) {
    const int mc = vc % r, mr = vc / r, g = gcd_int(r, c), lcm = r * c / g;
    int row = 0, col, k;
    *diag = ((mr - mc) % g + g) % g;
    col = *diag;
    *pos = 0;
    for (k = 0; k < lcm; ++k) {
        if (row == mc && col == mr) { *pos = k; return; }
        row = (row + 1) % r;
        col = (col + 1) % c;
    }
}

int orc_dist_stride(int dist, int r, int c) {
    switch (dist) {
    case D_MC: return r;
    case D_MR: return c;
    case D_VC: case D_VR: return r * c;
    case D_MD: return r * c / gcd_int(r, c);  /* MD_STAR.cpp:193: LCM */
    default: return 1;
    }
}

/* rank of vc in `dist`; for MD the root names the diagonal that holds the
 * matrix (CrossComm = MDPerp, MD_STAR.cpp:166-167) and the other diagonals
 * hold nothing */
int orc_dist_rank(int dist, int r, int c, int vc, int root) {
    const int mc = vc % r, mr = vc / r;
    int diag, pos;
    switch (dist) {
    case D_MC: return mc;
    case D_MR: return mr;
    case D_VC: return vc;
    case D_VR: return mr + c * mc;
    case D_STAR: return 0;
    case D_CIRC: return vc == root ? 0 : -1;
    case D_MD: orc_md_coords(r, c, vc, &diag, &pos); return diag == root ? pos : -1;
    default: return -1;
    }
}

/* ElementMatrix global<->local map (src/core/DistMatrix/ElementMatrix.cpp:604-675):
 * local (iLoc, jLoc) <-> global (colShift + iLoc*colStride, rowShift + jLoc*rowStride). */
static void block_map(int64_t H, int64_t W, int U, int V, int r, int c, int vc, int ca, int ra, int root,
                      int64_t* cs, int64_t* cstr, int64_t* rs, int64_t* rstr, int64_t* lh, int64_t* lw) {
    const int crank = orc_dist_rank(U, r, c, vc, root), rrank = orc_dist_rank(V, r, c, vc, root);
    *cstr = orc_dist_stride(U, r, c);
    *rstr = orc_dist_stride(V, r, c);
    if (crank < 0 || rrank < 0) { *lh = *lw = 0; *cs = *rs = 0; return; }
    *cs = orc_shift(crank, ca, *cstr);
    *rs = orc_shift(rrank, ra, *rstr);
    *lh = orc_length(H, *cs, *cstr);
    *lw = orc_length(W, *rs, *rstr);
}

void orc_local_block(const void* G, int64_t es, int64_t H, int64_t W, int64_t ldg, int U, int V, int r, int c,
                     int vc, int colAlign, int rowAlign, int root, void* out, int64_t ldo, int64_t* lh,
                     int64_t* lw) {
    int64_t cs, cstr, rs, rstr;
    block_map(H, W, U, V, r, c, vc, colAlign, rowAlign, root, &cs, &cstr, &rs, &rstr, lh, lw);
    const char* g = (const char*)G;
    char* o = (char*)out;
    for (int64_t j = 0; j < *lw; ++j)
        for (int64_t i = 0; i < *lh; ++i)
            memcpy(o + (i + j * ldo) * es, g + ((cs + i * cstr) + (rs + j * rstr) * ldg) * es, (size_t)es);
}

void orc_place_block(void* G, int64_t es, int64_t H, int64_t W, int64_t ldg, int U, int V, int r, int c, int vc,
                     int colAlign, int rowAlign, int root, const void* loc, int64_t ldl) {
    int64_t cs, cstr, rs, rstr, lh, lw;
    block_map(H, W, U, V, r, c, vc, colAlign, rowAlign, root, &cs, &cstr, &rs, &rstr, &lh, &lw);
    char* g = (char*)G;
    const char* l = (const char*)loc;
    for (int64_t j = 0; j < lw; ++j)
        for (int64_t i = 0; i < lh; ++i)
            memcpy(g + ((cs + i * cstr) + (rs + j * rstr) * ldg) * es, l + (i + j * ldl) * es, (size_t)es);
}

/* Counter-based hash (mirrors elemental_amd/csrc/kernels/elem.hpp bit for bit):
 * the reference's inputs come from a per-rank mt19937 (src/core/random.cpp:24-33,
 * src/matrices/random/independent/Uniform.cpp:53-59) and so depend on the grid;
 * parity runs need grid-independent inputs. */
uint64_t orc_splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
double orc_hash_unit(uint64_t seed, int64_t i, int64_t j) {
    uint64_t h = orc_splitmix64(seed ^ orc_splitmix64((uint64_t)i * 0xD1B54A32D192ED03ull + 0x1234567ull));
    h = orc_splitmix64(h ^ ((uint64_t)j * 0xA0761D6478BD642Full));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}
void orc_hash_fill_f64(int64_t H, int64_t W, uint64_t seed, double center, double radius, double* G, int64_t ldg) {
    for (int64_t j = 0; j < W; ++j)
        for (int64_t i = 0; i < H; ++i) G[i + j * ldg] = center + radius * (2.0 * orc_hash_unit(seed, i, j) - 1.0);
}
void orc_hash_fill_f32(int64_t H, int64_t W, uint64_t seed, double center, double radius, float* G, int64_t ldg) {
    for (int64_t j = 0; j < W; ++j)
        for (int64_t i = 0; i < H; ++i)
            G[i + j * ldg] = (float)(center + radius * (2.0 * orc_hash_unit(seed, i, j) - 1.0));
}

/* src/core/imports/blas/Gemm.hpp:47-260: scale C by beta (zero when beta == 0,
 * never reading C), then the naive loop nests: NN / NT accumulate column j as
 * axpys with gamma = alpha*B(l,j); TN / TT form dot products gamma =
 * sum_l A(l,i) op(B)(l,j) and add alpha*gamma. */
#define ORC_GEMM_BODY(T)                                                                        \
    int64_t i, j, l;                                                                            \
    if (beta == (T)0) {                                                                         \
        for (j = 0; j < n; ++j)                                                                 \
            for (i = 0; i < m; ++i) C[i + j * ldc] = (T)0;                                      \
    } else if (beta != (T)1) {                                                                  \
        for (j = 0; j < n; ++j)                                                                 \
            for (i = 0; i < m; ++i) C[i + j * ldc] *= beta;                                     \
    }                                                                                           \
    if (ta == 'N') {                                                                            \
        for (j = 0; j < n; ++j)                                                                 \
            for (l = 0; l < k; ++l) {                                                           \
                const T gamma = alpha * (tb == 'N' ? B[l + j * ldb] : B[j + l * ldb]);          \
                for (i = 0; i < m; ++i) C[i + j * ldc] += A[i + l * lda] * gamma;               \
            }                                                                                   \
    } else {                                                                                    \
        for (j = 0; j < n; ++j)                                                                 \
            for (i = 0; i < m; ++i) {                                                           \
                T gamma = (T)0;                                                                 \
                for (l = 0; l < k; ++l) gamma += A[l + i * lda] * (tb == 'N' ? B[l + j * ldb] : B[j + l * ldb]); \
                C[i + j * ldc] += alpha * gamma;                                                \
            }                                                                                   \
    }

void orc_gemm_f64(char ta, char tb, int64_t m, int64_t n, int64_t k, double alpha, const double* A, int64_t lda,
                  const double* B, int64_t ldb, double beta, double* C, int64_t ldc) {
    ORC_GEMM_BODY(double)
}
void orc_gemm_f32(char ta, char tb, int64_t m, int64_t n, int64_t k, float alpha, const float* A, int64_t lda,
                  const float* B, int64_t ldb, float beta, float* C, int64_t ldc) {
    ORC_GEMM_BODY(float)
}

/* SUMMA_NNC_impl (NN.hpp:341-385) on a simulated r x c grid, alignments 0:
 *   Scale(beta, C) (Gemm.cpp:282); for each panel k:
 *     A1[MC,*]   = A(:, k:k+nb)          -- RowAllGather over MR
 *     B1^T[MR,*] = (B(k:k+nb, :))^T      -- Transpose + RowAllGather over MC
 *     C_loc     += alpha A1_loc (B1^T_loc)^T   (LocalGemm NORMAL, TRANSPOSE, beta = 1)
 * Each rank's local blocks are extracted with the layout map above. */
void orc_summa_nnc_f64(int r, int c, int64_t m, int64_t n, int64_t k, int64_t nb, double alpha, const double* A,
                       int64_t lda, const double* B, int64_t ldb, double beta, double* C, int64_t ldc) {
    const int p = r * c;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i) C[i + j * ldc] = beta == 0.0 ? 0.0 : beta * C[i + j * ldc];
    /* global B^T (n x k) so the [MR,*] panel is a block of it */
    double* BT = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1) * (size_t)(k > 0 ? k : 1));
    for (int64_t l = 0; l < k; ++l)
        for (int64_t j = 0; j < n; ++j) BT[j + l * n] = B[l + j * ldb];
    for (int vc = 0; vc < p; ++vc) {
        int64_t lh, lw, lh2, lw2, lh3, lw3;
        const int64_t mloc = orc_max_length(m, r) + 1, nloc = orc_max_length(n, c) + 1;
        double* Cl = (double*)calloc((size_t)(mloc * nloc), sizeof(double));
        double* A1 = (double*)calloc((size_t)(mloc * (nb > 0 ? nb : 1)), sizeof(double));
        double* B1T = (double*)calloc((size_t)(nloc * (nb > 0 ? nb : 1)), sizeof(double));
        orc_local_block(C, 8, m, n, ldc, D_MC, D_MR, r, c, vc, 0, 0, 0, Cl, mloc, &lh, &lw);
        for (int64_t k0 = 0; k0 < k; k0 += nb) {
            const int64_t kb = (k - k0) < nb ? (k - k0) : nb;
            /* A1[MC,*] := A(:, k0:k0+kb) */
            orc_local_block(A + k0 * lda, 8, m, kb, lda, D_MC, D_STAR, r, c, vc, 0, 0, 0, A1, mloc, &lh2, &lw2);
            /* B1^T[MR,*] := B(k0:k0+kb, :)^T */
            orc_local_block(BT + k0 * n, 8, n, kb, n, D_MR, D_STAR, r, c, vc, 0, 0, 0, B1T, nloc, &lh3, &lw3);
            orc_gemm_f64('N', 'T', lh, lw, kb, alpha, A1, mloc, B1T, nloc, 1.0, Cl, mloc);
        }
        orc_place_block(C, 8, m, n, ldc, D_MC, D_MR, r, c, vc, 0, 0, 0, Cl, mloc);
        free(Cl);
        free(A1);
        free(B1T);
    }
    free(BT);
}

double orc_fro(int64_t m, int64_t n, const double* X, int64_t ldx) {
    long double s = 0.0L;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i) s += (long double)X[i + j * ldx] * X[i + j * ldx];
    return (double)sqrtl(s);
}
