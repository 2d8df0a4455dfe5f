// 16-bit local GEMM (f16 = the reference's gpu_half_type / rocblas_half path,
// bf16 = new) on gfx950 v_mfma_f32_16x16x32_{f16,bf16}, f32 accumulation.
//
// Replaces rocblas_hgemm (src/hydrogen/device/rocBLAS_API.cpp:151-170 via
// include/hydrogen/blas/GPU_BLAS_impl.hpp:397-423).  Note the reference's CPU
// half path accumulates in half (src/core/imports/blas/Gemm.hpp:47-260); this
// kernel accumulates in f32 and rounds once (better, within the per-type tolerance).
//
// Tile: 128x128 per 256-thread workgroup, 4 waves of 64x64 = 4x4 MFMA tiles,
// BK = 32 per slab (one MFMA k-step).  LDS images are k-contiguous rows
// ([i][k] for A, [j][k] for B, pitch 40 elements = 80 B) so each lane's
// 8-element operand fragment is one 16-byte ds_read.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.hpp"
#include "elem.hpp"

namespace elx {
namespace kern {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 32, NTHR = 256, KP = 40, GROUP_M = 8;
constexpr int EPT = BM * BK / NTHR;  // 16

struct HParams {
    i64 m, n, k;
    float alpha, beta;
    const uint16_t* A; i64 lda;
    const uint16_t* B; i64 ldb;
    uint16_t* C; i64 ldc;
    int tiles_m, tiles_n;
};

__device__ __forceinline__ void tile_of(int bid, int nwg, int tiles_m, int tiles_n, int& tm, int& tn) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int per_group = GROUP_M * tiles_n;
    const int group = wg / per_group;
    const int first_m = group * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    const int inner = wg - group * per_group;
    tm = first_m + inner % gsz;
    tn = inner / gsz;
}

// Stage op(X) (rows x BK slab, row index r along the output dim, k along the
// slab) into registers. KCONTIG: X(r,k) = X[k + r*ld]; else X(r,k) = X[r + k*ld].
template <bool KCONTIG>
__device__ __forceinline__ void load_slab(const uint16_t* X, i64 ld, i64 rows, i64 kdim, i64 r0, i64 k0, int tid,
                                          uint16_t (&v)[EPT]) {
    if (KCONTIG) {
        const int kk = tid & (BK - 1), r = tid >> 5;  // 8 rows per pass
        const bool kv = (k0 + kk) < kdim;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const i64 rr = r0 + r + 8 * e;
            v[e] = (kv && rr < rows) ? X[(k0 + kk) + rr * ld] : (uint16_t)0;
        }
    } else {
        const int r = tid & (BM - 1), kk = tid >> 7;  // 2 k per pass
        const bool rv = (r0 + r) < rows;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const i64 k = k0 + kk + 2 * e;
            v[e] = (rv && k < kdim) ? X[(r0 + r) + k * ld] : (uint16_t)0;
        }
    }
}
template <bool KCONTIG>
__device__ __forceinline__ void store_slab(uint16_t (*S)[KP], int tid, const uint16_t (&v)[EPT]) {
    if (KCONTIG) {
        const int kk = tid & (BK - 1), r = tid >> 5;
#pragma unroll
        for (int e = 0; e < EPT; ++e) S[r + 8 * e][kk] = v[e];
    } else {
        const int r = tid & (BM - 1), kk = tid >> 7;
#pragma unroll
        for (int e = 0; e < EPT; ++e) S[r][kk + 2 * e] = v[e];
    }
}

template <bool BF16>
__device__ __forceinline__ f32x4 mfma16(const uint4& a, const uint4& b, f32x4 c) {
    if constexpr (BF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

template <bool BF16, bool TA, bool TB>
__global__ __launch_bounds__(NTHR, 2) void gemm_half_kernel(HParams p) {
    using E = typename std::conditional<BF16, Elem<bf16_t>, Elem<f16_t>>::type;
    __shared__ __attribute__((aligned(16))) uint16_t As[2][BM][KP];
    __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN][KP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1, g = lane >> 4, c = lane & 15;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;

    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    // op(A)(i,k): TA -> A[k + i*lda] (k contiguous); op(B)(k,j): !TB -> B[k + j*ldb] (k contiguous)
    const int nk = (int)((p.k + BK - 1) / BK);
    uint16_t ra[EPT], rb[EPT];
    if (nk > 0) {
        load_slab<TA>(p.A, p.lda, p.m, p.k, m0, 0, tid, ra);
        load_slab<!TB>(p.B, p.ldb, p.n, p.k, n0, 0, tid, rb);
        store_slab<TA>(As[0], tid, ra);
        store_slab<!TB>(Bs[0], tid, rb);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const bool more = kt + 1 < nk;
        if (more) {
            load_slab<TA>(p.A, p.lda, p.m, p.k, m0, (i64)(kt + 1) * BK, tid, ra);
            load_slab<!TB>(p.B, p.ldb, p.n, p.k, n0, (i64)(kt + 1) * BK, tid, rb);
        }
        uint4 a[4], b[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) a[mi] = *reinterpret_cast<const uint4*>(&As[cur][wr * 64 + mi * 16 + c][8 * g]);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b[ni] = *reinterpret_cast<const uint4*>(&Bs[cur][wc * 64 + ni * 16 + c][8 * g]);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16<BF16>(a[mi], b[ni], acc[mi][ni]);
        if (more) {
            store_slab<TA>(As[cur ^ 1], tid, ra);
            store_slab<!TB>(Bs[cur ^ 1], tid, rb);
        }
        __syncthreads();
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const i64 j = n0 + wc * 64 + ni * 16 + c;
            if (j >= p.n) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 i = m0 + wr * 64 + mi * 16 + 4 * g + r;  // C/D map: row = 4*(lane>>4)+reg
                if (i < p.m) {
                    uint16_t* o = p.C + i + j * p.ldc;
                    float v = p.alpha * acc[mi][ni][r];
                    if (p.beta != 0.f) v += p.beta * E::load(*o);
                    *o = E::store(v);
                }
            }
        }
}

template <bool BF16, bool TA, bool TB>
hipError_t launch(const HParams& p, hipStream_t s) {
    hipLaunchKernelGGL((gemm_half_kernel<BF16, TA, TB>), dim3(p.tiles_m * p.tiles_n), dim3(NTHR), 0, s, p);
    return hipGetLastError();
}

}  // namespace

hipError_t gemm_mfma_h_simple(bool is_bf16, bool ta, bool tb, i64 m, i64 n, i64 k, float alpha, const uint16_t* A,
                       i64 lda, const uint16_t* B, i64 ldb, float beta, uint16_t* C, i64 ldc, hipStream_t s) {
    HParams p{m, n, k, alpha, beta, A, lda, B, ldb, C, ldc, (int)((m + BM - 1) / BM), (int)((n + BN - 1) / BN)};
    if (is_bf16) {
        if (ta) return tb ? launch<true, true, true>(p, s) : launch<true, true, false>(p, s);
        return tb ? launch<true, false, true>(p, s) : launch<true, false, false>(p, s);
    }
    if (ta) return tb ? launch<false, true, true>(p, s) : launch<false, true, false>(p, s);
    return tb ? launch<false, false, true>(p, s) : launch<false, false, false>(p, s);
}

}  // namespace kern
}  // namespace elx
