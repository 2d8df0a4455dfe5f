// Local panel update for gfx950: C := alpha op(A) op(B) + beta C, column-major.
//
// Replaces the reference's vendor GEMM call on the hot path
// (hydrogen::gpu_blas::Gemm -> rocblas_dgemm/sgemm, include/hydrogen/blas/GPU_BLAS_impl.hpp:397-423,
//  src/hydrogen/device/rocBLAS_API.cpp:151-170), which SUMMA calls once per panel
// (src/blas_like/level3/Gemm.cpp:163-186 LocalGemm -> Gemm_impl<GPU>).
//
// Design (MI355X-first):
//  * 128x128 output tile per 256-thread workgroup, 4 waves of 64x64, each wave a
//    4x4 grid of 16x16 MFMA accumulators (v_mfma_f64_16x16x4_f64 /
//    v_mfma_f32_16x16x4_f32: one operand element per lane, so every orientation
//    shares one LDS image [k][i] / [k][j]).
//  * BK = 16 k-slab, double-buffered in LDS; the next slab's global loads are
//    issued into registers before the current slab's MFMAs and written to the
//    other LDS buffer after them (one barrier per slab).
//  * LDS row pitch 145 elements: conflict-free for the contiguous (N) staging
//    writes, <=2-way for the transposed (T) staging writes and the MFMA reads.
//  * XCD-aware, bijective blockIdx remap + grouped tile order so the 32 CUs of
//    one XCD work on a compact patch of C and share A/B panels in their L2.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace elx {
namespace kern {

using i64 = int64_t;

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Mfma;
template <> struct Mfma<double> {
    using acc_t = f64x4;
    static __device__ __forceinline__ acc_t op(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // C/D map of v_mfma_f64_16x16x4_f64: row = (lane>>4) + 4*reg, col = lane&15
    static __device__ __forceinline__ int row(int g, int r) { return g + 4 * r; }
};
template <> struct Mfma<float> {
    using acc_t = f32x4;
    static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // C/D map of v_mfma_f32_16x16x4_f32: row = 4*(lane>>4) + reg, col = lane&15
    static __device__ __forceinline__ int row(int g, int r) { return 4 * g + r; }
};

template <typename T>
struct GemmParams {
    i64 m, n, k;
    T alpha, beta;
    const T* A; i64 lda;
    const T* B; i64 ldb;
    T* C; i64 ldc;
    int tiles_m, tiles_n;
};

constexpr int BM = 128, BN = 128, BK = 16, NTHR = 256, LDP = 145, GROUP_M = 8;
constexpr int EPT = BM * BK / NTHR;  // elements per thread per operand per slab = 8

// Map the flat workgroup id to a (tile_m, tile_n) pair.  Workgroups are dealt
// round-robin over the 8 XCDs (b and b+8 share one); remap so each XCD owns a
// contiguous run of the grouped order (bijective for any grid size).
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

// One k-slab of op(A) (BM x BK) into registers.  !TA: A(i,k)=A[i + k*lda]
// (i contiguous: lane -> i); TA: op(A)(i,k)=A[k + i*lda] (k contiguous: lane -> k).
template <typename T, bool TA>
__device__ __forceinline__ void load_a(const GemmParams<T>& p, i64 m0, i64 k0, int tid, T (&r)[EPT]) {
    if (!TA) {
        const int i = tid & (BM - 1), kk = tid >> 7;
        const bool iv = (m0 + i) < p.m;
        const T* base = p.A + (m0 + i) + (k0 + kk) * p.lda;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const bool v = iv && (k0 + kk + 2 * e) < p.k;
            r[e] = v ? base[(i64)(2 * e) * p.lda] : T(0);
        }
    } else {
        const int kk = tid & (BK - 1), i = tid >> 4;
        const bool kv = (k0 + kk) < p.k;
        const T* base = p.A + (k0 + kk) + (m0 + i) * p.lda;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const bool v = kv && (m0 + i + 16 * e) < p.m;
            r[e] = v ? base[(i64)(16 * e) * p.lda] : T(0);
        }
    }
}
template <typename T, bool TA>
__device__ __forceinline__ void store_a(T (*As)[LDP], int tid, const T (&r)[EPT]) {
    if (!TA) {
        const int i = tid & (BM - 1), kk = tid >> 7;
#pragma unroll
        for (int e = 0; e < EPT; ++e) As[kk + 2 * e][i] = r[e];
    } else {
        const int kk = tid & (BK - 1), i = tid >> 4;
#pragma unroll
        for (int e = 0; e < EPT; ++e) As[kk][i + 16 * e] = r[e];
    }
}
// One k-slab of op(B) (BK x BN).  !TB: B(k,j)=B[k + j*ldb] (k contiguous);
// TB: op(B)(k,j)=B[j + k*ldb] (j contiguous).
template <typename T, bool TB>
__device__ __forceinline__ void load_b(const GemmParams<T>& p, i64 n0, i64 k0, int tid, T (&r)[EPT]) {
    if (TB) {
        const int j = tid & (BN - 1), kk = tid >> 7;
        const bool jv = (n0 + j) < p.n;
        const T* base = p.B + (n0 + j) + (k0 + kk) * p.ldb;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const bool v = jv && (k0 + kk + 2 * e) < p.k;
            r[e] = v ? base[(i64)(2 * e) * p.ldb] : T(0);
        }
    } else {
        const int kk = tid & (BK - 1), j = tid >> 4;
        const bool kv = (k0 + kk) < p.k;
        const T* base = p.B + (k0 + kk) + (n0 + j) * p.ldb;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const bool v = kv && (n0 + j + 16 * e) < p.n;
            r[e] = v ? base[(i64)(16 * e) * p.ldb] : T(0);
        }
    }
}
template <typename T, bool TB>
__device__ __forceinline__ void store_b(T (*Bs)[LDP], int tid, const T (&r)[EPT]) {
    if (TB) {
        const int j = tid & (BN - 1), kk = tid >> 7;
#pragma unroll
        for (int e = 0; e < EPT; ++e) Bs[kk + 2 * e][j] = r[e];
    } else {
        const int kk = tid & (BK - 1), j = tid >> 4;
#pragma unroll
        for (int e = 0; e < EPT; ++e) Bs[kk][j + 16 * e] = r[e];
    }
}

template <typename T, bool TA, bool TB, bool BETA0>
__global__ __launch_bounds__(NTHR, 2) void gemm_tile_kernel(GemmParams<T> p) {
    using M = Mfma<T>;
    using acc_t = typename M::acc_t;
    __shared__ T As[2][BK][LDP];
    __shared__ T Bs[2][BK][LDP];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int g = lane >> 4, c = lane & 15;

    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;

    acc_t acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = acc_t{0, 0, 0, 0};

    const int nk = (int)((p.k + BK - 1) / BK);
    T ra[EPT], rb[EPT];
    if (nk > 0) {
        load_a<T, TA>(p, m0, 0, tid, ra);
        load_b<T, TB>(p, n0, 0, tid, rb);
        store_a<T, TA>(As[0], tid, ra);
        store_b<T, TB>(Bs[0], tid, rb);
    }
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const bool more = (kt + 1) < nk;
        if (more) {  // issue next slab's loads early; they land during the MFMAs
            load_a<T, TA>(p, m0, (i64)(kt + 1) * BK, tid, ra);
            load_b<T, TB>(p, n0, (i64)(kt + 1) * BK, tid, rb);
        }
#pragma unroll
        for (int s = 0; s < BK / 4; ++s) {
            T a[4], b[4];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) a[mi] = As[cur][4 * s + g][wr * 64 + mi * 16 + c];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) b[ni] = Bs[cur][4 * s + g][wc * 64 + ni * 16 + c];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = M::op(a[mi], b[ni], acc[mi][ni]);
        }
        if (more) {
            store_a<T, TA>(As[cur ^ 1], tid, ra);
            store_b<T, TB>(Bs[cur ^ 1], tid, rb);
        }
        __syncthreads();
    }

    // Epilogue: C = alpha*acc + beta*C (beta == 0 never reads C: BLAS semantics).
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const i64 j = n0 + wc * 64 + ni * 16 + c;
            if (j >= p.n) continue;
            T* ccol = p.C + j * p.ldc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 i = m0 + wr * 64 + mi * 16 + M::row(g, r);
                if (i < p.m) {
                    const T v = p.alpha * acc[mi][ni][r];
                    ccol[i] = BETA0 ? v : v + p.beta * ccol[i];
                }
            }
        }
    }
}

template <typename T, bool TA, bool TB>
static hipError_t launch_tn(const GemmParams<T>& p, hipStream_t s) {
    const int nwg = p.tiles_m * p.tiles_n;
    if (p.beta == T(0))
        hipLaunchKernelGGL((gemm_tile_kernel<T, TA, TB, true>), dim3(nwg), dim3(NTHR), 0, s, p);
    else
        hipLaunchKernelGGL((gemm_tile_kernel<T, TA, TB, false>), dim3(nwg), dim3(NTHR), 0, s, p);
    return hipGetLastError();
}

template <typename T>
hipError_t gemm_mfma(bool ta, bool tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda,
                     const T* B, i64 ldb, T beta, T* C, i64 ldc, hipStream_t s) {
    GemmParams<T> p{m, n, k, alpha, beta, A, lda, B, ldb, C, ldc,
                    (int)((m + BM - 1) / BM), (int)((n + BN - 1) / BN)};
    if (ta) return tb ? launch_tn<T, true, true>(p, s) : launch_tn<T, true, false>(p, s);
    return tb ? launch_tn<T, false, true>(p, s) : launch_tn<T, false, false>(p, s);
}

template hipError_t gemm_mfma<double>(bool, bool, i64, i64, i64, double, const double*, i64,
                                      const double*, i64, double, double*, i64, hipStream_t);
template hipError_t gemm_mfma<float>(bool, bool, i64, i64, i64, float, const float*, i64,
                                     const float*, i64, float, float*, i64, hipStream_t);

}  // namespace kern
}  // namespace elx
