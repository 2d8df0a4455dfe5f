// Local panel update for gfx950: C := alpha op(A) op(B) + beta C, column-major.
//
// Replaces the reference's vendor GEMM call on the hot path
// (hydrogen::gpu_blas::Gemm -> rocblas_dgemm/sgemm, include/hydrogen/blas/GPU_BLAS_impl.hpp:397-423,
//  src/hydrogen/device/rocBLAS_API.cpp:151-170), which SUMMA calls once per panel
// (src/blas_like/level3/Gemm.cpp:163-186 LocalGemm -> Gemm_impl<GPU>).
//
// Design (MI355X-first):
//  * One workgroup per BM x BN output tile, WAVES_M x WAVES_N waves; each wave
//    owns a grid of 16x16 MFMA accumulators (v_mfma_f64_16x16x4_f64 /
//    v_mfma_f32_16x16x4_f32: one operand element per lane, so every
//    orientation shares one LDS image [k][r]).  Shipped shapes (measured,
//    profiles/r01_tile_variants.log): f64 128x128 with 8 waves of 32x64
//    (2 workgroups per CU = 4 waves per SIMD, enough to hide the LDS->MFMA
//    latency of the 64-cycle f64 MFMA); f32 256x128 with 8 waves of 64x64
//    (1 workgroup per CU, fewer LDS reads and HBM bytes per MFMA).
//  * BK = 16 k-slab, double-buffered in LDS; the next slab's global loads are
//    issued into registers before the current slab's MFMAs and written to the
//    other LDS buffer after them (one barrier per slab).
//  * Loads never branch: indices are clamped into the matrix (always a valid
//    address) and out-of-range elements zeroed by a select at the LDS store,
//    so the wait for a slab's loads sits after the MFMAs.  With 16-B aligned
//    operands each lane moves a 16-B pair along the unit-stride dimension, and
//    offsets inside a slab are 32-bit off a per-slab uniform base.
//  * LDS pitch: ROWS+16 when r is HBM-contiguous (MFMA reads conflict-free),
//    ROWS+17 otherwise (the transposing staging writes conflict-free).
//  * XCD-aware, bijective blockIdx remap + grouped tile order so the 32 CUs of
//    one XCD work on a compact patch of C and share A/B panels in their L2.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <string>
#include "kernels.hpp"

namespace elx {
namespace kern {

using i64 = int64_t;

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <typename T> struct Mfma;
template <> struct Mfma<double> {
    using acc_t = f64x4;
    using pair_t = f64x2;
    static __device__ __forceinline__ acc_t op(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // C/D map of v_mfma_f64_16x16x4_f64: row = (lane>>4) + 4*reg, col = lane&15
    static __device__ __forceinline__ int row(int g, int r) { return g + 4 * r; }
};
template <> struct Mfma<float> {
    using acc_t = f32x4;
    using pair_t = f32x2;
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
    // split-k (gridDim.y = number of k chunks > 1): chunk z covers k in
    // [z*kchunk, min(k, (z+1)*kchunk)) and writes its raw partial product to
    // C + z*zstride (ldc = m, alpha = 1, beta = 0); splitk_reduce finishes.
    i64 kchunk, zstride;
};

constexpr int BK = 16, GROUP_M = 8;

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

// LDS image [k][r] of one operand slab (ROWS output rows x BK).
template <typename T, int ROWS, bool RCONTIG>
struct Img {
    static constexpr int P = RCONTIG ? ROWS + 16 : ROWS + 17;
    T d[BK][P];
    __device__ __forceinline__ T& at(int r, int k) { return d[k][r]; }
};

// Operand slab loader.  The operand is viewed as rows r (the output dimension:
// i for A, j for B) by k.  RCONTIG: X(r,k) = X[r + k*ld]; else X(r,k) = X[k + r*ld].
// Thread `tid` (of NTHR) owns element/pair p = tid + NTHR*q of the slab.
template <typename T, int ROWS, bool RCONTIG, bool VEC, int NTHR>
struct Slab {
    using pair_t = typename Mfma<T>::pair_t;
    static constexpr int STEP = VEC ? 2 : 1;
    static constexpr int EPT = ROWS * BK / NTHR;  // elements per thread
    static constexpr int NQ = EPT / STEP;          // loads per thread
    static __device__ __forceinline__ int r_of(int tid, int q) {
        const int p = tid + NTHR * q;
        if (RCONTIG) return VEC ? 2 * (p % (ROWS / 2)) : p % ROWS;
        return VEC ? p / (BK / 2) : p / BK;
    }
    static __device__ __forceinline__ int k_of(int tid, int q) {
        const int p = tid + NTHR * q;
        if (RCONTIG) return VEC ? p / (ROWS / 2) : p / ROWS;
        return VEC ? 2 * (p % (BK / 2)) : p % BK;
    }

    // Generic path (any alignment / size): 64-bit clamped addresses.
    static __device__ __forceinline__ void load_edge(const T* X, i64 ld, i64 rows, i64 kdim, i64 r0, i64 k0,
                                                     int tid, T (&v)[EPT], uint32_t& ok) {
        ok = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const i64 r = r0 + r_of(tid, q), k = k0 + k_of(tid, q);
            ok |= (uint32_t)((r < rows) & (k < kdim)) << q;
            if (VEC) {  // pairs never straddle the edge: even extent along the vector dimension
                const i64 rc = r < rows ? r : rows - (RCONTIG ? 2 : 1);
                const i64 kc = k < kdim ? k : kdim - (RCONTIG ? 1 : 2);
                const pair_t x = *reinterpret_cast<const pair_t*>(RCONTIG ? X + rc + kc * ld : X + kc + rc * ld);
                v[2 * q] = x[0];
                v[2 * q + 1] = x[1];
            } else {
                const i64 rc = r < rows ? r : rows - 1, kc = k < kdim ? k : kdim - 1;
                v[q] = RCONTIG ? X[rc + kc * ld] : X[kc + rc * ld];
            }
        }
    }

    // 32-bit path (VEC, ld < 2^24): every load is one 32-bit offset off the
    // slab's uniform base; rows are clamped against the tile's uniform bound.
    struct Off32 {
        int rmax;  // last valid local row of this tile (uniform)
    };
    static __device__ __forceinline__ Off32 off32_init(int, i64 r0, i64 rows, uint32_t) {
        const i64 rm = rows - r0 - (RCONTIG && VEC ? 2 : 1);
        return Off32{rm > (1 << 30) ? (1 << 30) : (int)rm};
    }
    // sbase = X + slab origin (uniform); kleft = k extent left from the slab origin
    static __device__ __forceinline__ void load32(const T* sbase, const Off32& st, int tid, uint32_t ld, int kleft,
                                                  T (&v)[EPT], uint32_t& ok) {
        ok = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int r = r_of(tid, q), kl = k_of(tid, q);
            const int rc = min(r, st.rmax);
            const int kc = min(kl, kleft - (RCONTIG ? 1 : 2));
            ok |= (uint32_t)((r <= st.rmax) & (kl < kleft)) << q;
            const uint32_t o = RCONTIG ? (uint32_t)rc + (uint32_t)kc * ld : (uint32_t)kc + (uint32_t)rc * ld;
            const pair_t x = *reinterpret_cast<const pair_t*>(sbase + o);
            v[2 * q] = x[0];
            v[2 * q + 1] = x[1];
        }
    }

    static __device__ __forceinline__ T sel(uint32_t ok, int q, T x) { return (ok >> q) & 1 ? x : T(0); }
    static __device__ __forceinline__ void store(Img<T, ROWS, RCONTIG>& S, int tid, const T (&v)[EPT], uint32_t ok) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int r = r_of(tid, q), k = k_of(tid, q);
            if (VEC) {
                S.at(r, k) = sel(ok, q, v[2 * q]);
                if (RCONTIG) S.at(r + 1, k) = sel(ok, q, v[2 * q + 1]);
                else S.at(r, k + 1) = sel(ok, q, v[2 * q + 1]);
            } else {
                S.at(r, k) = sel(ok, q, v[q]);
            }
        }
    }
};

template <int BM_, int BN_, int WAVES_M_, int WAVES_N_, int MINB_>
struct TileCfg {
    static constexpr int BM = BM_, BN = BN_, MINB = MINB_;
    static constexpr int WAVES_M = WAVES_M_, WAVES_N = WAVES_N_, NTHR = 64 * WAVES_M_ * WAVES_N_;
    static constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;  // wave tile
    static constexpr int WM = WTM / 16, WN = WTN / 16;            // MFMA tiles per wave
    static constexpr int WAVES_PER_EU = MINB_ * WAVES_M_ * WAVES_N_ / 4;
};
using Tile128 = TileCfg<128, 128, 2, 2, 2>;   // 4 waves of 64x64, 2 per SIMD
using Tile128w8 = TileCfg<128, 128, 4, 2, 2>; // 8 waves of 32x64, 4 per SIMD
using Tile256w8 = TileCfg<256, 128, 4, 2, 1>;  // 8 waves of 64x64, 2 per SIMD, 1 block/CU

template <typename T, typename CFG, bool TA, bool TB, bool BETA0, bool VEC, bool OFF32>
__global__ __launch_bounds__(CFG::NTHR, CFG::WAVES_PER_EU) void gemm_tile_kernel(GemmParams<T> p) {
    using M = Mfma<T>;
    using acc_t = typename M::acc_t;
    constexpr int BM = CFG::BM, BN = CFG::BN, WM = CFG::WM, WN = CFG::WN;
    constexpr int WTM = CFG::WTM, WTN = CFG::WTN;
    constexpr bool RA = !TA, RB = TB;  // op(A)(i,k): !TA -> A[i + k*lda]; op(B)(k,j): TB -> B[j + k*ldb]
    using SA = Slab<T, BM, RA, VEC, CFG::NTHR>;
    using SB = Slab<T, BN, RB, VEC, CFG::NTHR>;
    __shared__ __attribute__((aligned(16))) Img<T, BM, RA> As[2];
    __shared__ __attribute__((aligned(16))) Img<T, BN, RB> Bs[2];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wr = wave / CFG::WAVES_N, wc = wave % CFG::WAVES_N;
    const int g = lane >> 4, c = lane & 15;

    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;
    {  // this workgroup's k chunk (the whole k unless split)
        const i64 kz0 = (i64)blockIdx.y * p.kchunk;
        p.k = min(p.kchunk, p.k - kz0);
        p.A += RA ? kz0 * p.lda : kz0;
        p.B += RB ? kz0 * p.ldb : kz0;
        p.C += (i64)blockIdx.y * p.zstride;
    }

    acc_t acc[WM][WN];
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) acc[a][b] = acc_t{0, 0, 0, 0};

    const int nk = (int)((p.k + BK - 1) / BK);
    typename SA::Off32 sta{};
    typename SB::Off32 stb{};
    if (OFF32) {
        sta = SA::off32_init(tid, m0, p.m, (uint32_t)p.lda);
        stb = SB::off32_init(tid, n0, p.n, (uint32_t)p.ldb);
    }
    T ra[SA::EPT], rb[SB::EPT];
    uint32_t oka = 0, okb = 0;
    auto load_slab = [&](int kt) {
        const i64 k0 = (i64)kt * BK;
        if (OFF32) {
            const i64 kl = p.k - k0;
            const int kleft = kl > (1 << 20) ? (1 << 20) : (int)kl;
            SA::load32(p.A + (RA ? m0 + k0 * p.lda : m0 * p.lda + k0), sta, tid, (uint32_t)p.lda, kleft, ra, oka);
            SB::load32(p.B + (RB ? n0 + k0 * p.ldb : n0 * p.ldb + k0), stb, tid, (uint32_t)p.ldb, kleft, rb, okb);
        } else {
            SA::load_edge(p.A, p.lda, p.m, p.k, m0, k0, tid, ra, oka);
            SB::load_edge(p.B, p.ldb, p.n, p.k, n0, k0, tid, rb, okb);
        }
    };
    if (nk > 0) {
        load_slab(0);
        SA::store(As[0], tid, ra, oka);
        SB::store(Bs[0], tid, rb, okb);
    }
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const bool more = (kt + 1) < nk;
        if (more) load_slab(kt + 1);  // issued early; lands during the MFMAs
#pragma unroll
        for (int s = 0; s < BK / 4; ++s) {
            T a[WM], b[WN];
#pragma unroll
            for (int mi = 0; mi < WM; ++mi) a[mi] = As[cur].at(wr * WTM + mi * 16 + c, 4 * s + g);
#pragma unroll
            for (int ni = 0; ni < WN; ++ni) b[ni] = Bs[cur].at(wc * WTN + ni * 16 + c, 4 * s + g);
#pragma unroll
            for (int mi = 0; mi < WM; ++mi)
#pragma unroll
                for (int ni = 0; ni < WN; ++ni) acc[mi][ni] = M::op(a[mi], b[ni], acc[mi][ni]);
        }
        if (more) {
            SA::store(As[cur ^ 1], tid, ra, oka);
            SB::store(Bs[cur ^ 1], tid, rb, okb);
        }
        __syncthreads();
    }

    // Epilogue: C = alpha*acc + beta*C (beta == 0 never reads C: BLAS semantics).
    // Interior tiles issue a row of C loads before their first use (no
    // per-element branch), so the reads overlap instead of serialising.
    const i64 ib = m0 + wr * WTM, jb = n0 + wc * WTN;
    if (ib + WTM <= p.m && jb + WTN <= p.n) {
#pragma unroll
        for (int mi = 0; mi < WM; ++mi) {
            T cv[WN][4];
            if (!BETA0) {
#pragma unroll
                for (int ni = 0; ni < WN; ++ni)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        cv[ni][r] = p.C[(ib + mi * 16 + M::row(g, r)) + (jb + ni * 16 + c) * p.ldc];
            }
#pragma unroll
            for (int ni = 0; ni < WN; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    T& o = p.C[(ib + mi * 16 + M::row(g, r)) + (jb + ni * 16 + c) * p.ldc];
                    o = BETA0 ? p.alpha * acc[mi][ni][r] : p.alpha * acc[mi][ni][r] + p.beta * cv[ni][r];
                }
        }
        return;
    }
#pragma unroll
    for (int mi = 0; mi < WM; ++mi) {
#pragma unroll
        for (int ni = 0; ni < WN; ++ni) {
            const i64 j = jb + ni * 16 + c;
            if (j >= p.n) continue;
            T* ccol = p.C + j * p.ldc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 i = ib + mi * 16 + M::row(g, r);
                if (i < p.m) {
                    const T v = p.alpha * acc[mi][ni][r];
                    ccol[i] = BETA0 ? v : v + p.beta * ccol[i];
                }
            }
        }
    }
}

template <typename T, typename CFG, bool TA, bool TB, bool VEC, bool OFF32>
static hipError_t launch_cfg(GemmParams<T> p, hipStream_t s) {
    p.tiles_m = (int)((p.m + CFG::BM - 1) / CFG::BM);
    p.tiles_n = (int)((p.n + CFG::BN - 1) / CFG::BN);
    const int nwg = p.tiles_m * p.tiles_n;
    const int nz = (int)((p.k + p.kchunk - 1) / p.kchunk);
    if (p.beta == T(0))
        hipLaunchKernelGGL((gemm_tile_kernel<T, CFG, TA, TB, true, VEC, OFF32>), dim3(nwg, nz), dim3(CFG::NTHR), 0, s, p);
    else
        hipLaunchKernelGGL((gemm_tile_kernel<T, CFG, TA, TB, false, VEC, OFF32>), dim3(nwg, nz), dim3(CFG::NTHR), 0, s, p);
    return hipGetLastError();
}

// C = alpha * sum_z W[z] + beta * C, z in order (deterministic); W[z] is m x n with ld m.
template <typename T, bool BETA0>
__global__ __launch_bounds__(256) void splitk_reduce(i64 m, i64 n, int nz, T alpha, const T* __restrict__ W, T beta,
                                                     T* C, i64 ldc) {
    const i64 mn = m * n;
    for (i64 e = (i64)blockIdx.x * 256 + threadIdx.x; e < mn; e += (i64)gridDim.x * 256) {
        T acc = W[e];
        for (int z = 1; z < nz; ++z) acc += W[e + z * mn];
        const i64 i = e % m, j = e / m;
        T& o = C[i + j * ldc];
        o = BETA0 ? alpha * acc : alpha * acc + beta * o;
    }
}

template <typename T>
static hipError_t launch_reduce(i64 m, i64 n, int nz, T alpha, const T* W, T beta, T* C, i64 ldc, hipStream_t s) {
    const i64 mn = m * n;
    const int grid = (int)std::min<i64>((mn + 255) / 256, 256 * 16);
    if (beta == T(0))
        hipLaunchKernelGGL((splitk_reduce<T, true>), dim3(grid), dim3(256), 0, s, m, n, nz, alpha, W, beta, C, ldc);
    else
        hipLaunchKernelGGL((splitk_reduce<T, false>), dim3(grid), dim3(256), 0, s, m, n, nz, alpha, W, beta, C, ldc);
    return hipGetLastError();
}

// Split k when the output tiles alone cannot fill the chip (the Dot variant's
// 2000 x 2000 x 524288 blocks, SUMMA_*Dot): aim for two rounds of resident
// workgroups with chunks of >= 2048.  Returns the chunk count (1 = no split).
template <typename CFG>
static int split_count(i64 m, i64 n, i64 k) {
    const i64 nwg = ((m + CFG::BM - 1) / CFG::BM) * ((n + CFG::BN - 1) / CFG::BN);
    const i64 slots = 256 * CFG::MINB;  // resident workgroups on 256 CUs
    if (nwg >= slots || k < 2 * 2048) return 1;
    i64 z = (2 * slots + nwg - 1) / nwg;
    z = std::min<i64>(z, k / 2048);
    z = std::min<i64>(z, 16);
    return (int)std::max<i64>(z, 1);
}

template <typename T, typename CFG, bool TA, bool TB, bool VEC, bool OFF32>
static hipError_t launch_split(GemmParams<T> p, hipStream_t s) {
    const int z = split_count<CFG>(p.m, p.n, p.k);
    p.kchunk = std::max<i64>(p.k, 1);
    p.zstride = 0;
    if (z <= 1) return launch_cfg<T, CFG, TA, TB, VEC, OFF32>(p, s);
    const i64 kchunk = ((p.k + z - 1) / z + BK - 1) / BK * BK;
    const int nz = (int)((p.k + kchunk - 1) / kchunk);
    T* W = nullptr;
    const size_t bytes = sizeof(T) * (size_t)p.m * (size_t)p.n * (size_t)nz;
    hipError_t e = workspace_alloc(reinterpret_cast<void**>(&W), bytes, s);
    if (e != hipSuccess) return e;
    GemmParams<T> q = p;
    q.alpha = T(1);
    q.beta = T(0);
    q.C = W;
    q.ldc = p.m;
    q.kchunk = kchunk;
    q.zstride = p.m * p.n;
    e = launch_cfg<T, CFG, TA, TB, VEC, OFF32>(q, s);
    if (e == hipSuccess) e = launch_reduce(p.m, p.n, nz, p.alpha, W, p.beta, p.C, p.ldc, s);
    const hipError_t f = workspace_free(W, s);
    return e != hipSuccess ? e : f;
}

// Tile configuration of the register-staged kernel (measured on MI355X,
// 16384^3 NN, profiles/r01_tile_variants.log): f64 128x128 with 8 waves of
// 32x64 (66.1 TF vs 62.9 with 4 waves, 62.8 at 256x128); f32 256x128 with 8
// waves of 64x64, one block per CU (127.5 TF vs 124.5 at 128x128).  The
// LDS-DMA kernels take every shape their plan accepts; this kernel serves the
// rest (edges, k tails, unaligned operands).
template <typename T, bool TA, bool TB>
static hipError_t launch_tn(const GemmParams<T>& p, hipStream_t s) {
    // 16-byte loads need 16-byte aligned bases, even leading dimensions and an
    // even extent along each operand's unit-stride dimension.
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    const bool a_even = TA ? (p.k % 2 == 0) : (p.m % 2 == 0);
    const bool b_even = TB ? (p.n % 2 == 0) : (p.k % 2 == 0);
    const bool vec = al(p.A) && al(p.B) && p.lda % 2 == 0 && p.ldb % 2 == 0 && a_even && b_even;
    const bool off32 = vec && p.lda < (1 << 24) && p.ldb < (1 << 24);
    if (off32) {
        if (sizeof(T) == 8) return launch_split<T, Tile128w8, TA, TB, true, true>(p, s);
        return launch_split<T, Tile256w8, TA, TB, true, true>(p, s);
    }
    if (vec) return launch_split<T, Tile128, TA, TB, true, false>(p, s);
    return launch_split<T, Tile128, TA, TB, false, false>(p, s);
}

static DmaPlan plan_dma(bool ta, bool tb, i64 m, i64 n, i64 k, const double* A, i64 lda, const double* B, i64 ldb) {
    return gemm_f64_lds_dma_plan(ta, tb, m, n, k, A, lda, B, ldb);
}
static DmaPlan plan_dma(bool ta, bool tb, i64 m, i64 n, i64 k, const float* A, i64 lda, const float* B, i64 ldb) {
    return gemm_f32_lds_dma_plan(ta, tb, m, n, k, A, lda, B, ldb);
}
static hipError_t run_dma(bool ta, bool tb, i64 m, i64 n, i64 kmain, i64 kchunk, double alpha, const double* A,
                          i64 lda, const double* B, i64 ldb, double beta, double* C, i64 ldc, hipStream_t s) {
    return gemm_f64_lds_dma(ta, tb, m, n, kmain, kchunk, alpha, A, lda, B, ldb, beta, C, ldc, s);
}
static hipError_t run_dma(bool ta, bool tb, i64 m, i64 n, i64 kmain, i64 kchunk, float alpha, const float* A,
                          i64 lda, const float* B, i64 ldb, float beta, float* C, i64 ldc, hipStream_t s) {
    return gemm_f32_lds_dma(ta, tb, m, n, kmain, kchunk, alpha, A, lda, B, ldb, beta, C, ldc, s);
}

template <typename T>
hipError_t gemm_mfma(bool ta, bool tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda,
                     const T* B, i64 ldb, T beta, T* C, i64 ldc, hipStream_t s) {
    {
        // the LDS-DMA kernels (gemm_f64g.hip / gemm_f32g.hip: 70.9 vs 65.9 TF for
        // this file's register-staged kernel at f64 16384^3, profiles/r01_f64_ab.log)
        const DmaPlan d = plan_dma(ta, tb, m, n, k, A, lda, B, ldb);
        if (d.use) {
            hipError_t e;
            if (d.nz == 1) {
                e = run_dma(ta, tb, m, n, d.kmain, d.kmain, alpha, A, lda, B, ldb, beta, C, ldc, s);
            } else {  // split-k: nz partials into a stream-ordered workspace, then the ordered reduce
                T* W = nullptr;
                e = workspace_alloc(reinterpret_cast<void**>(&W), sizeof(T) * (size_t)m * (size_t)n * d.nz, s);
                if (e != hipSuccess) return e;
                e = run_dma(ta, tb, m, n, d.kmain, d.kchunk, T(1), A, lda, B, ldb, T(0), W, m, s);
                if (e == hipSuccess) e = launch_reduce(m, n, d.nz, alpha, W, beta, C, ldc, s);
                const hipError_t f = workspace_free(W, s);
                if (e == hipSuccess) e = f;
            }
            if (e != hipSuccess || d.kmain == k) return e;
            // k tail: C += alpha op(A)(:, kmain:) op(B)(kmain:, :) with the general kernel
            A += ta ? d.kmain : d.kmain * lda;
            B += tb ? d.kmain * ldb : d.kmain;
            k -= d.kmain;
            beta = T(1);
        }
    }
    GemmParams<T> p{m, n, k, alpha, beta, A, lda, B, ldb, C, ldc, 0, 0, std::max<i64>(k, 1), 0};
    if (ta) return tb ? launch_tn<T, true, true>(p, s) : launch_tn<T, true, false>(p, s);
    return tb ? launch_tn<T, false, true>(p, s) : launch_tn<T, false, false>(p, s);
}

template hipError_t gemm_mfma<double>(bool, bool, i64, i64, i64, double, const double*, i64,
                                      const double*, i64, double, double*, i64, hipStream_t);
template hipError_t gemm_mfma<float>(bool, bool, i64, i64, i64, float, const float*, i64,
                                     const float*, i64, float, float*, i64, hipStream_t);

}  // namespace kern
}  // namespace elx
