// fp32 local panel update, LDS-DMA path for gfx950: C := alpha op(A) op(B) + beta C
// (column-major).  Replaces rocblas_sgemm on the hot path (configs C3-fp32 and
// C4: src/hydrogen/device/rocBLAS_API.cpp:151-170 via GPU_BLAS_impl.hpp:397-423).
//
// Same skeleton as gemm_f64g.hip (128 x 128 tile, 8 waves of 32 x 64, two
// LDS-DMA stages, two workgroups per CU) with fp32 specifics:
//  * v_mfma_f32_16x16x4_f32 (exact f32, 32 cycles); BK = 32 so a k-contiguous
//    image row is again 128 B.
//  * k-permuted MFMA steps: in step s (0..7) lane group g = lane>>4 supplies
//    k = 8g + s (the same permutation for A and B, so every k of the slab is
//    summed exactly once).  A lane then needs 8 CONSECUTIVE k of its row for
//    the whole slab: for a k-contiguous (KC) operand that is two ds_read_b128
//    per slab instead of eight ds_read_b32.
//  * swizzles (16-B chunk index): KC rows c ^ ((r>>1)&5) — searched
//    exhaustively to make both b128 reads of all four lane groups
//    conflict-free; RC (rows contiguous, 512-B k-rows) c ^ 4((kk>>3)&1) — the two
//    k-rows a 32-lane half of a ds_read_b32 touches land in different 64-B halves.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include "kernels.hpp"
#include "lds_dma.hpp"

namespace elx {
namespace kern {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32, GROUP_M = 8;
// Tile BM x BN of waves WTM x WTN: 128 x 128 of 32 x 64 (8 waves, 2 x 4
// accumulators) or 64 x 64 (4 waves, 4 x 4); 64 x 64 of 32 x 32 (4 waves, 2 x 2)
// for grids with few 128 x 128 tiles.  Two LDS stages of the two operand images.
// NST_ > 2: an LDS ring of NST_ slabs (the next NST_ - 1 in flight) for grids of
// at most one workgroup per CU, where one slab of lead is shorter than the DMA's
// latency.
template <int BM_, int BN_, int WTM_, int WTN_, int NST_ = 2>
struct FShape {
    static constexpr int BM = BM_, BN = BN_, WTM = WTM_, WTN = WTN_, MI = WTM / 16, NI = WTN / 16;
    static constexpr int WM = BM / WTM, WN = BN / WTN, NW = WM * WN, NT = 64 * NW, NST = NST_;
    static constexpr int IMGA = BM * BK * 4, IMGB = BN * BK * 4, STAGE = IMGA + IMGB;
    static constexpr int IPS = STAGE / 1024 / NW;  // DMA instructions per wave and slab (the ring's vmcnt unit)
    static constexpr int MINB = NST_ > 2 ? 1 : BM == 64 && BN == 64 ? 4 : 2;  // workgroups per CU the launch bounds ask for
    static_assert((NST_ - 1) * IPS <= 63 && NST_ * STAGE <= 160 * 1024, "ring depth");
};

struct FParams {
    i64 m, n, k;  // k: multiple of BK
    float alpha, beta;
    const float* A; i64 lda;
    const float* B; i64 ldb;
    float* C; i64 ldc;
    int tiles_m, tiles_n;
    // split-k (gridDim.y chunks): chunk z covers k in [z*kchunk, min(k, (z+1)*kchunk))
    // and writes C + z*zstride (the caller passes a workspace, alpha = 1, beta = 0)
    i64 kchunk, zstride;
    int vec_c;  // C 16-B aligned with ldc % 4 == 0: the interior epilogue's 16-B accesses
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

__device__ __forceinline__ int swz_kc(int r) { return (r >> 1) & 5; }
__device__ __forceinline__ int swz_rc(int kk) { return ((kk >> 3) & 1) << 2; }

// ROWS / 8 wave-instructions of 1 KiB per image; wave w issues w, w + NW, ...
template <bool BUF, bool KC, int ROWS, int NW>
__device__ __forceinline__ void stage_img(const float* X, i64 ld, i64 rows, i64 R, i64 k0, lds_char* img, int w,
                                          int l) {
    static_assert((ROWS / 8) % NW == 0, "image instructions split evenly over the waves");
    const DmaSrc<BUF, float> src(KC ? X + R * ld + k0 : X + R + k0 * ld, (KC ? ROWS : BK) * ld * 4);
#pragma unroll
    for (int q = 0; q < ROWS / 8 / NW; ++q) {
        const int ins = w + NW * q;
        if (KC) {  // X(row, k) = X[k + row*ld]; 8 rows of 128 B per instruction
            const int r = ins * 8 + (l >> 3);
            const int c = (l & 7) ^ swz_kc(r);
            const i64 row = R + r < rows ? r : rows - 1 - R;
            src.load(row * ld + 4 * c, img + ins * 1024);
        } else {   // X(row, k) = X[row + k*ld]; 1024 / (4 ROWS) k-rows of 4 ROWS B per instruction
            constexpr int CPK = ROWS / 4, KPI = 64 / CPK;  // 16-B chunks per k-row, k-rows per instruction
            const int kk = ins * KPI + l / CPK;
            const int c = (l % CPK) ^ swz_rc(kk);
            const i64 col = R + 4 * c <= rows - 4 ? 4 * c : rows - 4 - R;
            src.load(col + kk * ld, img + ins * 1024);
        }
    }
}

// The slab's 8 operand values of one 16-row fragment: element s = X(R0 + (l&15), 8(l>>4) + s).
template <bool KC, int ROWS>
__device__ __forceinline__ void frag(const lds_char* img, int R0, int l, float (&v)[8]) {
    const int r = R0 + (l & 15), g = l >> 4;
    if (KC) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = 2 * g + h;
            const f32x4 x = *(const __attribute__((address_space(3))) f32x4*)(img + r * 128 + ((c ^ swz_kc(r)) << 4));
#pragma unroll
            for (int e = 0; e < 4; ++e) v[4 * h + e] = x[e];
        }
    } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int kk = 8 * g + s;
            const int off = kk * (ROWS * 4) + (((r >> 2) ^ swz_rc(kk)) << 4) + ((r & 3) << 2);
            v[s] = *(const __attribute__((address_space(3))) float*)(img + off);
        }
    }
}

struct Frame {
    const float* A; i64 lda, m, m0;
    const float* B; i64 ldb, n, n0;
    int w, l, wr, wc;
};

// __restrict__ LDS pointers: alias scopes so the in-flight DMA is not drained
// before the ds_reads (see gemm_h256.hip).
template <typename SH, bool KCA, bool KCB, bool BUF>
__device__ __forceinline__ void slab(const Frame& f, i64 knext, bool more, lds_char* __restrict__ next,
                                     const lds_char* __restrict__ cur, f32x4 (&acc)[SH::MI][SH::NI]) {
    if (more) {
        stage_img<BUF, KCA, SH::BM, SH::NW>(f.A, f.lda, f.m, f.m0, knext, next, f.w, f.l);
        stage_img<BUF, KCB, SH::BN, SH::NW>(f.B, f.ldb, f.n, f.n0, knext, next + SH::IMGA, f.w, f.l);
    }
    float a[SH::MI][8], b[SH::NI][8];
#pragma unroll
    for (int mi = 0; mi < SH::MI; ++mi) frag<KCA, SH::BM>(cur, f.wr * SH::WTM + mi * 16, f.l, a[mi]);
#pragma unroll
    for (int ni = 0; ni < SH::NI; ++ni) frag<KCB, SH::BN>(cur + SH::IMGA, f.wc * SH::WTN + ni * 16, f.l, b[ni]);
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int mi = 0; mi < SH::MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < SH::NI; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mi][s], b[ni][s], acc[mi][ni], 0, 0, 0);
}

// BUF: staging through buffer descriptors (lds_dma.hpp) where the offsets fit.
template <typename SH, bool KCA, bool KCB, bool BETA0, bool BUF>
__global__ __launch_bounds__(SH::NT, SH::MINB) void gemm_f32g_kernel(FParams p) {
    constexpr int BM = SH::BM, BN = SH::BN, STAGE = SH::STAGE;
    __shared__ __attribute__((aligned(1024))) char lds_raw[SH::NST * STAGE];
    lds_char* lds = (lds_char*)lds_raw;
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w / SH::WN, wc = w % SH::WN;  // WM (M) x WN (N) waves of WTM x WTN
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;
    {
        const i64 kz0 = (i64)blockIdx.y * p.kchunk;
        p.k = min(p.kchunk, p.k - kz0);
        p.A += KCA ? kz0 : kz0 * p.lda;
        p.B += KCB ? kz0 : kz0 * p.ldb;
        p.C += (i64)blockIdx.y * p.zstride;
    }
    const Frame f{p.A, p.lda, p.m, m0, p.B, p.ldb, p.n, n0, w, l, wr, wc};

    f32x4 acc[SH::MI][SH::NI];
#pragma unroll
    for (int a = 0; a < SH::MI; ++a)
#pragma unroll
        for (int b = 0; b < SH::NI; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / BK);
    if constexpr (SH::NST == 2) {
        stage_img<BUF, KCA, BM, SH::NW>(p.A, p.lda, p.m, m0, 0, lds, w, l);
        stage_img<BUF, KCB, BN, SH::NW>(p.B, p.ldb, p.n, n0, 0, lds + SH::IMGA, w, l);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int t = 0; t < nt; ++t) {
            const int cur = t & 1;
            slab<SH, KCA, KCB, BUF>(f, (i64)(t + 1) * BK, t + 1 < nt, lds + (cur ^ 1) * STAGE, lds + cur * STAGE,
                                    acc);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    } else {
        // ring: slabs t+1 .. t+AHEAD in flight while slab t computes; slab t+AHEAD
        // goes into the stage slab t-1 left (every wave passed the barrier after
        // it).  Barriers without __syncthreads' fence, which would drain the ring.
        constexpr int AHEAD = SH::NST - 1;
#pragma unroll
        for (int q = 0; q < AHEAD; ++q) {
            if (q < nt) {
                stage_img<BUF, KCA, BM, SH::NW>(p.A, p.lda, p.m, m0, (i64)q * BK, lds + q * STAGE, w, l);
                stage_img<BUF, KCB, BN, SH::NW>(p.B, p.ldb, p.n, n0, (i64)q * BK, lds + q * STAGE + SH::IMGA, w, l);
            }
        }
        if (nt >= AHEAD) wait_cnt<(AHEAD - 1) * SH::IPS, NOWAIT_LGKM>();  // slab 0 landed
        else wait_cnt<0, NOWAIT_LGKM>();
        dma_barrier();
        int cur = 0, nxt = AHEAD;  // stages of slab t and of slab t + AHEAD
        for (int t = 0; t < nt; ++t) {
            slab<SH, KCA, KCB, BUF>(f, (i64)(t + AHEAD) * BK, t + AHEAD < nt, lds + nxt * STAGE, lds + cur * STAGE,
                                    acc);
            // slab t+1 landed (the AHEAD-1 younger slabs may fly; near the end
            // drain fully) and this wave's reads of slab t retired
            if (t + AHEAD < nt) wait_cnt<(AHEAD - 1) * SH::IPS, 0>();
            else wait_cnt<0, 0>();
            dma_barrier();
            cur = cur + 1 == SH::NST ? 0 : cur + 1;
            nxt = nxt + 1 == SH::NST ? 0 : nxt + 1;
        }
    }

    // Epilogue: C/D map of v_mfma_f32_16x16x4_f32: row = 4*(lane>>4) + reg, col = lane&15
    const int g = l >> 4, c = l & 15;
    const i64 ib = m0 + wr * SH::WTM + 4 * g, jb = n0 + wc * SH::WTN + c;
    if (p.vec_c && m0 + BM <= p.m && n0 + BN <= p.n) {
        // interior tile: a 16-row block's C loads all issued before its first
        // store (the guarded form below serializes load -> wait -> store per
        // element, since the compiler cannot reorder loads across the stores)
#pragma unroll
        for (int mi = 0; mi < SH::MI; ++mi) {
            f32x4 cv[SH::NI];
            if (!BETA0) {
#pragma unroll
                for (int ni = 0; ni < SH::NI; ++ni)
                    cv[ni] = *reinterpret_cast<const f32x4*>(p.C + (jb + ni * 16) * p.ldc + ib + mi * 16);
            }
#pragma unroll
            for (int ni = 0; ni < SH::NI; ++ni) {
                f32x4 v = p.alpha * acc[mi][ni];
                if (!BETA0) v += p.beta * cv[ni];
                *reinterpret_cast<f32x4*>(p.C + (jb + ni * 16) * p.ldc + ib + mi * 16) = v;
            }
        }
        return;
    }
#pragma unroll
    for (int mi = 0; mi < SH::MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < SH::NI; ++ni) {
            const i64 j = jb + ni * 16;
            if (j >= p.n) continue;
            float* col = p.C + j * p.ldc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 i = ib + mi * 16 + r;
                if (i < p.m) {
                    const float v = p.alpha * acc[mi][ni][r];
                    col[i] = BETA0 ? v : v + p.beta * col[i];
                }
            }
        }
}

template <typename SH, bool KCA, bool KCB, bool BUF>
hipError_t launch_fw(FParams p, hipStream_t s) {
    p.tiles_m = (int)((p.m + SH::BM - 1) / SH::BM);
    p.tiles_n = (int)((p.n + SH::BN - 1) / SH::BN);
    const dim3 grid(p.tiles_m * p.tiles_n, (unsigned)((p.k + p.kchunk - 1) / p.kchunk));
    const dim3 block(SH::NT);
    if (p.beta == 0.f) hipLaunchKernelGGL((gemm_f32g_kernel<SH, KCA, KCB, true, BUF>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((gemm_f32g_kernel<SH, KCA, KCB, false, BUF>), grid, block, 0, s, p);
    return hipGetLastError();
}

// 64 x 64 tiles (four waves of 32 x 32, four workgroups per CU, whole k) where
// prefer_t64 (kernels.hpp) says they balance the CUs better; ELX_F32G_T64 = 0
// never, 2 always (tests).
bool t64_tiles(i64 m, i64 n) {
    static const int v = [] { const char* e = getenv("ELX_F32G_T64"); return e ? atoi(e) : 1; }();
    return prefer_t64(v, m, n);
}

template <bool KCA, bool KCB, bool BUF>
hipError_t launch_fb(const FParams& p, hipStream_t s) {
    // 64 x 64 wave tiles (the fp64 kernel's choice) measured a wash on square
    // shapes: within -2 .. +1.7 % of 32 x 64 (profiles/r01_f32_wave.log).  Both
    // operands k-contiguous with a long k per tile (C4's TN, k = 524288 whole or
    // in split-k chunks of 131072) is the exception: 64 x 64 gains 2.5-5.5 %
    // from k = 65536 up (141 -> 149 TF at 8192^2 x 524288; k = 16384 -0.6 %;
    // profiles/r03_f32_wtm.log)
    static const int wtm_env = [] { const char* v = getenv("ELX_F32G_WTM"); return v ? atoi(v) : 0; }();
    const int wtm = wtm_env ? wtm_env : (KCA && KCB && p.kchunk >= 32768) ? 64 : 32;
    if (t64_tiles(p.m, p.n)) {
        // at most one workgroup per CU: a 4-slab LDS ring unless NN (NT 1024^2 x
        // 2048 72.7 -> 93.7 TF, TN 96.4 -> 99.8, NN even; the fp64 kernel lost
        // with it; profiles/r04_small_ring_ab.log)
        const i64 wgs = (p.m + 63) / 64 * ((p.n + 63) / 64) * ((p.k + p.kchunk - 1) / p.kchunk);
        if (wgs <= 256 && (KCA || !KCB)) return launch_fw<FShape<64, 64, 32, 32, 4>, KCA, KCB, BUF>(p, s);
        return launch_fw<FShape<64, 64, 32, 32>, KCA, KCB, BUF>(p, s);
    }
    if (wtm == 64) return launch_fw<FShape<128, 128, 64, 64>, KCA, KCB, BUF>(p, s);
    return launch_fw<FShape<128, 128, 32, 64>, KCA, KCB, BUF>(p, s);
}

template <bool KCA, bool KCB>
hipError_t launch_f(const FParams& p, hipStream_t s) {
    static const bool global_only = [] { const char* v = getenv("ELX_F32G_STAGE"); return v && v[0] == 'g'; }();
    if (!global_only && dma_fits(KCA ? 128 : BK, p.lda, 4) && dma_fits(KCB ? 128 : BK, p.ldb, 4))
        return launch_fb<KCA, KCB, true>(p, s);
    return launch_fb<KCA, KCB, false>(p, s);
}

bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace

DmaPlan gemm_f32_lds_dma_plan(bool ta, bool tb, i64 m, i64 n, i64 k, const float* A, i64 lda, const float* B,
                              i64 ldb) {
    const bool kca = ta, kcb = !tb;
    const bool ok = k >= BK && al16(A) && al16(B) && lda % 4 == 0 && ldb % 4 == 0 && (kca || (m % 4 == 0 && m >= 4)) &&
                    (kcb || (n % 4 == 0 && n >= 4)) && m < (1ll << 31) && n < (1ll << 31);
    if (t64_tiles(m, n)) return dma_plan(ok, (m + 63) / 64 * ((n + 63) / 64), k, BK);
    return dma_plan(ok, (m + 127) / 128 * ((n + 127) / 128), k, BK);
}

hipError_t gemm_f32_lds_dma(bool ta, bool tb, i64 m, i64 n, i64 kmain, i64 kchunk, float alpha, const float* A,
                            i64 lda, const float* B, i64 ldb, float beta, float* C, i64 ldc, hipStream_t s) {
    FParams p{m, n, kmain, alpha, beta, A, lda, B, ldb, C, ldc, 0, 0, kchunk, m * n, (reinterpret_cast<uintptr_t>(C) & 15) == 0 && ldc % 4 == 0 && (kchunk >= kmain || m % 4 == 0)};
    const bool kca = ta, kcb = !tb;
    if (kca) return kcb ? launch_f<true, true>(p, s) : launch_f<true, false>(p, s);
    return kcb ? launch_f<false, true>(p, s) : launch_f<false, false>(p, s);
}

}  // namespace kern
}  // namespace elx
