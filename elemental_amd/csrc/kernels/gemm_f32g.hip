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
#include <type_traits>
#include <utility>
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

// ---------------------------------------------------------------------------
// Ring kernel (round 5; the fp32 form of gemm_f64g.hip's gemm_f64r_kernel): one
// workgroup per CU, a BT x BT tile of four waves (2 x 2) of BT/2 x BT/2, and a
// 5-slot LDS ring of K-tiles of RBK k whose operand images are 32 KiB each
// (BT 128 with RBK 64 for grids of many tiles, BT 64 with RBK 128 for grids of
// few).  One barrier per K-tile (8192 MFMA cycles at BT 128, 4096 at BT 64), no
// vmcnt(0) drain, the next K-tile and half of the one after in flight.
// K permutation: in k-step s (0..RBK/4-1) lane group g = lane>>4 supplies
// k = (RBK/4) g + s for A and B alike, so a lane's four k-steps of one "quad"
// are four consecutive k of its row: one ds_read_b128 per fragment and quad for
// a k-contiguous (KC) image, four ds_read_b32 for a rows-contiguous (RC) one.
// Swizzles (16-B chunk index): KC row r: c ^ (r & 15); RC k-row kk: c ^ 4 g(kk)
// with g(kk) = kk / (RBK/4) the lane group reading it.  Both conflict-free: the
// 16 lanes of a group read 16 distinct chunks mod 16 (KC) / one 64-B window, the
// four groups in four different windows (RC).
// K-tile t (NQ = RBK/16 quads of 4 k-steps; each quad's MFMAs run on operands
// read during the previous quad):
//   quads 0..NQ/2-1: the 8 pieces of A_{t+2} per wave, into B_{t-1}'s slot;
//   quads 0..NQ-2:   MFMAs, reads of the next quad from A_t, B_t;
//   after NQ-2:      vmcnt(8) (A_{t+1}, B_{t+1} landed), lgkmcnt(0), barrier;
//   quad NQ-1:       MFMAs, reads of quad (t+1, 0) from A_{t+1}, B_{t+1}, the 8
//                    pieces of B_{t+2} into A_t's slot.
// The hazard argument is gemm_f64r_kernel's (gemm_f64g.hip).
// ---------------------------------------------------------------------------
namespace fring {
constexpr int NSLOT = 5;
// UN: bytes of one operand image (32 KiB: one workgroup per CU; 8 KiB: the 64 x 64
// tiles with 32-deep K-tiles, four workgroups per CU)
template <int BT, int UN>
struct G {
    static constexpr int UNIT = UN, NPW = UN / 1024 / 4, MINB = 32768 / UN;
    static constexpr int RBK = UN / 4 / BT, WT = BT / 2, MI = WT / 16, NQ = RBK / 16, KS = RBK / 4;
    static constexpr int NM = 4 * MI * MI, NR = 2 * MI;  // MFMAs and fragment reads per quad
};
// KC rows of CPR 16-B chunks: c ^ (r & 15), or (r >> 1) & 7 for 128-B rows (the 16
// lanes of a b128 read then hit 16 distinct chunk slots either way)
template <int CPR>
__device__ __forceinline__ int swz_r(int r) { return CPR >= 16 ? r & 15 : (r >> 1) & 7; }
template <int RBK>
__device__ __forceinline__ int swz_k(int kk) { return ((kk / (RBK / 4)) & 3) << 2; }

// RC images in 256-B lines: a 1-KiB piece = four consecutive k-rows x one
// 256-B line of the k-row (NSEG lines per k-row).  Two whole 512-B k-rows per
// piece (BT 128) measured 3.5-6 % slower, as in the fp64 ring
// (profiles/r05ab_f32_lines_ab.log, r05aa_f64_rcblk_ab.log).
// per-lane element offset of piece `ins` (0..31) of one operand's K-tile image
template <int BT, int UN, bool KC>
__device__ __forceinline__ i64 piece_off(int ins, int l, i64 R0, i64 rows, i64 ld) {
    constexpr int RBK = G<BT, UN>::RBK, KS = G<BT, UN>::KS;
    if (KC) {  // whole rows of RBK floats, RPI rows per piece (the 256-B lines of
               // 512-B rows measured slower at BT 64: TN 1024^2 x 2048 124 -> 120 TF)
        constexpr int CPR = RBK / 4, RPI = 64 / CPR;
        const int r = ins * RPI + l / CPR;
        const int c = (l % CPR) ^ swz_r<CPR>(r);
        const i64 row = R0 + r < rows ? r : rows - 1 - R0;
        return row * ld + 4 * c;
    } else {   // k-rows 4 kq.. of BT floats, line ins % NSEG; chunk ^ 4 g(kq)
        constexpr int NSEG = BT * 4 / 256;
        const int kq = ins / NSEG;
        const int kk = kq * 4 + (l >> 4);
        const int c = (ins % NSEG) * 16 + ((l & 15) ^ (((kq / (KS / 4)) & 3) << 2));
        const i64 col = R0 + 4 * c <= rows - 4 ? 4 * c : rows - 4 - R0;
        return col + kk * ld;
    }
}

template <int BT, int UN, bool BUF, bool KC>
__device__ __forceinline__ void piece(const float* X, i64 ld, i64 R0, i64 k0, int off, i64 goff, int ins,
                                      lds_char* img) {
    const float* base = KC ? X + R0 * ld + k0 : X + R0 + k0 * ld;
    if constexpr (BUF) {
        const BufferSrc<float> src(base, (KC ? BT : G<BT, UN>::RBK) * ld * 4);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src.rs, (__attribute__((address_space(3))) void*)(img + ins * 1024),
                                                 16, off, 0, 0, 0);
    } else {
        __builtin_amdgcn_global_load_lds((const void*)(base + goff),
                                         (__attribute__((address_space(3))) void*)(img + ins * 1024), 16, 0, 0);
    }
}

// quad j's four values of one 16-row fragment: v[e] = X(R0 + (l&15), KS (l>>4) + 4 j + e)
template <int BT, int UN, bool KC>
__device__ __forceinline__ void quad(const lds_char* img, int R0, int j, int l, float (&v)[4]) {
    constexpr int RBK = G<BT, UN>::RBK, KS = G<BT, UN>::KS;
    const int r = R0 + (l & 15), g = l >> 4;
    if (KC) {
        constexpr int CPR = RBK / 4;
        const int c = (KS / 4) * g + j;
        const f32x4 x = *(const __attribute__((address_space(3))) f32x4*)(img + r * (RBK * 4) + ((c ^ swz_r<CPR>(r)) << 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = x[e];
    } else {
        constexpr int NSEG = BT * 4 / 256;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int kq = (KS / 4) * g + j;  // k = 4 kq + e
            const int off = (kq * NSEG + (r >> 6)) * 1024 + e * 256 +
                            ((((r & 63) >> 2) ^ (((kq / (KS / 4)) & 3) << 2)) << 4) + ((r & 3) << 2);
            v[e] = *(const __attribute__((address_space(3))) float*)(img + off);
        }
    }
}

template <int BT, int UN>
struct Ops { float a[G<BT, UN>::MI][4], b[G<BT, UN>::MI][4]; };
template <int NPW>
struct Pieces { int offA[NPW], offB[NPW]; i64 gA[NPW], gB[NPW]; };

// one quad: the MFMAs of four k-steps on `cur`; quad `jrd` of rdA / rdB into
// `nxt` over the first half of them (fragment f after MFMA f MI); NP pieces u0..
// of one unit into `st` over the second half (SB: of B, else of A).  Unrolled
// by a fold over the MFMA index, not a loop: the placement is then constexpr.
template <int BT, int UN, bool KCA, bool KCB, bool BUF, bool SB, int NP>
struct Quad {
    static constexpr int MI = G<BT, UN>::MI, NM = G<BT, UN>::NM, NR = G<BT, UN>::NR, WT = G<BT, UN>::WT, H = NM / 2;
    const FParams& p;
    i64 m0, n0;
    int w, l, wr, wc;
    const Pieces<G<BT, UN>::NPW>& pc;
    const lds_char* __restrict__ rdA;
    const lds_char* __restrict__ rdB;
    int jrd;
    lds_char* __restrict__ st;
    int u0;
    i64 k0;

    template <int I>
    __device__ __forceinline__ void step(f32x4 (&acc)[MI][MI], const Ops<BT, UN>& cur, Ops<BT, UN>& nxt) const {
        constexpr int e = I / (MI * MI), mi = (I / MI) % MI, ni = I % MI;
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.a[mi][e], cur.b[ni][e], acc[mi][ni], 0, 0, 0);
        if constexpr (I % MI == 0 && I / MI < NR) {
            constexpr int f = I / MI;
            if constexpr (f < MI) quad<BT, UN, KCA>(rdA, wr * WT + f * 16, jrd, l, nxt.a[f]);
            else quad<BT, UN, KCB>(rdB, wc * WT + (f - MI) * 16, jrd, l, nxt.b[f - MI]);
        }
        if constexpr (NP > 0 && I >= H && (I - H) % (H / NP) == 0) {
            const int u = u0 + (I - H) / (H / NP);
            if constexpr (SB) piece<BT, UN, BUF, KCB>(p.B, p.ldb, n0, k0, pc.offB[u], pc.gB[u], w + 4 * u, st);
            else piece<BT, UN, BUF, KCA>(p.A, p.lda, m0, k0, pc.offA[u], pc.gA[u], w + 4 * u, st);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the placement as written
    }
    template <int... Is>
    __device__ __forceinline__ void run(f32x4 (&acc)[MI][MI], const Ops<BT, UN>& cur, Ops<BT, UN>& nxt,
                                        std::integer_sequence<int, Is...>) const {
        (step<Is>(acc, cur, nxt), ...);
    }
};

template <int BT, int UN, bool KCA, bool KCB, bool BUF, bool SB, int NP>
__device__ __forceinline__ void qstep(const FParams& p, i64 m0, i64 n0, int w, int l, int wr, int wc,
                                      const Pieces<G<BT, UN>::NPW>& pc, const lds_char* __restrict__ rdA,
                                      const lds_char* __restrict__ rdB, int jrd, lds_char* __restrict__ st, int u0,
                                      i64 k0, f32x4 (&acc)[G<BT, UN>::MI][G<BT, UN>::MI], const Ops<BT, UN>& cur, Ops<BT, UN>& nxt) {
    const Quad<BT, UN, KCA, KCB, BUF, SB, NP> q{p, m0, n0, w, l, wr, wc, pc, rdA, rdB, jrd, st, u0, k0};
    q.run(acc, cur, nxt, std::make_integer_sequence<int, G<BT, UN>::NM>{});
}
}  // namespace fring

template <int BT, int UN, bool KCA, bool KCB, bool BETA0, bool BUF>
__global__ __launch_bounds__(256, (fring::G<BT, UN>::MINB)) void gemm_f32r_kernel(FParams p) {
    using namespace fring;
    using Gm = G<BT, UN>;
    constexpr int RBK = Gm::RBK, WT = Gm::WT, MI = Gm::MI, NQ = Gm::NQ, UNIT = Gm::UNIT, NPW = Gm::NPW;
    constexpr int PPQ = NPW / (NQ / 2);  // pieces of A_{t+2} per quad over the first half
    __shared__ __attribute__((aligned(1024))) char lds_raw[NSLOT * UNIT];
    lds_char* lds = (lds_char*)lds_raw;
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 1, wc = w & 1;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
    const i64 m0 = (i64)tm * BT, n0 = (i64)tn * BT;
    {
        const i64 kz0 = (i64)blockIdx.y * p.kchunk;
        p.k = min(p.kchunk, p.k - kz0);
        p.A += KCA ? kz0 : kz0 * p.lda;
        p.B += KCB ? kz0 : kz0 * p.ldb;
        p.C += (i64)blockIdx.y * p.zstride;
    }
    Pieces<NPW> pc;
#pragma unroll
    for (int u = 0; u < NPW; ++u) {
        pc.gA[u] = piece_off<BT, UN, KCA>(w + 4 * u, l, m0, p.m, p.lda);
        pc.gB[u] = piece_off<BT, UN, KCB>(w + 4 * u, l, n0, p.n, p.ldb);
        pc.offA[u] = (int)(pc.gA[u] * 4);
        pc.offB[u] = (int)(pc.gB[u] * 4);
    }
    f32x4 acc[MI][MI];
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int b = 0; b < MI; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / RBK);
    auto kt = [&](int t) { return (i64)min(t, nt - 1) * RBK; };
    // prologue: A_0, B_0, A_1, B_1 into slots 0..3; wait for A_0, B_0; quad (0,0)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int u = 0; u < NPW; ++u)
            piece<BT, UN, BUF, KCA>(p.A, p.lda, m0, kt(t), pc.offA[u], pc.gA[u], w + 4 * u, lds + 2 * t * UNIT);
#pragma unroll
        for (int u = 0; u < NPW; ++u)
            piece<BT, UN, BUF, KCB>(p.B, p.ldb, n0, kt(t), pc.offB[u], pc.gB[u], w + 4 * u, lds + (2 * t + 1) * UNIT);
    }
    wait_cnt<2 * NPW, NOWAIT_LGKM>();
    dma_barrier();
    Ops<BT, UN> X, Y;
#pragma unroll
    for (int f = 0; f < MI; ++f) {
        quad<BT, UN, KCA>(lds, wr * WT + f * 16, 0, l, X.a[f]);
        quad<BT, UN, KCB>(lds + UNIT, wc * WT + f * 16, 0, l, X.b[f]);
    }
    wait_cnt<NOWAIT_VM, 0>();
    auto ktile = [&](auto jc, int t) {
        constexpr int J = decltype(jc)::value;
        constexpr int sA = 2 * J % NSLOT, sB = (2 * J + 1) % NSLOT, sA1 = (2 * J + 2) % NSLOT,
                      sB1 = (2 * J + 3) % NSLOT, st0 = (2 * J + 4) % NSLOT, st1 = (2 * J + 5) % NSLOT;
        const lds_char* rA = lds + sA * UNIT;
        const lds_char* rB = lds + sB * UNIT;
        const i64 k2 = kt(t + 2);
        // quads 0..NQ-2 (operands alternate X -> Y -> X; NQ is even); A_{t+2} over the first half
        auto q = [&](auto qc) {
            constexpr int Q = decltype(qc)::value;
            constexpr int NP = Q < NQ / 2 ? PPQ : 0;
            if constexpr (Q % 2 == 0)
                qstep<BT, UN, KCA, KCB, BUF, false, NP>(p, m0, n0, w, l, wr, wc, pc, rA, rB, Q + 1, lds + st0 * UNIT,
                                                    Q * PPQ, k2, acc, X, Y);
            else
                qstep<BT, UN, KCA, KCB, BUF, false, NP>(p, m0, n0, w, l, wr, wc, pc, rA, rB, Q + 1, lds + st0 * UNIT,
                                                    Q * PPQ, k2, acc, Y, X);
            if constexpr (Q < NQ - 2) wait_cnt<NOWAIT_VM, 0>();
        };
        q(std::integral_constant<int, 0>{});
        if constexpr (NQ >= 4) {
            q(std::integral_constant<int, 1>{});
            q(std::integral_constant<int, 2>{});
        }
        if constexpr (NQ == 8) {
            q(std::integral_constant<int, 3>{});
            q(std::integral_constant<int, 4>{});
            q(std::integral_constant<int, 5>{});
            q(std::integral_constant<int, 6>{});
        }
        wait_cnt<NPW, 0>();
        dma_barrier();
        // quad NQ-1: quad (t+1, 0) from A_{t+1}, B_{t+1}; B_{t+2} into A_t's slot
        qstep<BT, UN, KCA, KCB, BUF, true, NPW>(p, m0, n0, w, l, wr, wc, pc, lds + sA1 * UNIT, lds + sB1 * UNIT, 0,
                                          lds + st1 * UNIT, 0, k2, acc, Y, X);
        wait_cnt<NOWAIT_VM, 0>();
    };
    for (int t = 0; t < nt; t += NSLOT) {
        ktile(std::integral_constant<int, 0>{}, t);
        if (t + 1 < nt) ktile(std::integral_constant<int, 1>{}, t + 1);
        if (t + 2 < nt) ktile(std::integral_constant<int, 2>{}, t + 2);
        if (t + 3 < nt) ktile(std::integral_constant<int, 3>{}, t + 3);
        if (t + 4 < nt) ktile(std::integral_constant<int, 4>{}, t + 4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail pieces

    // Epilogue: C/D map of v_mfma_f32_16x16x4_f32: row = 4*(lane>>4) + reg, col = lane&15
    const int g = l >> 4, c = l & 15;
    const i64 ib = m0 + wr * WT + 4 * g, jb = n0 + wc * WT + c;
    if (p.vec_c && m0 + BT <= p.m && n0 + BT <= p.n) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
            f32x4 cv[MI];
            if (!BETA0) {
#pragma unroll
                for (int ni = 0; ni < MI; ++ni)
                    cv[ni] = *reinterpret_cast<const f32x4*>(p.C + (jb + ni * 16) * p.ldc + ib + mi * 16);
            }
#pragma unroll
            for (int ni = 0; ni < MI; ++ni) {
                f32x4 v = p.alpha * acc[mi][ni];
                if (!BETA0) v += p.beta * cv[ni];
                *reinterpret_cast<f32x4*>(p.C + (jb + ni * 16) * p.ldc + ib + mi * 16) = v;
            }
        }
        return;
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < MI; ++ni) {
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

template <int BT, int UN, bool KCA, bool KCB>
hipError_t launch_fr(FParams p, hipStream_t s) {
    constexpr int RBK = fring::G<BT, UN>::RBK;
    p.tiles_m = (int)((p.m + BT - 1) / BT);
    p.tiles_n = (int)((p.n + BT - 1) / BT);
    const dim3 grid(p.tiles_m * p.tiles_n, (unsigned)((p.k + p.kchunk - 1) / p.kchunk));
    // buffer-descriptor DMA when every offset of an image fits 31 bits, else the
    // global (64-bit address) form; ELX_F32G_STAGE=g forces the latter (read per call:
    // the tests cover it without operands of 2^21+ elements per row)
    const char* stg = getenv("ELX_F32G_STAGE");
    const bool buf = !(stg && stg[0] == 'g') && dma_fits(KCA ? BT : RBK, p.lda, 4) &&
                     dma_fits(KCB ? BT : RBK, p.ldb, 4);
    if (p.beta == 0.f) {
        if (buf) hipLaunchKernelGGL((gemm_f32r_kernel<BT, UN, KCA, KCB, true, true>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((gemm_f32r_kernel<BT, UN, KCA, KCB, true, false>), grid, dim3(256), 0, s, p);
    } else {
        if (buf) hipLaunchKernelGGL((gemm_f32r_kernel<BT, UN, KCA, KCB, false, true>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((gemm_f32r_kernel<BT, UN, KCA, KCB, false, false>), grid, dim3(256), 0, s, p);
    }
    return hipGetLastError();
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
// never, 2 always (tests).  A grid of exactly 256 128-tiles (2048^2) takes them
// too when k is short (2048^3 NN 135.6 -> 140.9 TF, TN 141.3 -> 141.8; at
// 2048^2 x 16384 the 128-tiles stay ahead, 144.0 vs 141.2;
// profiles/r05ai_f32_t64_rule_ab.log).  k compared as k / 64 * 64, so that the
// plan (k) and the launch (its kmain) decide alike.
bool t64_tiles(i64 m, i64 n, i64 k) {
    static const int v = [] { const char* e = getenv("ELX_F32G_T64"); return e ? atoi(e) : 1; }();
    if (v == 1 && (m + 127) / 128 * ((n + 127) / 128) == 256 && k / 64 * 64 <= 4096) return true;
    return prefer_t64(v, m, n);
}

// the ring kernel's tile edge for this grid (0: the slab kernels).  Measured
// against the slab kernels in one process (profiles/r05t_f32_ring_ab.log, and
// with the RC images in 256-B lines profiles/r05ac_f32_ring_policy_ab.log):
//  * 64 x 64 ring on grids of at most 256 64-tiles (one round of workgroups):
//    1024^2 x 2048 NN / TN / NT / TT 95 / 100 / 94 / 95 -> 123 / 124 / 123 / 122
//    TF; with more (1536 x 2048^2, three per CU in turn) 128 -> 120-126: slab;
//  * 128 x 128 ring, one workgroup per CU, on grids of fewer than 512
//    128-tiles, every orientation: round 5 first measured it where A is
//    k-contiguous (16384^3 TN 150.0 -> 151, TT 148.5 -> 149.5, 8192^2 x 65536
//    149.4 -> 151.6); the grids where A rows-contiguous (NN, NT) then favoured
//    the slab kernel's two workgroups per CU (8192^3, 4096^3, C3-f32's panel)
//    are >= 512-tile grids, which now take the two-per-CU ring below.  Round 6
//    A/B on 257..511-tile grids (profiles/r06b_f32_ring_ab.log, one process,
//    slab / one-per-CU / two-per-CU): 3072 x 2560 x 4096 NN 130.3 / 136.1 /
//    133.2, NT 129.0 / 134.7 / 133.1, TN 129.7 / 138.4 / 133.5; 2560^2 x 8192
//    even (124.7 all, NT 115.4 all).
//  * 64 x 64 ring with 32-deep K-tiles (8 KiB images), four workgroups per CU
//    ("65" below), on every grid of 64-tiles since it beats both (one process,
//    profiles/r05ah_f32_ring65_ab.log): 1536 x 2048^2 NN / TN / NT / TT 127 / 129 /
//    128 / 126 (slab) -> 143 / 143 / 142 / 142 TF, 3072^3 135 -> 148, 2560^3 118 ->
//    133, 1536^3 93 -> 106, 1024^3 109 -> 116, 1024^2 x 2048 123.3 (one per CU)
//    -> 124.0.
//  * 128 x 128 ring with 32-deep K-tiles (16 KiB images), two workgroups per CU
//    ("129"), on grids of >= 512 128-tiles, every orientation
//    (profiles/r05aj_f32_ring129_ab.log): 16384^3 NN / NT / TN / TT (slab or
//    one-per-CU ring) 150.7 / 149.5 / 151.3 / 149.7 -> 153.9 / 154.0 / 153.6 /
//    153.7 TF, 4096^3 NN 146.6 -> 150.6, C3-f32's 65536 x 8192^2 panel 150.1 ->
//    153.2, C4's TN 8192^2 x 65536 151.8 -> 151.4; with fewer tiles the one-per-
//    CU ring keeps whole k (2048^2 x 16384 NN 147.2 vs 146.5 split, 143.4 slab).
// ELX_F32G_RING (read per call, for the A/B and the tests) overrides: bit 0 the
// one-per-CU 128 x 128 ring and bit 3 the two-per-CU one on every grid of
// 128-tiles, bit 1 the one-per-CU 64 x 64 ring and bit 2 the four-per-CU one on
// grids of 64-tiles (both set: the first on grids of <= 256 64-tiles), 0 none.
int ring_bt(i64 m, i64 n, i64 k) {
    const char* e = getenv("ELX_F32G_RING");
    if (t64_tiles(m, n, k)) {
        const int v = e ? atoi(e) : 4;
        const bool one_round = (m + 63) / 64 * ((n + 63) / 64) <= 256;
        if ((v & 2) && ((v & 4) == 0 || one_round) && (e || one_round)) return 64;
        return (v & 4) ? 65 : 0;
    }
    if (e) return (atoi(e) & 8) ? 129 : (atoi(e) & 1) ? 128 : 0;
    return (m + 127) / 128 * ((n + 127) / 128) >= 512 ? 129 : 128;
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
    const int bt = ring_bt(p.m, p.n, p.k);
    if (bt == 128 && p.k % 64 == 0 && p.kchunk % 64 == 0) return launch_fr<128, 32768, KCA, KCB>(p, s);
    if (bt == 64 && p.k % 128 == 0 && p.kchunk % 128 == 0) return launch_fr<64, 32768, KCA, KCB>(p, s);
    if (bt == 65 && p.k % 32 == 0 && p.kchunk % 32 == 0) return launch_fr<64, 8192, KCA, KCB>(p, s);
    if (bt == 129 && p.k % 32 == 0 && p.kchunk % 32 == 0) return launch_fr<128, 16384, KCA, KCB>(p, s);
    if (t64_tiles(p.m, p.n, p.k)) {
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
    const int bt = ring_bt(m, n, k);
    if (bt == 65) return dma_plan(ok && k >= 32, (m + 63) / 64 * ((n + 63) / 64), k, 32, 1024);
    if (bt == 129) return dma_plan(ok && k >= 32, (m + 127) / 128 * ((n + 127) / 128), k, 32, 512);
    if (bt) {  // one workgroup per CU, K-tiles of 8192 / bt
        const int rbk = 8192 / bt;
        return dma_plan(ok && k >= rbk, (m + bt - 1) / bt * ((n + bt - 1) / bt), k, rbk, 256);
    }
    if (t64_tiles(m, n, k)) return dma_plan(ok, (m + 63) / 64 * ((n + 63) / 64), k, BK);
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
