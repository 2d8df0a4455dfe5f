// 16-bit local GEMM, large-tile path for gfx950: C := alpha op(A) op(B) + beta C
// (column-major, f32 accumulation, bf16 or f16 storage).
//
// Replaces rocblas_hgemm on the hot path (src/hydrogen/device/rocBLAS_API.cpp:151-170
// via include/hydrogen/blas/GPU_BLAS_impl.hpp:397-423, LocalGemm at
// src/blas_like/level3/Gemm.cpp:163-186) for the shapes SUMMA produces (config
// C5: local 16384 x 8192 x kc panels).  Edges it does not take (k tail, small or
// oddly aligned operands) go to the simple kernel of gemm_half.hip.
//
// Design (MI355X-first; cdna_hip_programming.md §5 "Canonical CDNA GEMM"):
//  * 256 x 256 output tile per 512-thread workgroup (8 waves, 2 (M) x 4 (N)),
//    each wave 128 x 64 = 8 x 4 accumulators of v_mfma_f32_16x16x32_{bf16,f16};
//    BK = 64 per K-tile, one workgroup per CU.
//  * Operands are staged HBM -> LDS with global_load_lds (16 B per lane, no
//    VGPR round trip), two LDS stages of 64 KiB, the next K-tile in flight
//    while the current one feeds the MFMAs.
//  * Every orientation reads through the same two LDS image kinds:
//      KC (k contiguous in HBM: op(A) = A^T, op(B) = B): rows of 64 k = 128 B,
//         read with ds_read_b128 straight into the MFMA fragment;
//      RC (rows contiguous: op(A) = A, op(B) = B^T): k-rows of 128 elements
//         = 256 B, read with the gfx950 transposing ds_read_b64_tr_b16 (two
//         per fragment), so no transpose pass and no extra HBM traffic.
//    Both images are XOR-swizzled on the 16-B chunk index so the fragment
//    reads are bank-conflict-free; the swizzle is applied to the GLOBAL source
//    address of each glds lane (the LDS side of glds is lane-linear).
//  * XCD-aware bijective workgroup remap (as gemm_mfma.hip).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <utility>
#include "kernels.hpp"
#include "lds_dma.hpp"
#include "elem.hpp"

namespace elx {
namespace kern {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int BM = 256, BN = 256, BK = 64, NT = 512, GROUP_M = 8;
constexpr int HALF = 128 * BK * 2;  // one half-tile image: 128 rows x 64 k x 2 B = 16 KiB
constexpr int STAGE = 4 * HALF;     // A halves 0,1 then B halves 0,1

struct H2Params {
    i64 m, n, k;  // k: multiple of BK
    float alpha, beta;
    const uint16_t* A; i64 lda;
    const uint16_t* B; i64 ldb;
    uint16_t* C; i64 ldc;
    int tiles_m, tiles_n;
    int vec_c;    // C base 8-B aligned and ldc % 4 == 0
    int group_m;  // tile-order group height (ELX_H16_GROUP, default GROUP_M)
};

__device__ __forceinline__ void tile_of(int bid, int nwg, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int per_group = group_m * tiles_n;
    const int group = wg / per_group;
    const int first_m = group * group_m;
    const int gsz = min(tiles_m - first_m, group_m);
    const int inner = wg - group * per_group;
    tm = first_m + inner % gsz;
    tn = inner / gsz;
}

// XOR swizzles (16-B chunk index).  KC: 8 chunks per 128-B row, row r -> c ^ ((r>>1)&7):
// the 16 lanes of a ds_read_b128 group (rows r..r+15 of one or two k-chunks) land
// on 16 distinct 16-B bank slots.  RC: 16 chunks per 256-B k-row, k-row kk ->
// c ^ (2(kk&3) + 8((kk>>3)&1)): the 8 k-rows x 32 B a 32-lane half of a
// ds_read_b64_tr_b16 touches land on distinct bank slots; XOR values are even,
// so the two chunks of a 32-B column pair stay adjacent.
__device__ __forceinline__ int swz_kc(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int swz_rc(int kk) { return ((kk & 3) << 1) | (((kk >> 3) & 1) << 3); }

__device__ __forceinline__ void glds16(const uint16_t* src, lds_char* dst) {
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// Stage one half-tile (128 operand rows starting at global row R, 64 k from k0)
// into its LDS image.  16 wave-instructions of 1 KiB; wave w issues w and w+8.
template <bool KC>
__device__ __forceinline__ void stage_half(const uint16_t* X, i64 ld, i64 rows, i64 R, i64 k0, lds_char* img, int w,
                                           int l) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ins = w + 8 * q;
        if (KC) {  // X(row, k) = X[k + row*ld]; instruction = 8 rows of 128 B
            const int r = ins * 8 + (l >> 3);
            const int c = (l & 7) ^ swz_kc(r);
            i64 row = R + r;
            row = row < rows ? row : rows - 1;  // rows past the edge: any valid data (never stored)
            glds16(X + row * ld + k0 + 8 * c, img + ins * 1024);
        } else {   // X(row, k) = X[row + k*ld]; instruction = 4 k-rows of 256 B
            const int kk = ins * 4 + (l >> 4);
            const int c = (l & 15) ^ swz_rc(kk);
            i64 col = R + 8 * c;
            col = col <= rows - 8 ? col : rows - 8;
            glds16(X + col + (k0 + kk) * ld, img + ins * 1024);
        }
    }
}

// One MFMA operand fragment (16 operand rows from R0, k-step s of 32):
// lane l holds X(R0 + (l&15), 32s + 8(l>>4) + j), j = 0..7.
template <bool KC>
__device__ __forceinline__ u32x4 frag(const lds_char* img, int R0, int s, int l) {
    if (KC) {
        const int row = R0 + (l & 15), c = 4 * s + (l >> 4);
        return *(const __attribute__((address_space(3))) u32x4*)(img + row * 128 + ((c ^ swz_kc(row)) << 4));
    } else {
        const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
        const int c = (R0 >> 3) + (p >> 1);
        u32x4 out;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kk = 32 * s + 8 * g + 4 * h + q;
            const lds_char* a = img + kk * 256 + ((c ^ swz_rc(kk)) << 4) + ((p & 1) << 3);
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
            const u32x2 u = __builtin_bit_cast(u32x2, v);
            out[2 * h] = u[0];
            out[2 * h + 1] = u[1];
        }
        return out;
    }
}

template <bool BF16>
__device__ __forceinline__ f32x4 mfma(u32x4 a, u32x4 b, f32x4 c) {
    if constexpr (BF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                      0, 0);
}

struct Frame {  // per-workgroup constants of the main loop
    const uint16_t* A; i64 lda, m, m0;
    const uint16_t* B; i64 ldb, n, n0;
    int w, l, wr, wc;
};

// One main-loop step: stage K-tile t+1 into `next` (if any) and run the MFMAs of
// the K-tile already in `cur`.  The two LDS pointers are __restrict__ so the
// inlined accesses carry alias scopes: hipcc's waitcnt pass then knows the
// in-flight glds writes cannot alias the ds_reads and does not wait vmcnt(0)
// before them (without the scopes every ds_read would drain the prefetch).
template <bool BF16, bool KCA, bool KCB>
__device__ __forceinline__ void step(const Frame& f, i64 knext, bool more, lds_char* __restrict__ next,
                                     const lds_char* __restrict__ cur, f32x4 (&acc)[8][4]) {
    if (more) {
        stage_half<KCA>(f.A, f.lda, f.m, f.m0, knext, next, f.w, f.l);
        stage_half<KCA>(f.A, f.lda, f.m, f.m0 + 128, knext, next + HALF, f.w, f.l);
        stage_half<KCB>(f.B, f.ldb, f.n, f.n0, knext, next + 2 * HALF, f.w, f.l);
        stage_half<KCB>(f.B, f.ldb, f.n, f.n0 + 128, knext, next + 3 * HALF, f.w, f.l);
    }
    const lds_char* Ah = cur + f.wr * HALF;
    const lds_char* Bh = cur + 2 * HALF + (f.wc >> 1) * HALF;
    const int bc = (f.wc & 1) * 64;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
        u32x4 a[8], b[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) b[ni] = frag<KCB>(Bh, bc + ni * 16, s, f.l);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) a[mi] = frag<KCA>(Ah, mi * 16, s, f.l);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma<BF16>(a[mi], b[ni], acc[mi][ni]);
    }
}

template <bool BF16, int NI = 4>
__device__ __forceinline__ void epilogue(const H2Params& p, const f32x4 (&acc)[8][NI], i64 m0, i64 n0, int wr, int wc,
                                         int l);

// KCA: op(A) k-contiguous (TA); KCB: op(B) k-contiguous (!TB).
// FL: timing ablations only (wrong results): 1 = no staging after the first
// K-tile, 2 = no barrier, 8 = raw barrier without the DMA wait
template <bool BF16, bool KCA, bool KCB, int FL = 0>
__global__ __launch_bounds__(NT, 1) void gemm_h256_kernel(H2Params p) {
    __shared__ __attribute__((aligned(1024))) char lds_raw[2 * STAGE];
    lds_char* lds = (lds_char*)lds_raw;  // generic -> LDS address space

    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;
    const Frame f{p.A, p.lda, p.m, m0, p.B, p.ldb, p.n, n0, w, l, wr, wc};

    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / BK);
    stage_half<KCA>(f.A, f.lda, f.m, m0, 0, lds, w, l);
    stage_half<KCA>(f.A, f.lda, f.m, m0 + 128, 0, lds + HALF, w, l);
    stage_half<KCB>(f.B, f.ldb, f.n, n0, 0, lds + 2 * HALF, w, l);
    stage_half<KCB>(f.B, f.ldb, f.n, n0 + 128, 0, lds + 3 * HALF, w, l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        const int cur = t & 1;
        step<BF16, KCA, KCB>(f, (i64)(t + 1) * BK, !(FL & 1) && t + 1 < nt, lds + (cur ^ 1) * STAGE,
                             lds + cur * STAGE, acc);
        // the staged K-tile has landed and every wave is done reading the other
        if (FL & 8) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (!(FL & 2)) __syncthreads();
        }
    }

    epilogue<BF16>(p, acc, m0, n0, wr, wc, l);
}

// ---------------------------------------------------------------------------
// Phased variant: same tile, images and fragments, but each K-tile runs as four
// phases of 16 MFMAs (one 64 x 32 quadrant of the wave's 128 x 64 block), and
// the two wave groups (wr = 0, 1: the two waves sharing a SIMD) run one barrier
// apart, so in every barrier interval one wave of each SIMD issues MFMAs while
// its partner issues the next phase's fragment reads and one image of staging
// (cdna_hip_programming.md §5, "The 256^2 8-phase template").
//
// The four LDS images of a stage are the quadrant halves, not the wave-group
// halves: A image h holds rows {64h..64h+63} of both 128-row groups (image row
// r -> tile row 128(r>>6) + 64h + (r&63)), B image h holds columns
// {32h..32h+31} of each wave column (r -> 64(r>>5) + 32h + (r&31)), so the
// quadrant order (0,0) (0,1) (1,1) (1,0) consumes A0+B0, B1, A1, - and the
// next K-tile's images are staged in that same order, one per phase.
//
// Ordering (P = phase index, two barriers per phase, group 1 one barrier late):
//  RAW: an image staged in phase P is read in phase P+3 (P+4 for A0); every
//       wave waits for it in phase P+2 (s_waitcnt vmcnt(4): the two images
//       staged after it may stay in flight) before that phase's first barrier.
//  WAR: an image is restaged >= 4 phases after its last read, whose
//       completion the MFMAs of that phase already forced.
__device__ __forceinline__ i64 img_row(bool isB, int h, int r) {
    return isB ? (i64)((r >> 5) * 64 + h * 32 + (r & 31)) : (i64)((r >> 6) * 128 + h * 64 + (r & 63));
}

// Stage quadrant image `which` (0: A0, 1: A1, 2: B0, 3: B1) of K-tile k0: two
// 1-KiB wave-instructions per wave.
template <bool BUF, bool KC>
__device__ __forceinline__ void stage_q(const Frame& f, int which, i64 k0, lds_char* img) {
    const bool isB = which >= 2;
    const int h = which & 1;
    const uint16_t* X = isB ? f.B : f.A;
    const i64 ld = isB ? f.ldb : f.lda, rows = isB ? f.n : f.m, R0 = isB ? f.n0 : f.m0;
    // offsets from the tile's corner at k0: < 256 operand rows (KC) or BK k-rows (RC) of ld
    const DmaSrc<BUF, uint16_t> src(KC ? X + R0 * ld + k0 : X + R0 + k0 * ld, (KC ? 256 : BK) * ld * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int ins = f.w + 8 * j;
        if (KC) {
            const int r = ins * 8 + (f.l >> 3);
            const int c = (f.l & 7) ^ swz_kc(r);
            i64 row = img_row(isB, h, r);
            row = R0 + row < rows ? row : rows - 1 - R0;
            src.load(row * ld + 8 * c, img + ins * 1024);
        } else {
            const int kk = ins * 4 + (f.l >> 4);
            const int c = (f.l & 15) ^ swz_rc(kk);
            i64 col = img_row(isB, h, 8 * c);
            col = R0 + col <= rows - 8 ? col : rows - 8 - R0;
            src.load(col + kk * ld, img + ins * 1024);
        }
    }
}

__device__ __forceinline__ void bar8() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

template <bool BF16, int FL = 0>
__device__ __forceinline__ void cluster(f32x4 (&acc)[8][4], int mq, int nq, const u32x4 (&a)[8], const u32x4 (&b)[4]) {
    if (!(FL & 4)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
                acc[mq * 4 + mi][nq * 2 + ni] = mfma<BF16>(a[s * 4 + mi], b[s * 2 + ni], acc[mq * 4 + mi][nq * 2 + ni]);
    if (!(FL & 4)) __builtin_amdgcn_s_setprio(0);
}

// One K-tile: four phases over `cur`, staging K-tile knext into `next`.
template <bool BF16, bool KCA, bool KCB, bool BUF, int FL = 0>
__device__ __forceinline__ void step8(const Frame& f, i64 knext, bool more, lds_char* __restrict__ next,
                                      const lds_char* __restrict__ cur, f32x4 (&acc)[8][4]) {
    u32x4 a[8], b0[4], b1[4];
    const int ar = f.wr * 64, bcol = f.wc * 32;
    auto load_a = [&](const lds_char* img) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) a[s * 4 + mi] = frag<KCA>(img, ar + mi * 16, s, f.l);
    };
    auto load_b = [&](u32x4 (&b)[4], const lds_char* img) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b[s * 2 + ni] = frag<KCB>(img, bcol + ni * 16, s, f.l);
    };
    // phase 0: quadrant (0,0)
    load_b(b0, cur + 2 * HALF);
    load_a(cur);
    if (more) {
        if (!(FL & 1)) stage_q<BUF, KCA>(f, 0, knext, next);
        if (!(FL & 2)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar8();
    cluster<BF16, FL>(acc, 0, 0, a, b0);
    bar8();
    // phase 1: quadrant (0,1)
    load_b(b1, cur + 3 * HALF);
    if (more && !(FL & 1)) stage_q<BUF, KCB>(f, 2, knext, next + 2 * HALF);
    if (!(FL & 2)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    bar8();
    cluster<BF16, FL>(acc, 0, 1, a, b1);
    bar8();
    // phase 2: quadrant (1,1)
    load_a(cur + HALF);
    if (more && !(FL & 1)) stage_q<BUF, KCB>(f, 3, knext, next + 3 * HALF);
    bar8();
    cluster<BF16, FL>(acc, 1, 1, a, b1);
    bar8();
    // phase 3: quadrant (1,0)
    if (more && !(FL & 1)) stage_q<BUF, KCA>(f, 1, knext, next + HALF);
    if (!(FL & 2)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    bar8();
    cluster<BF16, FL>(acc, 1, 0, a, b0);
    bar8();
}

// BUF: staging through buffer descriptors (lds_dma.hpp) where the offsets fit.
// FL: timing ablations only (wrong results): 1 = no staging after the first
// K-tile, 2 = no counted vmcnt waits, 4 = no s_setprio
template <bool BF16, bool KCA, bool KCB, bool BUF, int FL = 0>
__global__ __launch_bounds__(NT, 1) void gemm_h8p_kernel(H2Params p) {
    __shared__ __attribute__((aligned(1024))) char lds_raw[2 * STAGE];
    lds_char* lds = (lds_char*)lds_raw;

    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;
    const Frame f{p.A, p.lda, p.m, m0, p.B, p.ldb, p.n, n0, w, l, wr, wc};

    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / BK);
    stage_q<BUF, KCA>(f, 0, 0, lds);
    stage_q<BUF, KCA>(f, 1, 0, lds + HALF);
    stage_q<BUF, KCB>(f, 2, 0, lds + 2 * HALF);
    stage_q<BUF, KCB>(f, 3, 0, lds + 3 * HALF);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar8();
    if (wr == 1) bar8();  // group 1 runs one barrier behind group 0
    for (int t = 0; t < nt; ++t) {
        const int cur = t & 1;
        step8<BF16, KCA, KCB, BUF, FL>(f, (i64)(t + 1) * BK, t + 1 < nt, lds + (cur ^ 1) * STAGE, lds + cur * STAGE, acc);
    }
    if (wr == 0) bar8();  // matches group 1's last barrier

    epilogue<BF16>(p, acc, m0, n0, wr, wc, l);
}

// ---------------------------------------------------------------------------
// Balanced-read variant of the phased kernel: the same tile, images, quadrant
// order and barrier schedule, but the next K-tile's images are staged in the
// order B0, A0, B1, A1 and B0(t+1) is read in phase 3 of K-tile t (into the B
// register set B1(t) just vacated), so the fragment reads per phase are
// 8, 4, 8, 4 instead of 12, 4, 8, 0 (the 12-read phase 0 is as long in LDS
// cycles as its 16 MFMAs).  The two B register sets swap roles every K-tile
// (the loop is unrolled by two).  Every phase waits vmcnt(4): the image read
// in the next phase was staged two phases earlier (RAW), and every image is
// restaged >= 4 phases after its last read (WAR).
// ---------------------------------------------------------------------------
template <bool BF16, bool KCA, bool KCB, bool BUF>
__device__ __forceinline__ void step8b(const Frame& f, i64 knext, bool more, lds_char* __restrict__ next,
                                       const lds_char* __restrict__ cur, f32x4 (&acc)[8][4], u32x4 (&a)[8],
                                       u32x4 (&bY)[4], u32x4 (&bX)[4]) {
    const int ar = f.wr * 64, bcol = f.wc * 32;
    auto load_a = [&](const lds_char* img) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) a[s * 4 + mi] = frag<KCA>(img, ar + mi * 16, s, f.l);
    };
    auto load_b = [&](u32x4 (&b)[4], const lds_char* img) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b[s * 2 + ni] = frag<KCB>(img, bcol + ni * 16, s, f.l);
    };
    auto wait = [&]() {
        if (more) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    // phase 0: quadrant (0,0): A0(t) read now, B0(t) already in bY
    load_a(cur);
    if (more) stage_q<BUF, KCB>(f, 2, knext, next + 2 * HALF);
    wait();
    bar8();
    cluster<BF16>(acc, 0, 0, a, bY);
    bar8();
    // phase 1: quadrant (0,1) from B1(t)
    load_b(bX, cur + 3 * HALF);
    if (more) stage_q<BUF, KCA>(f, 0, knext, next);
    wait();
    bar8();
    cluster<BF16>(acc, 0, 1, a, bX);
    bar8();
    // phase 2: quadrant (1,1) from A1(t)
    load_a(cur + HALF);
    if (more) stage_q<BUF, KCB>(f, 3, knext, next + 3 * HALF);
    wait();
    bar8();
    cluster<BF16>(acc, 1, 1, a, bX);
    bar8();
    // phase 3: quadrant (1,0) from registers; B0(t+1) (waited in phase 2) read into bX
    if (more) {
        load_b(bX, next + 2 * HALF);
        stage_q<BUF, KCA>(f, 1, knext, next + HALF);
    }
    wait();
    bar8();
    cluster<BF16>(acc, 1, 0, a, bY);
    bar8();
}

template <bool BF16, bool KCA, bool KCB, bool BUF>
__global__ __launch_bounds__(NT, 1) void gemm_h8b_kernel(H2Params p) {
    __shared__ __attribute__((aligned(1024))) char lds_raw[2 * STAGE];
    lds_char* lds = (lds_char*)lds_raw;

    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;
    const Frame f{p.A, p.lda, p.m, m0, p.B, p.ldb, p.n, n0, w, l, wr, wc};

    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / BK);
    stage_q<BUF, KCB>(f, 2, 0, lds + 2 * HALF);
    stage_q<BUF, KCA>(f, 0, 0, lds);
    stage_q<BUF, KCB>(f, 3, 0, lds + 3 * HALF);
    stage_q<BUF, KCA>(f, 1, 0, lds + HALF);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar8();
    u32x4 a[8], b0[4], b1[4];
    {
        const int bcol = wc * 32;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b0[s * 2 + ni] = frag<KCB>(lds + 2 * HALF, bcol + ni * 16, s, l);
    }
    if (wr == 1) bar8();  // group 1 runs one barrier behind group 0
    for (int t = 0; t < nt; t += 2) {
        step8b<BF16, KCA, KCB, BUF>(f, (i64)(t + 1) * BK, t + 1 < nt, lds + STAGE, lds, acc, a, b0, b1);
        if (t + 1 < nt)
            step8b<BF16, KCA, KCB, BUF>(f, (i64)(t + 2) * BK, t + 2 < nt, lds, lds + STAGE, acc, a, b1, b0);
    }
    if (wr == 0) bar8();  // matches group 1's last barrier

    epilogue<BF16>(p, acc, m0, n0, wr, wc, l);
}

// ---------------------------------------------------------------------------
// Deep-prefetch two-phase variant: the same tile, images and fragments, but each
// K-tile runs as TWO phases of 32 MFMAs (phase h: the wave's rows {64h..64h+63}
// x all 64 of its columns), so every barrier interval carries twice the MFMA
// work of the phased kernels, and the B fragments are read once per K-tile and
// kept for both phases.  Staging runs ~1.5 K-tiles ahead in the same two LDS
// stages: the images of K-tile s that phase 0 reads (B0, B1, A0) are free once
// phase 0's reads have retired, so K-tile s+2's B0, B1, A0 are staged into them
// in phase 1 of s, and s+2's A1 in phase 0 of s+1 (into the slot K-tile s's A1
// leaves when its phase-1 reads retire).  Per wave and phase: reads, staging,
// `s_waitcnt vmcnt(8)` (the images read next were staged >= 3 intervals
// earlier; the 8 youngest pieces may stay in flight), `lgkmcnt(0)` (every read
// of this interval retired before the barrier, so the other group may restage
// what it read: WAR), barrier, 32 MFMAs, barrier; the two wave groups one
// barrier apart as in the phased kernels.
// ---------------------------------------------------------------------------
template <bool BF16>
__device__ __forceinline__ void cluster32(f32x4 (&acc)[8][4], int h, const u32x4 (&a)[8], const u32x4 (&b)[8]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[h * 4 + mi][ni] = mfma<BF16>(a[s * 4 + mi], b[s * 4 + ni], acc[h * 4 + mi][ni]);
    __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void wait_stage(bool deep) {
    if (deep) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// phase 0 of K-tile t (in `cur`): B and A0 fragments read from cur, K-tile t+1's
// A1 staged into `nxtA1` (t+1's stage), then the first 32 MFMAs
template <bool BF16, bool KCA, bool KCB, bool BUF>
__device__ __forceinline__ void phase0(const Frame& f, const lds_char* __restrict__ cur, lds_char* __restrict__ nxtA1,
                                       i64 k1, bool st, bool deep, f32x4 (&acc)[8][4], u32x4 (&a)[8], u32x4 (&b)[8]) {
    const int ar = f.wr * 64, bcol = f.wc * 32;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
                b[s * 4 + h * 2 + ni] = frag<KCB>(cur + (2 + h) * HALF, bcol + ni * 16, s, f.l);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) a[s * 4 + mi] = frag<KCA>(cur, ar + mi * 16, s, f.l);
    if (st) stage_q<BUF, KCA>(f, 1, k1, nxtA1);
    wait_stage(deep);
    bar8();
    cluster32<BF16>(acc, 0, a, b);
    bar8();
}

// phase 1 of K-tile t: A1 fragments read from cur, K-tile t+2's B0, B1, A0 staged
// into cur's (now free) slots, then the second 32 MFMAs
template <bool BF16, bool KCA, bool KCB, bool BUF>
__device__ __forceinline__ void phase1(const Frame& f, const lds_char* __restrict__ curA1, lds_char* __restrict__ curA0,
                                       lds_char* __restrict__ curB, i64 k2, bool st, bool deep, f32x4 (&acc)[8][4],
                                       u32x4 (&a)[8], const u32x4 (&b)[8]) {
    const int ar = f.wr * 64;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) a[s * 4 + mi] = frag<KCA>(curA1, ar + mi * 16, s, f.l);
    if (st) {
        stage_q<BUF, KCB>(f, 2, k2, curB);
        stage_q<BUF, KCB>(f, 3, k2, curB + HALF);
        stage_q<BUF, KCA>(f, 0, k2, curA0);
    }
    wait_stage(deep);
    bar8();
    cluster32<BF16>(acc, 1, a, b);
    bar8();
}

template <bool BF16, bool KCA, bool KCB, bool BUF>
__global__ __launch_bounds__(NT, 1) void gemm_h4d_kernel(H2Params p) {
    __shared__ __attribute__((aligned(1024))) char lds_raw[2 * STAGE];
    lds_char* lds = (lds_char*)lds_raw;

    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;
    const Frame f{p.A, p.lda, p.m, m0, p.B, p.ldb, p.n, n0, w, l, wr, wc};

    f32x4 acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / BK);
    // prologue: K-tile 0 whole, K-tile 1's B0, B1, A0
    stage_q<BUF, KCB>(f, 2, 0, lds + 2 * HALF);
    stage_q<BUF, KCB>(f, 3, 0, lds + 3 * HALF);
    stage_q<BUF, KCA>(f, 0, 0, lds);
    stage_q<BUF, KCA>(f, 1, 0, lds + HALF);
    if (nt > 1) {
        stage_q<BUF, KCB>(f, 2, BK, lds + STAGE + 2 * HALF);
        stage_q<BUF, KCB>(f, 3, BK, lds + STAGE + 3 * HALF);
        stage_q<BUF, KCA>(f, 0, BK, lds + STAGE);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar8();
    if (wr == 1) bar8();  // group 1 runs one barrier behind group 0
    u32x4 a[8], b[8];
    for (int t = 0; t < nt; t += 2) {
        // K-tile t in stage 0, t+1 in stage 1 (the loop is unrolled by two so the
        // stage pointers are compile-time offsets of the LDS base)
        phase0<BF16, KCA, KCB, BUF>(f, lds, lds + STAGE + HALF, (i64)(t + 1) * BK, t + 1 < nt, t + 2 < nt, acc, a, b);
        phase1<BF16, KCA, KCB, BUF>(f, lds + HALF, lds, lds + 2 * HALF, (i64)(t + 2) * BK, t + 2 < nt, t + 2 < nt, acc,
                                    a, b);
        if (t + 1 < nt) {
            phase0<BF16, KCA, KCB, BUF>(f, lds + STAGE, lds + HALF, (i64)(t + 2) * BK, t + 2 < nt, t + 3 < nt, acc, a,
                                        b);
            phase1<BF16, KCA, KCB, BUF>(f, lds + STAGE + HALF, lds + STAGE, lds + STAGE + 2 * HALF, (i64)(t + 3) * BK,
                                        t + 3 < nt, t + 3 < nt, acc, a, b);
        }
    }
    if (wr == 0) bar8();  // matches group 1's last barrier

    epilogue<BF16>(p, acc, m0, n0, wr, wc, l);
}

// ---------------------------------------------------------------------------
// Four-wave kernel: the same 256 x 256 output tile, but 4 waves (2 x 2), one per
// SIMD, each owning 128 x 128 = 8 x 8 accumulators (256 AGPRs; the wave has the
// whole 512-entry file).  Per FLOP this halves the B-fragment LDS reads of the
// eight-wave kernels (a wave's fragments feed 8 x 8 MFMAs instead of 8 x 4), cuts
// a third of all LDS instructions, and leaves no partner wave on the SIMD to take
// matrix-pipe slots or issue bandwidth (MI355X_MICROARCH.md "Two waves per SIMD"
// items 1-3): each wave issues its own fragment reads and staging between its
// MFMAs.  hipBLASLt's bf16 kernels on these shapes have the same geometry
// (MT256x256x64, MI16x16, 4 waves: profiles/r03_vendor_pmc.json).
//
// Staging unit = one operand's K-tile image (256 rows x 64 k = 32 KiB, the KC /
// RC half images of the kernels above: 128-B KC rows, 256-B RC k-rows), in a
// ring of 5 slots (160 KiB): A_t is unit 2t, B_t unit 2t+1, unit u in slot u % 5.
// Each K-tile runs as two k-steps of 64 MFMAs per wave:
//   (t,0): MFMAs on fragments (t,0) [set X]; read fragments (t,1) [set Y] from
//          A_t, B_t; stage A_{t+2} into B_{t-1}'s slot; then vmcnt(8) (A_{t+1}
//          and B_{t+1} landed, A_{t+2} may stay in flight), lgkmcnt(0), barrier;
//   (t,1): MFMAs on (t,1) [Y]; read (t+1,0) [X] from A_{t+1}, B_{t+1}; stage
//          B_{t+2} into A_t's slot; lgkmcnt(0), no barrier.
// RAW: A_{t+1}, B_{t+1} are read from (t,1) on, after every wave's wait and the
// barrier ending (t,0).  WAR: A_t's and B_t's last reads are issued in (t,0) and
// retired before that barrier; their slots are restaged in (t,1) and (t+1,0).
// No wave can be two k-steps ahead of another (it would have passed a barrier
// the other has not reached), so one barrier per K-tile suffices.  Units past
// the end re-stage the last K-tile into a slot nobody reads again, so every
// k-step issues the same 8 pieces and the counted wait is exact without branches.
// The accumulators are tied to AGPRs through inline asm (mfma_acc).
// ---------------------------------------------------------------------------
namespace w4 {
constexpr int UNIT = 256 * BK * 2;  // one operand's K-tile image: 32 KiB
constexpr int NSLOT = 5;

// per-lane offset (elements from the image's corner at k0) of piece j (0..31)
// of one operand's K-tile image: half j >> 4, wave-instruction j & 15 of it, as
// stage_half lays them out
template <bool KC>
__device__ __forceinline__ i64 piece_off(int j, int l, i64 R0, i64 rows, i64 ld) {
    const int h = j >> 4, ins = j & 15;
    if (KC) {
        const int r = ins * 8 + (l >> 3);
        const int c = (l & 7) ^ swz_kc(r);
        const i64 row0 = h * 128 + r;
        const i64 row = R0 + row0 < rows ? row0 : rows - 1 - R0;
        return row * ld + 8 * c;
    } else {
        const int kk = ins * 4 + (l >> 4);
        const int c = (l & 15) ^ swz_rc(kk);
        const i64 col0 = h * 128 + 8 * c;
        const i64 col = R0 + col0 <= rows - 8 ? col0 : rows - 8 - R0;
        return col + kk * ld;
    }
}

template <bool KC>
__device__ __forceinline__ const uint16_t* tile_base(const uint16_t* X, i64 ld, i64 R0, i64 k0) {
    return KC ? X + R0 * ld + k0 : X + R0 + k0 * ld;
}

// AUX: cache-policy bits of the DMA (0 = default; 17 = sc0 sc1, which hipBLASLt's
// kernels put on one operand's DirectToLds loads)
template <bool BUF, bool KC, int AUX = 0>
__device__ __forceinline__ void piece(const uint16_t* X, i64 ld, i64 R0, i64 k0, int off, i64 goff, int j,
                                      lds_char* img) {
    if constexpr (BUF) {
        const BufferSrc<uint16_t> src(tile_base<KC>(X, ld, R0, k0), (KC ? 256 : BK) * ld * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src.rs, (__attribute__((address_space(3))) void*)(img + j * 1024), 16,
                                                 off, 0, 0, AUX);
    } else {
        glds16(tile_base<KC>(X, ld, R0, k0) + goff, img + j * 1024);
    }
}

struct Sets {
    u32x4 a[8], b[8];
};

// acc += a b with the accumulator tied to one AGPR quad.  Written as asm: the
// builtin's accumulators get rotated through fresh registers (earlyclobber form)
// at 256 live accumulators, costing ~2 v_accvgpr moves per MFMA.  Only other
// MFMAs of the same accumulator read it inside the loop (accumulate chains need
// no wait states); the kernel pads before the epilogue's first read (settle).
template <bool BF16>
__device__ __forceinline__ void mfma_acc(f32x4& acc, const u32x4& a, const u32x4& b) {
    if constexpr (BF16) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// 8-pass MFMA result -> any non-MFMA reader: 12 wait states (then the registers
// are handed to the compiler through empty asm statements ordered after the pad)
__device__ __forceinline__ void settle(f32x4 (&acc)[8][8]) {
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) asm volatile("" : "+a"(acc[a][b]));
}

// C tile of one wave (128 x 128): accumulator (mi, ni) holds rows
// rb + 16 mi + 4 (l >> 4) + {0..3}, column cb + 16 ni + (l & 15).  One row of
// accumulators at a time (C loads, then stores), so at most 32 values live in
// VGPRs; interior tiles with an 8-B-aligned C take the unchecked path.
template <bool BF16>
__device__ __forceinline__ void epilogue4(const H2Params& p, const f32x4 (&acc)[8][8], i64 m0, i64 n0, int wr, int wc,
                                          int l) {
    using E = typename std::conditional<BF16, Elem<bf16_t>, Elem<f16_t>>::type;
    const i64 rb = m0 + wr * 128 + 4 * (l >> 4), cb = n0 + wc * 128 + (l & 15);
    const bool fast = p.vec_c && m0 + BM <= p.m && n0 + BN <= p.n;
    if (fast) {
        uint16_t* o0 = p.C + rb + cb * p.ldc;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
            uint2 cv[8];
#pragma unroll
            for (int ni = 0; ni < 8; ++ni)
                cv[ni] = p.beta != 0.f ? *reinterpret_cast<const uint2*>(o0 + mi * 16 + ni * 16 * p.ldc) : make_uint2(0, 0);
#pragma unroll
            for (int ni = 0; ni < 8; ++ni) {
                const uint16_t in[4] = {(uint16_t)(cv[ni].x & 0xffff), (uint16_t)(cv[ni].x >> 16),
                                        (uint16_t)(cv[ni].y & 0xffff), (uint16_t)(cv[ni].y >> 16)};
                uint16_t r16[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = p.alpha * acc[mi][ni][r];
                    if (p.beta != 0.f) v += p.beta * E::load(in[r]);
                    r16[r] = E::store(v);
                }
                *reinterpret_cast<uint2*>(o0 + mi * 16 + ni * 16 * p.ldc) =
                    make_uint2((uint32_t)r16[0] | ((uint32_t)r16[1] << 16), (uint32_t)r16[2] | ((uint32_t)r16[3] << 16));
            }
        }
    } else {
        epilogue<BF16, 8>(p, acc, m0, n0, wr, wc, l);
    }
}

struct Pieces {  // this wave's staging pieces w + 4u, u = 0..7, of each operand's image
    int offA[8], offB[8];
    i64 gA[8], gB[8];
};

// One k-step: 64 MFMAs on `cur`, the 16 fragments of k-step `srd` of the K-tile in
// (rdA, rdB) into `nxt`, and the 8 pieces of one unit (operand SB ? B : A at k0)
// into `st`.  The LDS pointers are __restrict__ so the inlined accesses carry
// alias scopes: hipcc's waitcnt pass then knows the in-flight DMA cannot alias
// the fragment reads (without them it drains vmcnt(0) before every
// ds_read_b64_tr_b16).
template <bool BF16, bool KCA, bool KCB, bool BUF, bool SB, int FL>
__device__ __forceinline__ void kstep(const H2Params& p, i64 m0, i64 n0, int w, int l, int wr, int wc,
                                      const Pieces& pc, const lds_char* __restrict__ rdA,
                                      const lds_char* __restrict__ rdB, int srd, lds_char* __restrict__ st, i64 k0,
                                      f32x4 (&acc)[8][8], const Sets& cur, Sets& nxt) {
    // Placement (measured, profiles/r03_h16_four_wave.log): the 16 fragment reads
    // of the next k-step go out in the first part of the k-step and the 8 staging
    // pieces in the second half, one per 4-MFMA group, in both k-steps: a piece
    // issued among the reads costs more MFMA time than the later landing of B_{t+2}
    // (issued in the second half of (t,1), read after (t+1,0)) costs in waiting.
    // Default: reads 1 per MFMA in groups 0-3 (+1-2 % over 2 per group in groups
    // 0-7, FL 128); FL 256: pieces in groups 5-12.
    constexpr int QB = (FL & 256) ? 5 : 8;
    constexpr int RPG = (FL & 128) ? 2 : 4;  // fragment reads per 4-MFMA group
#pragma unroll
    for (int q = 0; q < 16; ++q) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int mi = q >> 1, ni = (q & 1) * 4 + t;
            mfma_acc<BF16>(acc[mi][ni], cur.a[mi], cur.b[ni]);
            if (!(FL & 1) && t == 1 && q >= QB && q < QB + 8) {
                const int u = q - QB;
                if constexpr ((FL & 2048) != 0) {
                    if (u == 0) __builtin_amdgcn_s_setprio(3);
                }
                if constexpr (SB) piece<BUF, KCB, (FL & 1024) ? 17 : 0>(p.B, p.ldb, n0, k0, pc.offB[u], pc.gB[u], w + 4 * u, st);
                else piece<BUF, KCA, (FL & 512) ? 17 : 0>(p.A, p.lda, m0, k0, pc.offA[u], pc.gA[u], w + 4 * u, st);
                if constexpr ((FL & 2048) != 0) {
                    if (u == 7) __builtin_amdgcn_s_setprio(0);
                }
            }
            if constexpr (RPG == 4) {  // read f = 4q + t: A fragments 0-7, then B 0-7
                const int f = 4 * q + t;
                if (!(FL & 2) && f < 16) {
                    if (f < 8) nxt.a[f] = frag<KCA>(rdA + wr * HALF, f * 16, srd, l);
                    else nxt.b[f - 8] = frag<KCB>(rdB + wc * HALF, (f - 8) * 16, srd, l);
                }
            }
        }
        if (RPG == 2 && !(FL & 2) && q < 8) {
            nxt.a[q] = frag<KCA>(rdA + wr * HALF, q * 16, srd, l);
            nxt.b[q] = frag<KCB>(rdB + wc * HALF, q * 16, srd, l);
        }
    }
}
}  // namespace w4

// FL: timing ablations only (wrong results): 1 = no staging after the prologue,
// 2 = no fragment reads, 4 = no barrier, 32 = no wait for the staged K-tile;
// placement variants (correct): 128, 256 (kstep); 2048 = s_setprio 3 over the
// staging pieces of each k-step (hipBLASLt's loop raises the priority there; no
// gain); 512 / 1024 = A / B staged with the sc0 sc1 cache policy
template <bool BF16, bool KCA, bool KCB, bool BUF, int FL = 0>
__global__ __launch_bounds__(256, 1) void gemm_h4w_kernel(H2Params p) {
    using namespace w4;
    __shared__ __attribute__((aligned(1024))) char lds_raw[NSLOT * UNIT];
    lds_char* lds = (lds_char*)lds_raw;

    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 1, wc = w & 1;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;

    Pieces pc;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        pc.gA[u] = piece_off<KCA>(w + 4 * u, l, m0, p.m, p.lda);
        pc.gB[u] = piece_off<KCB>(w + 4 * u, l, n0, p.n, p.ldb);
        pc.offA[u] = (int)(pc.gA[u] * 2);
        pc.offB[u] = (int)(pc.gB[u] * 2);
    }

    f32x4 acc[8][8];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / BK);
    auto kt = [&](int t) { return (i64)min(t, nt - 1) * BK; };
    auto slot = [&](int u) { return lds + (u % NSLOT) * UNIT; };
    // prologue: A_0, B_0, A_1, B_1 into slots 0..3; wait for A_0, B_0; fragments (0,0)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int u = 0; u < 8; ++u) piece<BUF, KCA>(p.A, p.lda, m0, kt(t), pc.offA[u], pc.gA[u], w + 4 * u, lds + 2 * t * UNIT);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            piece<BUF, KCB>(p.B, p.ldb, n0, kt(t), pc.offB[u], pc.gB[u], w + 4 * u, lds + (2 * t + 1) * UNIT);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    bar8();
    Sets X, Y;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        X.a[q] = frag<KCA>(lds + wr * HALF, q * 16, 0, l);
        X.b[q] = frag<KCB>(lds + UNIT + wc * HALF, q * 16, 0, l);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // One K-tile; J = t % 5 makes every slot a compile-time offset of the LDS
    // base (the loop is unrolled by the ring length), so the fragment reads and
    // the DMA destinations need no address arithmetic in the loop.
    auto ktile = [&](auto jc, int t) {
        constexpr int J = decltype(jc)::value;
        constexpr int sA = 2 * J % NSLOT, sB = (2 * J + 1) % NSLOT, sA1 = (2 * J + 2) % NSLOT,
                      sB1 = (2 * J + 3) % NSLOT, st0 = (2 * J + 4) % NSLOT, st1 = (2 * J + 5) % NSLOT;
        // (t,0): stage A_{t+2} into B_{t-1}'s slot
        w4::kstep<BF16, KCA, KCB, BUF, false, FL>(p, m0, n0, w, l, wr, wc, pc, lds + sA * UNIT, lds + sB * UNIT, 1,
                                                 lds + st0 * UNIT, kt(t + 2), acc, X, Y);
        if constexpr (!(FL & 32)) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!(FL & 4)) bar8();
        // (t,1): stage B_{t+2} into A_t's slot
        w4::kstep<BF16, KCA, KCB, BUF, true, FL>(p, m0, n0, w, l, wr, wc, pc, lds + sA1 * UNIT, lds + sB1 * UNIT, 0,
                                                lds + st1 * UNIT, kt(t + 2), acc, Y, X);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    for (int t = 0; t < nt; t += NSLOT) {
        ktile(std::integral_constant<int, 0>{}, t);
        if (t + 1 < nt) ktile(std::integral_constant<int, 1>{}, t + 1);
        if (t + 2 < nt) ktile(std::integral_constant<int, 2>{}, t + 2);
        if (t + 3 < nt) ktile(std::integral_constant<int, 3>{}, t + 3);
        if (t + 4 < nt) ktile(std::integral_constant<int, 4>{}, t + 4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail pieces
    w4::settle(acc);
    w4::epilogue4<BF16>(p, acc, m0, n0, wr, wc, l);
}

// One 16 x 16 accumulator tile: rows i..i+15 (4 per lane), column j.
template <bool BF16>
__device__ __forceinline__ void epi_one(const H2Params& p, const f32x4 v4, i64 i, i64 j) {
    using E = typename std::conditional<BF16, Elem<bf16_t>, Elem<f16_t>>::type;
    if (j >= p.n || i >= p.m) return;
    uint16_t* o = p.C + i + j * p.ldc;
    if (p.vec_c && i + 3 < p.m) {
        uint2 cv = make_uint2(0, 0);
        if (p.beta != 0.f) cv = *reinterpret_cast<const uint2*>(o);
        const uint16_t in[4] = {(uint16_t)(cv.x & 0xffff), (uint16_t)(cv.x >> 16), (uint16_t)(cv.y & 0xffff),
                                (uint16_t)(cv.y >> 16)};
        uint16_t r16[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = p.alpha * v4[r];
            if (p.beta != 0.f) v += p.beta * E::load(in[r]);
            r16[r] = E::store(v);
        }
        *reinterpret_cast<uint2*>(o) = make_uint2((uint32_t)r16[0] | ((uint32_t)r16[1] << 16),
                                                  (uint32_t)r16[2] | ((uint32_t)r16[3] << 16));
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (i + r >= p.m) break;
            float v = p.alpha * v4[r];
            if (p.beta != 0.f) v += p.beta * E::load(o[r]);
            o[r] = E::store(v);
        }
    }
}

// every tile with compile-time indices (a fold, not a loop: a loop the unroller
// declines would index the accumulators dynamically and push them to scratch)
template <bool BF16, int NI, int... Q>
__device__ __forceinline__ void epilogue_seq(const H2Params& p, const f32x4 (&acc)[8][NI], i64 rb, i64 cb,
                                             std::integer_sequence<int, Q...>) {
    (epi_one<BF16>(p, acc[Q / NI][Q % NI], rb + (Q / NI) * 16, cb + (Q % NI) * 16), ...);
}

template <bool BF16, int NI>
__device__ __forceinline__ void epilogue(const H2Params& p, const f32x4 (&acc)[8][NI], i64 m0, i64 n0, int wr, int wc,
                                         int l) {
    const i64 rb = m0 + wr * 128 + 4 * (l >> 4), cb = n0 + wc * (16 * NI) + (l & 15);
    epilogue_seq<BF16, NI>(p, acc, rb, cb, std::make_integer_sequence<int, 8 * NI>{});
}

template <typename K>
hipError_t launch(K kernel, const H2Params& p, hipStream_t s) {
    hipLaunchKernelGGL(kernel, dim3(p.tiles_m * p.tiles_n), dim3(NT), 0, s, p);
    return hipGetLastError();
}

template <bool BF16, bool KCA, bool KCB, bool BUF>
hipError_t launch_p(const H2Params& p, hipStream_t s, int fl) {
    if constexpr (BF16 && KCA && KCB) {
        if (fl == 1) return launch(gemm_h8p_kernel<BF16, KCA, KCB, BUF, 1>, p, s);
        if (fl == 2) return launch(gemm_h8p_kernel<BF16, KCA, KCB, BUF, 2>, p, s);
        if (fl == 3) return launch(gemm_h8p_kernel<BF16, KCA, KCB, BUF, 3>, p, s);
        if (fl == 4) return launch(gemm_h8p_kernel<BF16, KCA, KCB, BUF, 4>, p, s);
    }
    return launch(gemm_h8p_kernel<BF16, KCA, KCB, BUF>, p, s);
}

// Kernel choice (launch_h256): four-wave (default, =w), deep-prefetch two-phase
// (=d), balanced-read (=b), phased (=p), two-stage (=s);
// ELX_H16_FLAGS picks a timing ablation (profiles/r01_h16_ablation.log) of the
// two-stage bf16 NN or phased bf16 TN kernel.
template <bool BF16, bool KCA, bool KCB>
hipError_t launch_h256(const H2Params& p, hipStream_t s) {
    // read per call (not cached) so tools/h16_ab.py can interleave kernel variants
    // in one process (cdna_hip_programming.md §5.4 rule 24); getenv is ~0.1 us
    const char* kv = getenv("ELX_H16_KERNEL");
    const char* fv = getenv("ELX_H16_FLAGS");
    const int fl = fv ? atoi(fv) : 0;
    const bool two_stage = kv && kv[0] == 's';
    // default (=w): the four-wave kernel (+1-3 % over the deep-prefetch kernel on
    // NN / TN / NT / TT at 16384^3 and 32768^3, profiles/r03_h16_four_wave.log);
    // =d the deep-prefetch two-phase kernel (+2-5 % over the balanced-read kernel,
    // profiles/r02_h16_deep.log); =b the balanced-read kernel
    // (profiles/r02_h16_experiments.log); =p the phased kernel (and its
    // ablations); =s the two-stage kernel
    const bool balanced = kv && kv[0] == 'b';
    const bool deep = kv && kv[0] == 'd';
    const bool four = !kv || kv[0] == 'w';
    if (four) {
        const bool buf = dma_fits(KCA ? 256 : BK, p.lda, 2) && dma_fits(KCB ? 256 : BK, p.ldb, 2);
        auto go = [&](auto kernel) {
            hipLaunchKernelGGL(kernel, dim3(p.tiles_m * p.tiles_n), dim3(256), 0, s, p);
            return hipGetLastError();
        };
        if constexpr (BF16 && KCB) {
            if (buf && fl == 1) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 1>);
            if (buf && fl == 2) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 2>);
            if (buf && fl == 3) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 3>);
            if (buf && fl == 128) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 128>);
            if (buf && fl == 256) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 256>);
            if (buf && fl == 2048) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 2048>);
            if (buf && fl == 512) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 512>);
            if (buf && fl == 1024) return go(gemm_h4w_kernel<BF16, KCA, KCB, true, 1024>);
        }
        return buf ? go(gemm_h4w_kernel<BF16, KCA, KCB, true>) : go(gemm_h4w_kernel<BF16, KCA, KCB, false>);
    }
    if (deep && fl == 0) {
        if (dma_fits(KCA ? 256 : BK, p.lda, 2) && dma_fits(KCB ? 256 : BK, p.ldb, 2))
            return launch(gemm_h4d_kernel<BF16, KCA, KCB, true>, p, s);
        return launch(gemm_h4d_kernel<BF16, KCA, KCB, false>, p, s);
    }
    if (balanced && fl == 0) {
        if (dma_fits(KCA ? 256 : BK, p.lda, 2) && dma_fits(KCB ? 256 : BK, p.ldb, 2))
            return launch(gemm_h8b_kernel<BF16, KCA, KCB, true>, p, s);
        return launch(gemm_h8b_kernel<BF16, KCA, KCB, false>, p, s);
    }
    if (two_stage) {
        if constexpr (BF16 && !KCA && KCB) {
            if (fl == 1) return launch(gemm_h256_kernel<BF16, KCA, KCB, 1>, p, s);
            if (fl == 2) return launch(gemm_h256_kernel<BF16, KCA, KCB, 2>, p, s);
            if (fl == 3) return launch(gemm_h256_kernel<BF16, KCA, KCB, 3>, p, s);
            if (fl == 8) return launch(gemm_h256_kernel<BF16, KCA, KCB, 8>, p, s);
        }
        return launch(gemm_h256_kernel<BF16, KCA, KCB>, p, s);
    }
    static const bool global_only = [] { const char* v = getenv("ELX_H16_STAGE"); return v && v[0] == 'g'; }();
    if (!global_only && dma_fits(KCA ? 256 : BK, p.lda, 2) && dma_fits(KCB ? 256 : BK, p.ldb, 2))
        return launch_p<BF16, KCA, KCB, true>(p, s, fl);
    return launch_p<BF16, KCA, KCB, false>(p, s, fl);
}

bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

bool four_wave() {
    const char* v = getenv("ELX_H16_KERNEL");
    return !v || v[0] == 'w';
}

// Tile-order group height (per call, like the kernel knobs: tools/h16_ab.py).
// Default 8 for the eight-wave kernels; 4 for the four-wave kernel, whose 32
// concurrent tiles per XCD then span 4 x 8 tiles (+1-3 % over 8 x 4 at 32768^3
// and 16384^3, profiles/r03_h16_four_wave.log).
int GroupM(bool four) {
    // clamped to >= 1: tile_of divides by it, and a zero group height ("", "0")
    // would map workgroups to tiles far outside the operands (an illegal-address
    // fault, which is how tools/h16_ab.py's "KERNEL:FLAGS" specs once passed 0)
    const char* v = getenv("ELX_H16_GROUP");
    const int g = v ? atoi(v) : four ? 4 : GROUP_M;
    return g >= 1 ? g : 1;
}

}  // namespace

#ifndef ELX_KERNEL_PROBE
hipError_t gemm_mfma_h(bool is_bf16, bool ta, bool tb, i64 m, i64 n, i64 k, float alpha, const uint16_t* A,
                       i64 lda, const uint16_t* B, i64 ldb, float beta, uint16_t* C, i64 ldc, hipStream_t s) {
    const bool kca = ta, kcb = !tb;
    // (a 4-slot BK = 32 ring with 3 K-tiles in flight measured 5-10 % slower:
    //  profiles/r01_h16_ring_ab.log)
    const i64 kmain = k / BK * BK;
    // the large-tile path: 16-B aligned rows/columns for glds, RC operands a
    // multiple of 8 long (whole 16-B chunks), and enough tiles to fill the chip
    const bool ok = kmain > 0 && al16(A) && al16(B) && lda % 8 == 0 && ldb % 8 == 0 &&
                    (kca || (m % 8 == 0 && m >= 8)) && (kcb || (n % 8 == 0 && n >= 8)) &&
                    ((m + BM - 1) / BM) * ((n + BN - 1) / BN) >= 64 && m < (1ll << 31) && n < (1ll << 31);
    if (!ok) return gemm_mfma_h_simple(is_bf16, ta, tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
    H2Params p{m, n, kmain, alpha, beta, A, lda, B, ldb, C, ldc, (int)((m + BM - 1) / BM), (int)((n + BN - 1) / BN),
               (reinterpret_cast<uintptr_t>(C) & 7) == 0 && ldc % 4 == 0, GroupM(four_wave())};
    hipError_t e;
    if (is_bf16) {
        if (kca) e = kcb ? launch_h256<true, true, true>(p, s) : launch_h256<true, true, false>(p, s);
        else e = kcb ? launch_h256<true, false, true>(p, s) : launch_h256<true, false, false>(p, s);
    } else {
        if (kca) e = kcb ? launch_h256<false, true, true>(p, s) : launch_h256<false, true, false>(p, s);
        else e = kcb ? launch_h256<false, false, true>(p, s) : launch_h256<false, false, false>(p, s);
    }
    if (e != hipSuccess || kmain == k) return e;
    // k tail (< 64): C += alpha op(A)(:, kmain:) op(B)(kmain:, :)
    const uint16_t* At = ta ? A + kmain : A + kmain * lda;
    const uint16_t* Bt = tb ? B + kmain * ldb : B + kmain;
    return gemm_mfma_h_simple(is_bf16, ta, tb, m, n, k - kmain, alpha, At, lda, Bt, ldb, 1.0f, C, ldc, s);
}

#endif  // ELX_KERNEL_PROBE

}  // namespace kern
}  // namespace elx
