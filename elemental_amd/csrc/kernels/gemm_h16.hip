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
//  * 256 x 256 output tile per 256-thread workgroup: four waves (2 x 2), one
//    per SIMD, each 128 x 128 = 8 x 8 accumulators of
//    v_mfma_f32_16x16x32_{bf16,f16}; BK = 64 per K-tile, one workgroup per CU.
//  * Operands are staged HBM -> LDS with LDS DMA (buffer_load ... lds, 16 B per
//    lane, no VGPR round trip) into a five-slot ring (below).
//  * Every orientation reads through the same two LDS image kinds:
//      KC (k contiguous in HBM: op(A) = A^T, op(B) = B): rows of 64 k = 128 B,
//         read with ds_read_b128 straight into the MFMA fragment;
//      RC (rows contiguous: op(A) = A, op(B) = B^T): k-rows of 128 elements
//         = 256 B, read with the gfx950 transposing ds_read_b64_tr_b16 (two
//         per fragment), so no transpose pass and no extra HBM traffic.
//    Both images are XOR-swizzled on the 16-B chunk index so the fragment
//    reads are bank-conflict-free; the swizzle is applied to the GLOBAL source
//    address of each DMA lane (the LDS side of the DMA is lane-linear).
//  * XCD-aware bijective workgroup remap with grouped tile order (tile_of).
// History: the round-1/2 eight-wave kernels (two-stage, phased, balanced-read,
// deep-prefetch) lived here behind ELX_H16_KERNEL until round 4; their
// measurements are in profiles/r01_gemm16_h256.log, r01_h16_ablation.log,
// r02_h16_deep.log and r03_h16_four_wave.log (the four-wave kernel beat each).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
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


constexpr int BK = 64;
constexpr int HALF = 128 * BK * 2;  // one RC half image: 64 k-rows x 128 operand rows x 2 B = 16 KiB

struct H2Params {
    i64 m, n, k;  // k: multiple of BK
    float alpha, beta;
    const uint16_t* A; i64 lda;
    const uint16_t* B; i64 ldb;
    uint16_t* C; i64 ldc;
    int tiles_m, tiles_n;
    int vec_c;    // C base 8-B aligned and ldc % 4 == 0
    int group_m;  // tile-order group height (ELX_H16_GROUP, default 8)
    int sblock;   // 1: super-block order (tile_of_sb); needs the grid to be whole super-blocks
    int sb_xr, sb_pr;  // its geometry
    // split-k (gridDim.y chunks, W != null): chunk z covers k in [z*kchunk,
    // min(k, (z+1)*kchunk)) and writes its raw f32 product to W + z*m*n (ld m);
    // h16_splitk_reduce applies alpha / beta and rounds once
    i64 kchunk;
    float* W;
    // > 0: launch only the first dp_tiles tiles of the tile order (the
    // data-parallel rounds of gemm_mfma_h's tail split); 0: every tile
    int dp_tiles;
    // k beyond the last whole K-tile (0..63), added by the workgroup after its
    // K-tile loop, before the one rounding (split-k: by the last chunk)
    int ktail;
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

// Super-block order: the 256 workgroups that run at once (one per CU) cover one
// 16 x 16 block of tiles, each XCD an 8 x 4 part of it (bid & 7 is the XCD a
// workgroup is dispatched to, bid >> 3 its turn there: 32 at a time).  An XCD's
// L2 sees the same 8 + 4 operand slices per K-tile as in tile_of's grouped
// order, but the eight XCDs now read 16 A and 16 B slices between them instead
// of 64 A and 4 B, so the Infinity Cache serves what one XCD fetched to the
// others and HBM reads less per launch.
// Geometry: the XCDs form an xr x (8 / xr) grid of parts of pr x (32 / pr)
// tiles each (default 2 x 4 parts of 8 x 4).
__device__ __forceinline__ void tile_of_sb(int bid, int tiles_n, int xr, int pr, int& tm, int& tn) {
    const int xcd = bid & 7, i = bid >> 3, r = i >> 5, s = i & 31;
    const int pc = 32 / pr, sbr = xr * pr, sbc = (8 / xr) * pc;
    const int sbn = tiles_n / sbc;
    tm = (r / sbn) * sbr + (xcd % xr) * pr + (s % pr);
    tn = (r % sbn) * sbc + (xcd / xr) * pc + (s / pr);
}

// XOR swizzles (16-B chunk index).  KC: 8 chunks per 128-B row, row r -> c ^ ((r>>1)&7):
// the 16 lanes of a ds_read_b128 group (rows r..r+15 of one or two k-chunks) land
// on 16 distinct 16-B bank slots.  RC: 16 chunks per 256-B k-row, k-row kk ->
// c ^ (2(kk&3) + 8((kk>>3)&1)): the 8 k-rows x 32 B a 32-lane half of a
// ds_read_b64_tr_b16 touches land on distinct bank slots; XOR values are even,
// so the two chunks of a 32-B column pair stay adjacent.
__device__ __forceinline__ int swz_kc(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int swz_rc(int kk) { return ((kk & 3) << 1) | (((kk >> 3) & 1) << 3); }
// RC images of 64-column blocks (the last block of a 192-row tile): 8 chunks per
// 128-B k-row, k-row kk -> c ^ (2((kk>>1)&1) + 4((kk>>3)&1)).  A 32-lane half of
// ds_read_b64_tr_b16 touches k-rows b + {0,1,2,3,8,9,10,11} (b a multiple of 4),
// 32 B each; a 128-B pitch puts odd k-rows in the upper half of a 256-B bank row,
// and within each parity the four k-rows get the four even XOR values, so the 16
// chunk slots are distinct.
__device__ __forceinline__ int swz_rc8(int kk) { return (((kk >> 1) & 1) << 1) | (((kk >> 3) & 1) << 2); }
// RC images of 32-column blocks (the last block of a 160- or 224-row tile): 4
// chunks per 64-B k-row, k-row kk -> c ^ 2((kk>>3)&1).  The same half-wave's
// eight k-rows fall four to a bank row (kk & 3 picks the 64-B quarter), and the
// two that share a quarter (kk, kk + 8) get different chunk pairs.
__device__ __forceinline__ int swz_rc4(int kk) { return ((kk >> 3) & 1) << 1; }

__device__ __forceinline__ void glds16(const uint16_t* src, lds_char* dst) {
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// One MFMA operand fragment (16 operand rows from R0, k-step s of 32):
// lane l holds X(R0 + (l&15), 32s + 8(l>>4) + j), j = 0..7.  RC: `narrow`
// selects the block kind: 0 = 128 columns (256-B k-rows, swz_rc), 1 = 64
// columns (128-B k-rows, swz_rc8), 2 = 32 columns (64-B k-rows, swz_rc4).
template <bool KC>
__device__ __forceinline__ u32x4 frag(const lds_char* img, int R0, int s, int l, int narrow = 0) {
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
            const lds_char* a = narrow == 0   ? img + kk * 256 + ((c ^ swz_rc(kk)) << 4) + ((p & 1) << 3)
                                : narrow == 1 ? img + kk * 128 + ((c ^ swz_rc8(kk)) << 4) + ((p & 1) << 3)
                                              : img + kk * 64 + ((c ^ swz_rc4(kk)) << 4) + ((p & 1) << 3);
            const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
            const u32x2 u = __builtin_bit_cast(u32x2, v);
            out[2 * h] = u[0];
            out[2 * h + 1] = u[1];
        }
        return out;
    }
}

// (wait_cnt: lds_dma.hpp)

__device__ __forceinline__ void bar8() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
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
template <bool BF16, int MI, int NI, int... Q>
__device__ __forceinline__ void epilogue_seq(const H2Params& p, const f32x4 (&acc)[MI][NI], i64 rb, i64 cb,
                                             std::integer_sequence<int, Q...>) {
    (epi_one<BF16>(p, acc[Q / NI][Q % NI], rb + (Q / NI) * 16, cb + (Q % NI) * 16), ...);
}

// wave (wr, wc) owns rows m0 + wr * 16 MI .. and columns n0 + wc * 16 NI ..
template <bool BF16, int MI, int NI>
__device__ __forceinline__ void epilogue(const H2Params& p, const f32x4 (&acc)[MI][NI], i64 m0, i64 n0, int wr, int wc,
                                         int l) {
    const i64 rb = m0 + wr * (16 * MI) + 4 * (l >> 4), cb = n0 + wc * (16 * NI) + (l & 15);
    epilogue_seq<BF16, MI, NI>(p, acc, rb, cb, std::make_integer_sequence<int, MI * NI>{});
}

// Four-wave kernel: a 256 x 256 output tile over 4 waves (2 x 2), one per
// SIMD, each owning 128 x 128 = 8 x 8 accumulators (256 AGPRs; the wave has the
// whole 512-entry file).  Per FLOP this halves the B-fragment LDS reads of the
// eight-wave kernels (a wave's fragments feed 8 x 8 MFMAs instead of 8 x 4), cuts
// a third of all LDS instructions, and leaves no partner wave on the SIMD to take
// matrix-pipe slots or issue bandwidth (MI355X_MICROARCH.md "Two waves per SIMD"
// items 1-3): each wave issues its own fragment reads and staging between its
// MFMAs.  hipBLASLt's bf16 kernels on these shapes have the same geometry
// (MT256x256x64, MI16x16, 4 waves: profiles/r03_vendor_pmc.json).
//
// The same loop at half the tile (WM = 4: 128 x 128 per workgroup, 64 x 64 =
// 4 x 4 accumulators per wave, 80 KiB of ring, two workgroups per CU) serves the
// grids on which 256 x 256 tiles leave CUs idle (fewer than 256 of them: 2048^3
// has 64, i.e. a quarter of the chip).  Round 5.  Round 6 adds WM = 6 / 5 / 7
// (192 / 160 / 224 tiles, one workgroup per CU) for grids those edges fill in
// whole rounds, and WM = 2 (64 x 64, 2 x 2 accumulators per wave, 40 KiB of
// ring, four workgroups per CU) for small grids; h16_plan (kernels.hpp) picks
// the tile.
//
// Staging unit = one operand's K-tile image (BM rows x 64 k: 32 KiB at WM = 8,
// 16 KiB at WM = 4; the KC / RC images: 128-B KC rows, or 256-B RC k-rows in
// 128-row halves), in a ring of 5 slots: A_t is unit 2t, B_t unit 2t+1, unit u
// in slot u % 5.  A unit is 4 WM one-KiB pieces, WM per wave.  Each K-tile runs
// as two k-steps of WM^2 MFMAs per wave:
//   (t,0): MFMAs on fragments (t,0) [set X]; read fragments (t,1) [set Y] from
//          A_t, B_t; stage A_{t+2} into B_{t-1}'s slot; then vmcnt(WM) (A_{t+1}
//          and B_{t+1} landed, A_{t+2} may stay in flight), lgkmcnt(0), barrier;
//   (t,1): MFMAs on (t,1) [Y]; read (t+1,0) [X] from A_{t+1}, B_{t+1}; stage
//          B_{t+2} into A_t's slot; lgkmcnt(0), no barrier.
// RAW: A_{t+1}, B_{t+1} are read from (t,1) on, after every wave's wait and the
// barrier ending (t,0).  WAR: A_t's and B_t's last reads are issued in (t,0) and
// retired before that barrier; their slots are restaged in (t,1) and (t+1,0).
// No wave can be two k-steps ahead of another (it would have passed a barrier
// the other has not reached), so one barrier per K-tile suffices.  Units past
// the end re-stage the last K-tile into a slot nobody reads again, so every
// k-step issues the same WM pieces and the counted wait is exact without branches.
// The accumulators are tied to AGPRs through inline asm (mfma_acc).
// ---------------------------------------------------------------------------
namespace w4 {
constexpr int NSLOT = 5;
template <int WM> struct Geo {
    static constexpr int BM = 32 * WM;           // tile edge (rows of op(A), columns of op(B))
    static constexpr int UNIT = BM * BK * 2;     // one operand's K-tile image
    static constexpr int WROWS = 16 * WM;        // operand rows one wave reads
    // RC images: BM / 128 blocks of 128 columns (256-B k-rows, HALF bytes
    // each), then a block of 64 columns (128-B k-rows, 8 KiB) if BM % 128 >= 64,
    // then one of 32 columns (64-B k-rows, 4 KiB) if BM % 64 == 32: WM 8 / 4 =
    // 128-blocks only, WM 6 = 128 + 64, WM 5 = 128 + 32, WM 7 = 128 + 64 + 32
    static constexpr int RCFULL = BM / 128;
    static constexpr bool RC64 = (BM % 128) >= 64, RC32 = (BM % 64) == 32;
    static constexpr int C64 = 128 * RCFULL, C32 = C64 + (RC64 ? 64 : 0);       // first column of each
    static constexpr int J64 = 16 * RCFULL, J32 = J64 + (RC64 ? 8 : 0);          // first piece of each
    static constexpr int O64 = RCFULL * HALF, O32 = O64 + (RC64 ? HALF / 2 : 0);  // byte offset of each
};

// per-lane offset (elements from the image's corner at k0) of piece j of one
// operand's K-tile image, as the image is laid out: KC rows 8j..8j+7 (128 B
// each); RC k-rows 4(j & 15)..+3 of the 128-column block j >> 4, or, in a
// 64-column block (WM 6, 7), k-rows 8i..8i+7 of it (i = j - J64), or, in a
// 32-column block (WM 5, 7), k-rows 16i..16i+15 (i = j - J32)
template <int WM, bool KC>
__device__ __forceinline__ i64 piece_off(int j, int l, i64 R0, i64 rows, i64 ld) {
    const int h = j >> 4, ins = j & 15;
    if (KC) {
        const int r = ins * 8 + (l >> 3);
        const int c = (l & 7) ^ swz_kc(r);
        const i64 row0 = h * 128 + r;
        const i64 row = R0 + row0 < rows ? row0 : rows - 1 - R0;
        return row * ld + 8 * c;
    } else {
        using G = Geo<WM>;
        int kk, c;
        i64 col0;
        if (G::RC32 && j >= G::J32) {  // 32-column block: 16 k-rows x 64 B per piece
            kk = (j - G::J32) * 16 + (l >> 2);
            c = (l & 3) ^ swz_rc4(kk);
            col0 = G::C32 + 8 * c;
        } else if (G::RC64 && j >= G::J64) {  // 64-column block: 8 k-rows x 128 B
            kk = (j - G::J64) * 8 + (l >> 3);
            c = (l & 7) ^ swz_rc8(kk);
            col0 = G::C64 + 8 * c;
        } else {
            kk = ins * 4 + (l >> 4);
            c = (l & 15) ^ swz_rc(kk);
            col0 = h * 128 + 8 * c;
        }
        const i64 col = R0 + col0 <= rows - 8 ? col0 : rows - 8 - R0;
        return col + kk * ld;
    }
}

// the same offsets for the k-tail K-tile (ktail < 64 valid k): k-rows (RC) past
// the tail are clamped to its last one, 16-B k-chunks (KC) past it to chunk 0
// (with a k-contiguous operand the host takes the in-kernel tail only for
// ktail % 8 == 0, so no chunk straddles it and nothing is read past k).  The
// values read for k >= ktail are zeroed in the fragments before use.
template <int WM, bool KC>
__device__ __forceinline__ i64 piece_off_tail(int j, int l, i64 R0, i64 rows, i64 ld, int ktail) {
    const i64 o = piece_off<WM, KC>(j, l, R0, rows, ld);
    if (KC) {
        const i64 kin = o % ld;  // 8 c: the chunk's first k
        return kin < ktail ? o : o - kin;
    }
    const i64 kk = o / ld;
    return kk < ktail ? o : o - (kk - (ktail - 1)) * ld;
}

template <bool KC>
__device__ __forceinline__ const uint16_t* tile_base(const uint16_t* X, i64 ld, i64 R0, i64 k0) {
    return KC ? X + R0 * ld + k0 : X + R0 + k0 * ld;
}

template <int BMR, bool BUF, bool KC>
__device__ __forceinline__ void piece(const uint16_t* X, i64 ld, i64 R0, i64 k0, int off, i64 goff, int j,
                                      lds_char* img) {
    if constexpr (BUF) {
        const BufferSrc<uint16_t> src(tile_base<KC>(X, ld, R0, k0), (KC ? BMR : BK) * ld * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src.rs, (__attribute__((address_space(3))) void*)(img + j * 1024), 16,
                                                 off, 0, 0, 0);
    } else {
        glds16(tile_base<KC>(X, ld, R0, k0) + goff, img + j * 1024);
    }
}

// a wave's operand fragment f (16 rows) of k-step s: KC images are one block of
// 128-B rows; RC images are 128-column blocks (then a 64- and / or a
// 32-column one, Geo), so a wave's rows may start inside one
template <int WM, bool KC>
__device__ __forceinline__ u32x4 wfrag(const lds_char* img, int w_r, int f, int s, int l) {
    constexpr int WR = Geo<WM>::WROWS;
    const int r0 = w_r * WR + f * 16;
    if constexpr (KC) {
        return frag<true>(img, r0, s, l);
    } else {
        using G = Geo<WM>;
        if (G::RC32 && r0 >= G::C32) return frag<false>(img + G::O32, r0 - G::C32, s, l, 2);
        if (G::RC64 && r0 >= G::C64) return frag<false>(img + G::O64, r0 - G::C64, s, l, 1);
        return frag<false>(img + (r0 >> 7) * HALF, r0 & 127, s, l, 0);
    }
}

template <int WM>
struct Sets {
    u32x4 a[WM], b[WM];
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
template <int WM>
__device__ __forceinline__ void settle(f32x4 (&acc)[WM][WM]) {
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WM; ++b) asm volatile("" : "+a"(acc[a][b]));
}

// Split-k partial of one wave: the raw f32 accumulators into W (ld m)
template <int WM>
__device__ __forceinline__ void epilogue_partial(const H2Params& p, const f32x4 (&acc)[WM][WM], i64 m0, i64 n0,
                                                 int wr, int wc, int l) {
    const i64 rb = m0 + wr * (16 * WM) + 4 * (l >> 4), cb = n0 + wc * (16 * WM) + (l & 15);
    const bool vec = (p.m & 3) == 0;
#pragma unroll
    for (int mi = 0; mi < WM; ++mi)
#pragma unroll
        for (int ni = 0; ni < WM; ++ni) {
            const i64 i = rb + mi * 16, j = cb + ni * 16;
            if (j >= p.n || i >= p.m) continue;
            float* o = p.W + i + j * p.m;
            if (vec) {
                *reinterpret_cast<f32x4*>(o) = acc[mi][ni];
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (i + r < p.m) o[r] = acc[mi][ni][r];
            }
        }
}

// C = alpha sum_z W_z + beta C, rounded once to the 16-bit type
template <bool BF16>
__global__ __launch_bounds__(256) void h16_splitk_reduce(i64 m, i64 n, int nz, float alpha, const float* __restrict__ W,
                                                         float beta, uint16_t* __restrict__ C, i64 ldc) {
    using E = typename std::conditional<BF16, Elem<bf16_t>, Elem<f16_t>>::type;
    const i64 mn = m * n;
    for (i64 e = (i64)blockIdx.x * 256 + threadIdx.x; e < mn; e += (i64)gridDim.x * 256) {
        float v = 0.f;
        for (int z = 0; z < nz; ++z) v += W[z * mn + e];
        const i64 i = e % m, j = e / m;
        uint16_t* o = C + i + j * ldc;
        v *= alpha;
        if (beta != 0.f) v += beta * E::load(*o);
        *o = E::store(v);
    }
}

// The same sum, four rows of one column per thread (16-B partial loads, 8-B C
// accesses; m % 4 == 0, C 8-B aligned, ldc % 4 == 0): grid (ceil(m / 1024), n).
// Same order of additions (W_0 + W_1 + ...), so the same bits.
template <bool BF16>
__global__ __launch_bounds__(256) void h16_splitk_reduce4(i64 m, i64 n, int nz, float alpha,
                                                          const float* __restrict__ W, float beta,
                                                          uint16_t* __restrict__ C, i64 ldc) {
    using E = typename std::conditional<BF16, Elem<bf16_t>, Elem<f16_t>>::type;
    const i64 i = ((i64)blockIdx.x * 256 + threadIdx.x) * 4, j = blockIdx.y;
    if (i >= m) return;
    const i64 mn = m * n;
    const float* w = W + j * m + i;
    f32x4 v = *reinterpret_cast<const f32x4*>(w);
    for (int z = 1; z < nz; ++z) v += *reinterpret_cast<const f32x4*>(w + z * mn);
    uint16_t* o = C + i + j * ldc;
    uint2 cv = make_uint2(0, 0);
    if (beta != 0.f) cv = *reinterpret_cast<const uint2*>(o);
    const uint16_t in[4] = {(uint16_t)(cv.x & 0xffff), (uint16_t)(cv.x >> 16), (uint16_t)(cv.y & 0xffff),
                            (uint16_t)(cv.y >> 16)};
    uint16_t r16[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float x = v[r] * alpha;
        if (beta != 0.f) x += beta * E::load(in[r]);
        r16[r] = E::store(x);
    }
    *reinterpret_cast<uint2*>(o) = make_uint2((uint32_t)r16[0] | ((uint32_t)r16[1] << 16),
                                              (uint32_t)r16[2] | ((uint32_t)r16[3] << 16));
}

// C tile of one wave (16 WM x 16 WM): accumulator (mi, ni) holds rows
// rb + 16 mi + 4 (l >> 4) + {0..3}, column cb + 16 ni + (l & 15).  One row of
// accumulators at a time (C loads, then stores), so at most 4 WM values live in
// VGPRs; interior tiles with an 8-B-aligned C take the unchecked path.
template <bool BF16, int WM>
__device__ __forceinline__ void epilogue4(const H2Params& p, const f32x4 (&acc)[WM][WM], i64 m0, i64 n0, int wr,
                                          int wc, int l) {
    using E = typename std::conditional<BF16, Elem<bf16_t>, Elem<f16_t>>::type;
    constexpr int BM = Geo<WM>::BM;
    const i64 rb = m0 + wr * (16 * WM) + 4 * (l >> 4), cb = n0 + wc * (16 * WM) + (l & 15);
    const bool fast = p.vec_c && m0 + BM <= p.m && n0 + BM <= p.n;
    if (fast) {
        uint16_t* o0 = p.C + rb + cb * p.ldc;
#pragma unroll
        for (int mi = 0; mi < WM; ++mi) {
            uint2 cv[WM];
#pragma unroll
            for (int ni = 0; ni < WM; ++ni)
                cv[ni] = p.beta != 0.f ? *reinterpret_cast<const uint2*>(o0 + mi * 16 + ni * 16 * p.ldc) : make_uint2(0, 0);
#pragma unroll
            for (int ni = 0; ni < WM; ++ni) {
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
        epilogue<BF16, WM, WM>(p, acc, m0, n0, wr, wc, l);
    }
}

template <int WM>
struct Pieces {  // this wave's staging pieces w + 4u, u = 0..WM-1, of each operand's image
    int offA[WM], offB[WM];
    i64 gA[WM], gB[WM];
};

// One k-step: WM^2 MFMAs on `cur`, the 2 WM fragments of k-step `srd` of the
// K-tile in (rdA, rdB) into `nxt`, and the WM pieces of one unit (operand SB ? B
// : A at k0) into `st`.  The LDS pointers are __restrict__ so the inlined
// accesses carry alias scopes: hipcc's waitcnt pass then knows the in-flight DMA
// cannot alias the fragment reads (without them it drains vmcnt(0) before every
// ds_read_b64_tr_b16).
template <int WM, bool BF16, bool KCA, bool KCB, bool BUF, bool SB>
__device__ __forceinline__ void kstep(const H2Params& p, i64 m0, i64 n0, int w, int l, int wr, int wc,
                                      const Pieces<WM>& pc, const lds_char* __restrict__ rdA,
                                      const lds_char* __restrict__ rdB, int srd, lds_char* __restrict__ st, i64 k0,
                                      f32x4 (&acc)[WM][WM], const Sets<WM>& cur, Sets<WM>& nxt) {
    constexpr int BMR = Geo<WM>::BM;
    // Placement (measured at WM = 8, profiles/r03_h16_four_wave.log): the 2 WM
    // fragment reads of the next k-step go out one per MFMA in the first 2 WM
    // MFMAs, the WM staging pieces evenly over the second half of the k-step's
    // MFMAs: a piece issued among the reads costs more MFMA time than the later
    // landing of B_{t+2} (issued in the second half of (t,1), read after
    // (t+1,0)) costs in waiting.
    constexpr int NM = WM * WM, GAP = WM / 2;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        mfma_acc<BF16>(acc[i / WM][i % WM], cur.a[i / WM], cur.b[i % WM]);
        if (i >= NM / 2 && (i - NM / 2) % GAP == 1 % GAP && (i - NM / 2) / GAP < WM) {
            const int u = (i - NM / 2) / GAP;
            if constexpr (SB) piece<BMR, BUF, KCB>(p.B, p.ldb, n0, k0, pc.offB[u], pc.gB[u], w + 4 * u, st);
            else piece<BMR, BUF, KCA>(p.A, p.lda, m0, k0, pc.offA[u], pc.gA[u], w + 4 * u, st);
        }
        if (i < 2 * WM) {  // read i: A fragments 0..WM-1, then B
            if (i < WM) nxt.a[i] = wfrag<WM, KCA>(rdA, wr, i, srd, l);
            else nxt.b[i - WM] = wfrag<WM, KCB>(rdB, wc, i - WM, srd, l);
        }
    }
}
}  // namespace w4

// PART: split-k partials (p.W, gridDim.y chunks), a separate instantiation so the
// default kernel's epilogue keeps its register allocation.  WM = 8: one
// workgroup per CU (the whole register file and LDS); WM = 4: two.
// SWP: B is the operand of the even units (staged first in a K-tile, one k-step
// more DMA lead), A of the odd ones.
template <int WM, bool BF16, bool KCA, bool KCB, bool BUF, bool PART, bool SWP = false>
__global__ __launch_bounds__(256, WM >= 5 ? 1 : WM >= 4 ? 2 : 4) void gemm_h4w_kernel(H2Params p) {
    using namespace w4;
    constexpr int BMR = Geo<WM>::BM, UNIT = Geo<WM>::UNIT;
    __shared__ __attribute__((aligned(1024))) char lds_raw[NSLOT * UNIT];
    lds_char* lds = (lds_char*)lds_raw;

    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 1, wc = w & 1;
    int tm, tn;
    if (p.sblock) tile_of_sb(blockIdx.x, p.tiles_n, p.sb_xr, p.sb_pr, tm, tn);
    else tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
    const i64 m0 = (i64)tm * BMR, n0 = (i64)tn * BMR;
    if constexpr (PART) {  // this workgroup's k chunk
        const i64 kz0 = (i64)blockIdx.y * p.kchunk;
        p.k = min(p.kchunk, p.k - kz0);
        p.A += KCA ? kz0 : kz0 * p.lda;
        p.B += KCB ? kz0 : kz0 * p.ldb;
        p.W += (i64)blockIdx.y * p.m * p.n;
    }

    Pieces<WM> pc;
#pragma unroll
    for (int u = 0; u < WM; ++u) {
        pc.gA[u] = piece_off<WM, KCA>(w + 4 * u, l, m0, p.m, p.lda);
        pc.gB[u] = piece_off<WM, KCB>(w + 4 * u, l, n0, p.n, p.ldb);
        pc.offA[u] = (int)(pc.gA[u] * 2);
        pc.offB[u] = (int)(pc.gB[u] * 2);
    }

    f32x4 acc[WM][WM];
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WM; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

    const int nt = (int)(p.k / BK);
    auto kt = [&](int t) { return (i64)min(t, nt - 1) * BK; };
    // prologue: A_0, B_0, A_1, B_1 into slots 0..3; wait for A_0, B_0; fragments (0,0)
    constexpr int OA = SWP ? 1 : 0, OB = SWP ? 0 : 1;  // unit parity of A / B
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        if constexpr (SWP) {
#pragma unroll
            for (int u = 0; u < WM; ++u)
                piece<BMR, BUF, KCB>(p.B, p.ldb, n0, kt(t), pc.offB[u], pc.gB[u], w + 4 * u, lds + (2 * t + OB) * UNIT);
        }
#pragma unroll
        for (int u = 0; u < WM; ++u)
            piece<BMR, BUF, KCA>(p.A, p.lda, m0, kt(t), pc.offA[u], pc.gA[u], w + 4 * u, lds + (2 * t + OA) * UNIT);
        if constexpr (!SWP) {
#pragma unroll
            for (int u = 0; u < WM; ++u)
                piece<BMR, BUF, KCB>(p.B, p.ldb, n0, kt(t), pc.offB[u], pc.gB[u], w + 4 * u, lds + (2 * t + OB) * UNIT);
        }
    }
    wait_cnt<2 * WM, NOWAIT_LGKM>();
    bar8();
    Sets<WM> X, Y;
#pragma unroll
    for (int q = 0; q < WM; ++q) {
        X.a[q] = wfrag<WM, KCA>(lds + OA * UNIT, wr, q, 0, l);
        X.b[q] = wfrag<WM, KCB>(lds + OB * UNIT, wc, q, 0, l);
    }
    wait_cnt<NOWAIT_VM, 0>();
    // One K-tile; J = t % 5 makes every slot a compile-time offset of the LDS
    // base (the loop is unrolled by the ring length), so the fragment reads and
    // the DMA destinations need no address arithmetic in the loop.
    auto ktile = [&](auto jc, int t) {
        constexpr int J = decltype(jc)::value;
        constexpr int sA = (2 * J + OA) % NSLOT, sB = (2 * J + OB) % NSLOT, sA1 = (2 * J + 2 + OA) % NSLOT,
                      sB1 = (2 * J + 2 + OB) % NSLOT, st0 = (2 * J + 4) % NSLOT, st1 = (2 * J + 5) % NSLOT;
        // (t,0): stage the even unit of t+2 (A_{t+2}; B_{t+2} if SWP) into the odd
        // unit of t-1's slot
        w4::kstep<WM, BF16, KCA, KCB, BUF, SWP>(p, m0, n0, w, l, wr, wc, pc, lds + sA * UNIT, lds + sB * UNIT, 1,
                                                   lds + st0 * UNIT, kt(t + 2), acc, X, Y);
        wait_cnt<WM, 0>();
        bar8();
        // (t,1): stage the odd unit of t+2 into the even unit of t's slot
        w4::kstep<WM, BF16, KCA, KCB, BUF, !SWP>(p, m0, n0, w, l, wr, wc, pc, lds + sA1 * UNIT, lds + sB1 * UNIT, 0,
                                                    lds + st1 * UNIT, kt(t + 2), acc, Y, X);
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
    // The k tail (< 64 k past the last whole K-tile), in the same accumulators so
    // C is rounded once: every wave has finished the loop (barrier), the tail's
    // A and B images go into slots 0 and 1 with k clamped into the tail, and the
    // fragments' k >= ktail are zeroed before the MFMAs (both operands: what was
    // read there may be anything).  Outside the loop: the loop is untouched.
    int ktail = p.ktail;
    if constexpr (PART) ktail = blockIdx.y + 1 == gridDim.y ? ktail : 0;
    if (ktail > 0) {
        bar8();
        const i64 k0 = (i64)nt * BK;
#pragma unroll
        for (int u = 0; u < WM; ++u) {
            const i64 ga = w4::piece_off_tail<WM, KCA>(w + 4 * u, l, m0, p.m, p.lda, ktail);
            const i64 gb = w4::piece_off_tail<WM, KCB>(w + 4 * u, l, n0, p.n, p.ldb, ktail);
            w4::piece<BMR, BUF, KCA>(p.A, p.lda, m0, k0, (int)(ga * 2), ga, w + 4 * u, lds);
            w4::piece<BMR, BUF, KCB>(p.B, p.ldb, n0, k0, (int)(gb * 2), gb, w + 4 * u, lds + UNIT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar8();
#pragma unroll
        for (int sk = 0; sk < 2; ++sk) {
            // lane l holds k = 32 sk + 8 (l >> 4) + j, j = 0..7, two per 32-bit word
            u32x4 mask;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = 32 * sk + 8 * (l >> 4) + 2 * q;
                mask[q] = (k < ktail ? 0xffffu : 0u) | (k + 1 < ktail ? 0xffff0000u : 0u);
            }
            Sets<WM> T;
#pragma unroll
            for (int q = 0; q < WM; ++q) {
                T.a[q] = wfrag<WM, KCA>(lds, wr, q, sk, l) & mask;
                T.b[q] = wfrag<WM, KCB>(lds + UNIT, wc, q, sk, l) & mask;
            }
            asm volatile("s_nop 4" ::: "memory");  // VALU-written operands -> asm MFMA
#pragma unroll
            for (int i = 0; i < WM * WM; ++i) w4::mfma_acc<BF16>(acc[i / WM][i % WM], T.a[i / WM], T.b[i % WM]);
        }
    }
    w4::settle<WM>(acc);
    if constexpr (PART) w4::epilogue_partial<WM>(p, acc, m0, n0, wr, wc, l);
    else w4::epilogue4<BF16, WM>(p, acc, m0, n0, wr, wc, l);
}

// (Measured and removed in round 4: a two-barrier loop that keeps every wave's
// fragment reads and every wave's DMA issue in different barrier intervals, as
// hipBLASLt's MT256x256x64 loop does — correct, but 1-6 % slower than this
// one-barrier loop on every orientation, profiles/r04_h16_two_barrier_ab.log.)

template <int WM, bool BF16, bool KCA, bool KCB>
hipError_t launch_h16(const H2Params& p, hipStream_t s) {
    constexpr int BMR = w4::Geo<WM>::BM;
    // buffer-descriptor DMA when every offset of an image fits 31 bits, else the
    // global (64-bit address) form
    // (ELX_H16_STAGE=g, read per call, forces the global form: the tests cover it)
    const char* stg = getenv("ELX_H16_STAGE");
    const bool buf = !(stg && stg[0] == 'g') && dma_fits(KCA ? BMR : BK, p.lda, 2) && dma_fits(KCB ? BMR : BK, p.ldb, 2);
    const dim3 grid(p.dp_tiles > 0 ? p.dp_tiles : p.tiles_m * p.tiles_n,
                    p.W ? (unsigned)((p.k + p.kchunk - 1) / p.kchunk) : 1u);
    // B's units first (SWP) except for NN, 256 x 256 tiles: one process, bf16
    // 16384^3 NN / NT / TN / TT 1523 / 1421 / 1514 / 1428 -> 1494 / 1459 / 1529 /
    // 1509 TF with B first, 32768^3 NN 1451 -> 1432, TT 1379 -> 1440
    // (profiles/r05as_h16_swap_ab.log): the operand whose misses land later (a
    // rows-contiguous B, or B when the two are alike) gets the longer DMA lead.
    // ELX_H16_SWAP = 0 / 1 forces (read per call, A/B and tests).
    const char* sw = getenv("ELX_H16_SWAP");
    const bool swp = sw ? sw[0] == '1' : (WM == 8 && (KCA || !KCB));
    if (p.W) {
        if (buf) hipLaunchKernelGGL((gemm_h4w_kernel<WM, BF16, KCA, KCB, true, true>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((gemm_h4w_kernel<WM, BF16, KCA, KCB, false, true>), grid, dim3(256), 0, s, p);
    } else if (swp && buf) {
        hipLaunchKernelGGL((gemm_h4w_kernel<WM, BF16, KCA, KCB, true, false, true>), grid, dim3(256), 0, s, p);
    } else {
        if (buf) hipLaunchKernelGGL((gemm_h4w_kernel<WM, BF16, KCA, KCB, true, false>), grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL((gemm_h4w_kernel<WM, BF16, KCA, KCB, false, false>), grid, dim3(256), 0, s, p);
    }
    return hipGetLastError();
}

template <int WM>
hipError_t launch_h16_all(bool is_bf16, bool kca, bool kcb, const H2Params& p, hipStream_t s) {
    if (is_bf16) {
        if (kca) return kcb ? launch_h16<WM, true, true, true>(p, s) : launch_h16<WM, true, true, false>(p, s);
        return kcb ? launch_h16<WM, true, false, true>(p, s) : launch_h16<WM, true, false, false>(p, s);
    }
    if (kca) return kcb ? launch_h16<WM, false, true, true>(p, s) : launch_h16<WM, false, true, false>(p, s);
    return kcb ? launch_h16<WM, false, false, true>(p, s) : launch_h16<WM, false, false, false>(p, s);
}

bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

// Tile-order group height: 8, so the 32 concurrent tiles of an XCD span 8 x 4
// tiles.  Round 3 measured 4 ahead by 1-3 % (profiles/r03_h16_four_wave.log); with
// the round-4 loop (precise waits) 8 is ahead in one process, interleaved: bf16 NN
// 32768^3 +0.7-2.7 %, f16 +0.3-0.9 %, TN 16384^3 even (profiles/r04_h16_group_ab.log),
// and reads 106 instead of 131 GB over the fabric per C5 launch, L2 hit 81 vs 77 %
// (profiles/r04_h16_group_sweep.log).  ELX_H16_GROUP overrides (read per call: A/B tools interleave values), clamped
// to >= 1 because tile_of divides by it.
int GroupM() {
    const char* v = getenv("ELX_H16_GROUP");
    const int g = v ? atoi(v) : 8;
    return g >= 1 ? g : 1;
}

}  // namespace

// Tile size and split-k of the four-wave kernel: h16_plan in kernels.hpp.

#ifndef ELX_KERNEL_PROBE
namespace {
hipError_t gemm_mfma_h_plan(bool is_bf16, bool ta, bool tb, i64 m, i64 n, i64 k, float alpha, const uint16_t* A,
                            i64 lda, const uint16_t* B, i64 ldb, float beta, uint16_t* C, i64 ldc, hipStream_t s,
                            const H16Plan* forced);
}

hipError_t gemm_mfma_h(bool is_bf16, bool ta, bool tb, i64 m, i64 n, i64 k, float alpha, const uint16_t* A,
                       i64 lda, const uint16_t* B, i64 ldb, float beta, uint16_t* C, i64 ldc, hipStream_t s) {
    return gemm_mfma_h_plan(is_bf16, ta, tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s, nullptr);
}

namespace {
hipError_t gemm_mfma_h_plan(bool is_bf16, bool ta, bool tb, i64 m, i64 n, i64 k, float alpha, const uint16_t* A,
                            i64 lda, const uint16_t* B, i64 ldb, float beta, uint16_t* C, i64 ldc, hipStream_t s,
                            const H16Plan* forced) {
    const bool kca = ta, kcb = !tb;
    const i64 kmain = k / BK * BK;
    const H16Plan pl = forced ? *forced : h16_plan(m, n, kmain, kca && kcb);
    const int BMR = pl.wm * 32;
    const i64 tiles = ((m + BMR - 1) / BMR) * ((n + BMR - 1) / BMR);
    // the LDS-DMA path: 16-B aligned rows/columns for the DMA, RC operands a
    // multiple of 8 long (whole 16-B chunks), and enough workgroups
    const bool ok = kmain > 0 && al16(A) && al16(B) && lda % 8 == 0 && ldb % 8 == 0 &&
                    (kca || (m % 8 == 0 && m >= 8)) && (kcb || (n % 8 == 0 && n >= 8)) && tiles * pl.nz >= 64 &&
                    m < (1ll << 31) && n < (1ll << 31);
    if (!ok) return gemm_mfma_h_simple(is_bf16, ta, tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
    const int tm_ = (int)((m + BMR - 1) / BMR), tn_ = (int)((n + BMR - 1) / BMR);
    // The super-block order (tile_of_sb) for grids of whole super-blocks of at
    // most 64 x 64 tiles, one workgroup per CU.  In one process against the
    // grouped order (profiles/r05f_h16_map_ab.log, r05f_h16_map_sweep.log,
    // r05k_map_ab.log): bf16 TN 16384^3 +2.7-15 % (1478 -> 1520 TF; 1319 -> 1515
    // on a box where the grouped order ran slow), NN 16384^3 +3-4 %; 2 x 4 XCD
    // parts of 8 x 4 tiles was the best of six geometries.  At 32768^3 (C5) it
    // is even to -1.6 % and reads 1.6x the grouped order's bytes over the fabric
    // (L2 hit 72 vs 81 %, profiles/r05j_c5_pmc.json vs r05j_c5m0_pmc.json), so
    // larger grids keep the grouped order.  ELX_H16_MAP = 0 / 1 forces the
    // grouped / super-block order, ELX_H16_SB = "xr,pr" sets the geometry (both
    // read per call, for A/B).
    const char* sbv = getenv("ELX_H16_MAP");
    int xr = 2, pr = 8;
    if (const char* g = getenv("ELX_H16_SB")) {
        int a = 0, b = 0;
        if (sscanf(g, "%d,%d", &a, &b) == 2 && a >= 1 && a <= 8 && 8 % a == 0 && b >= 1 && b <= 32 && 32 % b == 0) {
            xr = a;
            pr = b;
        }
    }
    const int sbr = xr * pr, sbc = (8 / xr) * (32 / pr);
    const int mode = sbv ? atoi(sbv) : ((i64)tm_ * tn_ <= 4096 ? 1 : 0);
    // (192-tiles measured even to +1 % in the grouped order: 3072^3 NN 1080 ->
    // 1089, 6144^3 1305 -> 1315, profiles/r06c_h16_tile192_sweep.log)
    const int sblock = mode == 1 && pl.wm == 8 && pl.nz == 1 && tm_ % sbr == 0 && tn_ % sbc == 0;
    // the k tail goes into the kernel (one rounding of C) unless a k-contiguous
    // operand would need a 16-B chunk straddling k (k % 8 != 0): then a second
    // pass adds it to the rounded C (ELX_H16_KTAIL = 0 forces that, for A/B)
    const char* kt_env = getenv("ELX_H16_KTAIL");
    const bool tail_in = kmain != k && !(kt_env && kt_env[0] == '0') && (!(kca || kcb) || k % 8 == 0);
    H2Params p{m, n, kmain, alpha, beta, A, lda, B, ldb, C, ldc, tm_, tn_,
               (reinterpret_cast<uintptr_t>(C) & 7) == 0 && ldc % 4 == 0, GroupM(), sblock, xr, pr, pl.kchunk,
               nullptr, 0, tail_in ? (int)(k - kmain) : 0};
    const i64 nz = pl.nz;
    hipError_t e;
    auto launch = [&]() {
        switch (pl.wm) {
        case 8: return launch_h16_all<8>(is_bf16, kca, kcb, p, s);
        case 7: return launch_h16_all<7>(is_bf16, kca, kcb, p, s);
        case 6: return launch_h16_all<6>(is_bf16, kca, kcb, p, s);
        case 5: return launch_h16_all<5>(is_bf16, kca, kcb, p, s);
        case 2: return launch_h16_all<2>(is_bf16, kca, kcb, p, s);
        default: return launch_h16_all<4>(is_bf16, kca, kcb, p, s);
        }
    };
    // Data-parallel rounds + a tail of smaller tiles (round 6).  A grid whose
    // last round holds at most a quarter of the slots (256 one-per-CU tiles,
    // 512 two-per-CU 128-tiles) leaves most CUs idle for one whole tile's K.  The tiles
    // of that round are the last ones of the grouped order: in the last group
    // of tile rows, its last columns.  Rounded up to whole group columns they
    // form one rectangle of C; the full rounds run as one launch over the
    // first tiles of the order (dp_tiles), and the rectangle as its own GEMM,
    // whose plan gives it tiles small enough (or split-k) to spread over the
    // chip.  Every element of C is written by exactly one of the two, each
    // rounding once.  In one process, tail on / off (profiles/
    // r06j_h16_tail_split_ab.log, bf16 at beta 0; hipBLASLt): NN 7168^3 (784 =
    // 3 x 256 + 16 256-tiles) 1226 -> 1423 TF (1165), 10240^3 (1600 = 6 x 256 +
    // 64) 1322 -> 1375 (1280), 6144^3 in 256-tiles (576 = 2 x 256 + 64) 1231 ->
    // 1290 (1285), TN 1263 -> 1328, 3072^2 x 4096 in 128-tiles (576 = 512 + 64)
    // 864 -> 904; a last round of half the slots lost (6144 x 4096^2, 384 =
    // 256 + 128: 1193 -> 1167), hence the quarter.  A last round of 256-tiles
    // a quarter to a third full (not TN) runs as split-k over the same tiles
    // instead, z = 256 / tiles >= 3 chunks of k each (f32 partials, one
    // reduce): in one process against the 256-tile grid and the plan without
    // it (profiles/r06v_h16_tailsk_ab.log, beta 0): 4608^3 (324 = 256 + 68)
    // NN 994 / 1042 -> 1107 TF, NT 966 / 1026 -> 1086, f16 NN 991 / 986 ->
    // 1078; TN's 224-tiles stay ahead (1160 vs 1129), and at half a round the
    // split loses (6144 x 4096^2: 1105 vs 1156), hence z >= 3.  The group
    // height shrinks (8 -> 6 at 4608^3) where the last group holds fewer tiles
    // than the tail.  ELX_H16_TAIL = 0 turns both off, ELX_H16_TAILSK = 0 the
    // split-k form (read per call, for A/B).
    const char* tv = getenv("ELX_H16_TAIL");
    const bool tail_on = !(tv && tv[0] == '0') && !forced;
    const i64 slots = pl.wm == 4 ? 512 : pl.wm == 2 ? 1024 : 256;
    if (tail_on && nz == 1 && !sblock && (kmain == k || tail_in) && k >= 1024 && tiles > slots) {
        const i64 rem = tiles % slots;
        // split-k tail: see h16_plan; ELX_H16_TAILSK = 0 turns it off (per call)
        const char* skv = getenv("ELX_H16_TAILSK");
        const bool tail_sk = !(skv && skv[0] == '0') && pl.wm == 8 && !(kca && kcb) && rem > slots / 4 &&
                             3 * rem <= slots;
        // the group height whose last group holds the whole tail (G = 8 unless
        // the last group is shorter than the tail)
        int G = p.group_m;
        for (int g = G; g >= 2; --g) {
            const int gs = tm_ - (tm_ - 1) / g * g;
            if ((i64)gs * tn_ >= rem) { G = g; break; }
        }
        const int last = (tm_ - 1) / G, gsz = tm_ - last * G;  // the last group's tile rows
        const i64 cols = (rem + gsz - 1) / gsz;                 // its tail columns
        if (rem > 0 && (rem <= slots / 4 || tail_sk) && cols <= tn_) {
            p.group_m = G;
            p.dp_tiles = (int)(tiles - cols * gsz);
            e = launch();
            if (e != hipSuccess) return e;
            const i64 i0 = (i64)last * G * BMR, j0 = (tn_ - cols) * BMR;
            const uint16_t* At = ta ? A + i0 * lda : A + i0;
            const uint16_t* Bt = tb ? B + j0 : B + j0 * ldb;
            if (!tail_sk)
                return gemm_mfma_h(is_bf16, ta, tb, m - i0, n - j0, k, alpha, At, lda, Bt, ldb, beta, C + i0 + j0 * ldc,
                                   ldc, s);
            // split-k tail: the same tiles, each over z >= 3 chunks of k, z = slots / tiles
            H16Plan tp = pl;
            const i64 z = std::max<i64>(1, slots / (cols * gsz));
            tp.kchunk = ((kmain + z - 1) / z + BK - 1) / BK * BK;
            tp.nz = (kmain + tp.kchunk - 1) / tp.kchunk;
            return gemm_mfma_h_plan(is_bf16, ta, tb, m - i0, n - j0, k, alpha, At, lda, Bt, ldb, beta,
                                    C + i0 + j0 * ldc, ldc, s, &tp);
        }
    }
    if (nz > 1) {
        e = workspace_alloc(reinterpret_cast<void**>(&p.W), sizeof(float) * (size_t)m * (size_t)n * (size_t)nz, s);
        if (e != hipSuccess) return e;
    }
    e = launch();
    if (nz > 1) {
        const char* rv = getenv("ELX_H16_RED");
        const bool red4 = !(rv && rv[0] == '0') && m % 4 == 0 && n <= 65535 &&
                          (reinterpret_cast<uintptr_t>(C) & 7) == 0 && ldc % 4 == 0;
        if (e == hipSuccess && red4) {
            const dim3 grid((unsigned)((m + 1023) / 1024), (unsigned)n);
            if (is_bf16)
                hipLaunchKernelGGL((w4::h16_splitk_reduce4<true>), grid, dim3(256), 0, s, m, n, (int)nz, alpha, p.W,
                                   beta, C, ldc);
            else
                hipLaunchKernelGGL((w4::h16_splitk_reduce4<false>), grid, dim3(256), 0, s, m, n, (int)nz, alpha, p.W,
                                   beta, C, ldc);
            e = hipGetLastError();
        } else if (e == hipSuccess) {
            const i64 mn = m * n;
            const unsigned grid = (unsigned)std::min<i64>((mn + 255) / 256, 2048);
            if (is_bf16)
                hipLaunchKernelGGL((w4::h16_splitk_reduce<true>), dim3(grid), dim3(256), 0, s, m, n, (int)nz, alpha, p.W,
                                   beta, C, ldc);
            else
                hipLaunchKernelGGL((w4::h16_splitk_reduce<false>), dim3(grid), dim3(256), 0, s, m, n, (int)nz, alpha, p.W,
                                   beta, C, ldc);
            e = hipGetLastError();
        }
        const hipError_t f = workspace_free(p.W, s);
        if (e == hipSuccess) e = f;
    }
    if (e != hipSuccess || kmain == k || tail_in) return e;
    // k tail (< 64) as a second pass: C += alpha op(A)(:, kmain:) op(B)(kmain:, :)
    const uint16_t* At = ta ? A + kmain : A + kmain * lda;
    const uint16_t* Bt = tb ? B + kmain * ldb : B + kmain;
    return gemm_mfma_h_simple(is_bf16, ta, tb, m, n, k - kmain, alpha, At, lda, Bt, ldb, 1.0f, C, ldc, s);
}
}  // namespace

#endif  // ELX_KERNEL_PROBE

}  // namespace kern
}  // namespace elx
