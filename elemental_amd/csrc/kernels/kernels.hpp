// Host-side launch interface of the gfx950 kernels (no exceptions; return hipError_t).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdlib>

namespace elx {
namespace kern {

// Stream-ordered scratch for the launchers (split-k partials): the library's
// caching allocator (runtime.cpp), never a driver mempool of its own.
// Returns hipErrorOutOfMemory instead of throwing.
hipError_t workspace_alloc(void** p, size_t bytes, hipStream_t s);
hipError_t workspace_free(void* p, hipStream_t s);

using i64 = int64_t;

template <typename T>
hipError_t gemm_mfma(bool ta, bool tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda,
                     const T* B, i64 ldb, T beta, T* C, i64 ldc, hipStream_t s);
// LDS-DMA kernels (gemm_f64g.hip / gemm_f32g.hip, 128x128 tiles, 2 workgroups per
// CU).  The plan says whether a shape takes them and how k is cut: kmain (a
// multiple of the slab depth; the caller adds the k - kmain tail with the
// general kernel, beta = 1) over nz chunks of kchunk (nz > 1: split-k into a
// workspace of nz m x n partials, alpha = 1, beta = 0, then splitk_reduce).
struct DmaPlan {
    bool use;
    i64 kmain, kchunk;
    int nz;
};
// slots: workgroups the chip holds at once (512: two per CU; the fp64 ring
// kernel's one per CU: 256, so its 2048^2 x 16384 runs whole-k, 256 tiles, with
// no partials' round trip)
inline DmaPlan dma_plan(bool ok, i64 tiles, i64 k, int bk, i64 slots = 512) {
    DmaPlan d{false, 0, 0, 1};
    if (!ok) return d;
    d.kmain = k / bk * bk;
    if (tiles >= slots) {
        d.use = true;
        d.kchunk = d.kmain;
        return d;
    }
    // few tiles: split k for two rounds of workgroups, in chunks of >= 2048 (whole
    // slabs); with fewer tiles than CUs, chunks down to 256 (1024^3 f64: 64 tiles
    // -> 4 chunks, 150 -> 60 us; at 2048^3, 256 tiles, chunks of 512 measured
    // slower than none: the partials' HBM round trip outweighs the fill)
    static const i64 min_env = [] { const char* v = getenv("ELX_DMA_MIN_CHUNK"); return v ? atoll(v) : 0ll; }();
    const i64 min_chunk = min_env >= bk ? min_env : tiles < 256 ? 256 : 2048;
    i64 z = (2 * slots + tiles - 1) / tiles;
    // 33..255 tiles (one workgroup per CU or fewer): 4 chunks up to 200 tiles, 2
    // above, measured best of 2..8 (f64 1024^2 x 2048 44.7 -> 49.4 TF, 1536 x 2048 x
    // 2048 47.4 -> 54.7, 1920 x 2048 x 2048 51.0 -> 57.4; f32 likewise;
    // profiles/r03_f64_small.log).  Fewer tiles keep two rounds of workgroups.
    if (tiles > 32 && tiles < 256) z = tiles <= 200 ? 4 : 2;
    z = z < d.kmain / min_chunk ? z : d.kmain / min_chunk;
    z = z < 16 ? z : 16;
    if (z < 2) {
        // k too short to split: the DMA kernel on the few tiles there are, or
        // (ELX_DMA_FEW=0) the register-staged kernel
        static const bool few = [] { const char* v = getenv("ELX_DMA_FEW"); return !v || v[0] != '0'; }();
        d.use = few && d.kmain > 0;
        d.kchunk = d.kmain;
        return d;
    }
    d.use = true;
    d.kchunk = ((d.kmain + z - 1) / z + bk - 1) / bk * bk;
    d.nz = (int)((d.kmain + d.kchunk - 1) / d.kchunk);
    return d;
}
// 128 x 128 or 64 x 64 tiles for the LDS-DMA kernels (fp64 and fp32).  Grids
// of fewer 128-tiles than CUs take 64 x 64 tiles (four times the workgroups,
// with dma_plan's split-k on that count): 1024^3 fp32 69 -> 93 TF, fp64 38 -> 46;
// 512^2 x 2048 fp32 37 -> 52; 1024^2 x 2048 even (profiles/r04_small_t64_ab.log).
// Above that, the tile count per CU rounds up to whole tiles, so a grid leaves
// CUs idle in its last round unless its tile count is a multiple of 256; 64 x 64
// tiles (four per CU in flight, ~5 % slower per FLOP than 128 x 128 where both
// fill the chip: profiles/r04_t64_rule_ab.log) win when their balance beats the
// 128-tile one by more than that: 1536 x 2048 (192 vs 768 tiles), 2560^2, 3072^2
// (576 vs 2304: fp64 51.8 -> 67.0 TF, fp32 109 -> 132), 3584^2; not 2048^2,
// 4096^2 or any other multiple of 256 128-tiles.  mode: 0 never, 2 always
// (tests), else this rule.  small: the largest 128-tile count that always takes
// 64 x 64 tiles (255 for both: round 4 sent fp64's 2048^2 grid of 256 tiles to
// its eight-wave 64 x 64 tiles, which beat the slab kernel's 128 x 128 there,
// NN 64.0 -> 66.2 TF; the round-5 ring kernel beats both, 69.3 TF,
// profiles/r05o_ring_ab.log).
inline bool prefer_t64(int mode, i64 m, i64 n, i64 small = 255) {
    if (mode == 0 || mode == 2) return mode == 2;
    const i64 t128 = (m + 127) / 128 * ((n + 127) / 128), t64 = (m + 63) / 64 * ((n + 63) / 64);
    if (t128 <= small) return true;
    const auto bal = [](i64 t) { return (double)t / (double)(256 * ((t + 255) / 256)); };
    return 0.95 * bal(t64) > bal(t128);
}
DmaPlan gemm_f64_lds_dma_plan(bool ta, bool tb, i64 m, i64 n, i64 k, const double* A, i64 lda, const double* B,
                              i64 ldb);
hipError_t gemm_f64_lds_dma(bool ta, bool tb, i64 m, i64 n, i64 kmain, i64 kchunk, double alpha, const double* A,
                            i64 lda, const double* B, i64 ldb, double beta, double* C, i64 ldc, hipStream_t s);
DmaPlan gemm_f32_lds_dma_plan(bool ta, bool tb, i64 m, i64 n, i64 k, const float* A, i64 lda, const float* B,
                              i64 ldb);
hipError_t gemm_f32_lds_dma(bool ta, bool tb, i64 m, i64 n, i64 kmain, i64 kchunk, float alpha, const float* A,
                            i64 lda, const float* B, i64 ldb, float beta, float* C, i64 ldc, hipStream_t s);
// 16-bit GEMMs: is_bf16 selects bf16 vs f16 storage; f32 accumulation.
// the 16-bit four-wave kernel's plan (gemm_h16.hip): tile 32 wm (wm 8 or 4),
// nz split-k chunks of kchunk (nz = 1: whole k)
struct H16Plan { int wm; i64 nz, kchunk; };
// Tile size and split-k of the four-wave kernel (gemm_h16.hip; host-only, here
// so tests/cpp/test_tile_rule.cpp checks it without a GPU).
//  * 256 x 256 tiles (WM = 8) unless fewer than half the CUs would get one;
//    then 128 x 128 tiles (WM = 4, two workgroups per CU), a grid four times as
//    wide.  In one process against the 256-tiles (profiles/r05b_h16_sweep.log):
//    bf16 2048^3 382 -> 673 TF (hipBLASLt 659), 2560^3 (100 tiles) 542 -> 810,
//    1536 x 2048^2 217 -> 528, 1024^3 69 -> 177, 1024^2 x 8192 347 -> 486 (with
//    split-k), 2048^2 x 8192 873 -> 998; but 3072^3 (144 tiles) 834 -> 768 and
//    4096^3 (256) 1309 -> 1139: where 256-tiles fill half the chip or more, their
//    halved LDS reads per FLOP win.
//  * 192 x 192 tiles (WM = 6, one workgroup per CU, round 6) where the
//    256-tiles leave more than a quarter of their last round's CUs idle
//    (utilisation u8 = tiles / (rounds x 256) <= 0.75) and a round of 192-tiles
//    fills clearly better, 128-tiles (two per CU, 512 slots per round) where
//    they do: each candidate scored u x its measured relative rate (192 and
//    128: 0.8 of the 256-tile loop at full rounds), the 256-tiles kept unless
//    beaten.  Measured in one process beside hipBLASLt on two boxes
//    (profiles/r06c_h16_tile192_sweep.log, r06d_h16_tile_map.log,
//    r06e_h16_midsize_vs_vendor_b0.log, r06h_h16_tile_map_b0.log; bf16 NN,
//    256 / 192 / 128 / vendor): 3072^3 (u8 0.56, u6 1.0) 830 / 1094 / 767 / 973
//    and 896 / 1042 / 816 / 966; 4608^3 (u8 0.63, 128-tiles 0.84) 968 / 989 /
//    1017 and 1015 / 897 / 1075; 4096 x 2048 x 4096 (u8 0.5, u4 1.0) 817 / 1014
//    / 1090; 6144^3 (u8 0.75) 1161 / 1294 / 1114 and 1212 / 1195 / 1179: the
//    192-tile's rate varies more between boxes (it reads a third more operand
//    bytes per FLOP than the 256-tile).  A grid whose last round of 256-tiles
//    is at most a quarter full counts as 0.95: gemm_mfma_h's tail split runs
//    that round on smaller tiles (6144^3: 256-tiles with the tail 1290 TF, the
//    192-tiles 1185 on the same box, profiles/r06j_h16_tail_split_ab.log); one
//    a quarter to a third full (not TN) as 0.9: the tail runs split-k (4608^3 NN
//    1107 TF against 1042 on 128-tiles, profiles/r06v_h16_tailsk_ab.log).  At
//    exactly 0.75 (1.5 rounds: 6144 x 4096, 3072 x 8192) the 256-tiles stay:
//    the half-filled round runs at a higher clock than its share predicts
//    (bf16 NN 6144 x 4096 x 8192 1273 vs 1087 TF on 128-tiles, x 4096 1116 vs
//    1108 at beta 1 and 1182 vs 1139 at beta 0, f16 1148 vs 1128; NT 1084 vs
//    1099; profiles/r06y_h16_t384_ab.log).  Below 128 256-tiles the 128-tiles
//    stay (2560^3: 128-tiles 856 / 880 against 834 / 710 for 192), except for
//    TN grids of nearly a full round of 160-tiles (below).
//  * TN (both operands k-contiguous) may also take 224 x 224 (WM = 7) and
//    160 x 160 (WM = 5) tiles, rated 0.92 and 0.8: TN 3584^3 (16 x 16 224-tiles)
//    1209 -> 1320 TF (hipBLASLt 1358), TN 2560^3 (16 x 16 160-tiles) 863 -> 999
//    (980).  With a rows-contiguous operand they lose (NN 3584^3 224-tiles 1074
//    vs 1181: their last RC block is 32 columns, 64-B k-rows, twice the DMA
//    requests per byte of the 128-column blocks), so other orientations never
//    take them.
//  * 64 x 64 tiles (WM = 2, four workgroups per CU) where 64 to 255 128-tiles
//    leave CUs idle and k is too short to split: in one process at beta 1
//    (profiles/r06z2_h16_t64_ab.log, bf16, 128 -> 64): 1024^3 175 -> 290 TF,
//    1024 x 2048 x 1024 340 -> 474, 2048 x 1024 x 4096 431 -> 570, 1536^3 359
//    -> 417, 1536 x 2048^2 522 -> 549; at 256 128-tiles and above the 128-tiles
//    win (2048^3 674 vs 580, 2560^3 805 vs 538), and split-k beats them where k
//    is long (1024^2 x 8192 490 vs 374).  ELX_H16_TILE = 256 / 224 / 192 / 160 /
//    128 / 64 forces one (read per
//    call, for A/B).
inline H16Plan h16_plan(i64 m, i64 n, i64 kmain, bool tn = false) {
    constexpr i64 BK = 64;  // the four-wave kernel's K-tile
    const char* tv = getenv("ELX_H16_TILE");
    const int force = tv ? atoi(tv) : 0;
    auto tiles_of = [&](i64 bm) { return ((m + bm - 1) / bm) * ((n + bm - 1) / bm); };
    auto util = [](i64 t, i64 slots) { return (double)t / (double)(((t + slots - 1) / slots) * slots); };
    H16Plan pl;
    if (force == 64 || force == 128 || force == 160 || force == 192 || force == 224 || force == 256) {
        pl.wm = force / 32;
    } else if (tiles_of(256) < 128) {
        pl.wm = tn && tiles_of(160) >= 224 ? 5 : 4;
        // 64 x 64 tiles (four workgroups per CU) where the 128-tiles fill fewer
        // than one CU each and would not split k
        const i64 t4 = tiles_of(128);
        if (pl.wm == 4 && t4 >= 64 && t4 < 256) {
            const i64 z4 = t4 <= 64 && kmain >= 8 * BK ? std::min<i64>((256 + t4 - 1) / t4, kmain / (16 * BK)) : 1;
            if (z4 < 2) pl.wm = 2;
        }
    } else {
        // gemm_mfma_h runs a last round of at most a quarter of the slots as
        // a separate GEMM on smaller tiles (the tail split): such a grid counts
        // as nearly full
        const char* tl = getenv("ELX_H16_TAIL");
        const char* sk = getenv("ELX_H16_TAILSK");
        const i64 t8 = tiles_of(256), r8 = t8 % 256;
        const bool tail_ok = !(tl && tl[0] == '0') && t8 > 256 && kmain >= 1024;
        const bool tail8 = tail_ok && r8 > 0 && r8 <= 64;
        // a quarter to a third of a round: the split-k tail (not TN)
        const bool sk8 = tail_ok && !tn && !(sk && sk[0] == '0') && r8 > 64 && 3 * r8 <= 256;
        const double u8 = tail8 ? 0.95 : sk8 ? 0.9 : util(t8, 256);
        pl.wm = 8;
        if (u8 < 0.75) {
            double best = u8;
            const double s6 = 0.8 * util(tiles_of(192), 256), s4 = 0.8 * util(tiles_of(128), 512);
            if (s6 > best) { best = s6; pl.wm = 6; }
            if (s4 > best) { best = s4; pl.wm = 4; }
        }
        if (tn && u8 < 1.0) {
            double best = pl.wm == 8 ? u8 : pl.wm == 6 ? 0.8 * util(tiles_of(192), 256) : 0.8 * util(tiles_of(128), 512);
            const double s7 = 0.92 * util(tiles_of(224), 256), s5 = 0.8 * util(tiles_of(160), 256);
            if (s7 > best) { best = s7; pl.wm = 7; }
            if (s5 > best) { best = s5; pl.wm = 5; }
        }
    }
    const i64 bm = pl.wm * 32;
    const i64 tiles = ((m + bm - 1) / bm) * ((n + bm - 1) / bm);
    const char* sv = getenv("ELX_H16_SPLIT");
    const i64 split_cap = sv ? (i64)atoi(sv) : 64;
    pl.nz = 1;
    pl.kchunk = kmain;
    if (split_cap > 1 && tiles <= 64 && kmain >= 8 * BK) {
        const i64 min_kt = tiles >= 64 ? 16 : 4;
        const i64 z = std::min<i64>(std::min<i64>((256 + tiles - 1) / tiles, kmain / (min_kt * BK)), split_cap);
        if (z >= 2) {
            pl.kchunk = ((kmain + z - 1) / z + BK - 1) / BK * BK;
            pl.nz = (kmain + pl.kchunk - 1) / pl.kchunk;
        }
    }
    return pl;
}

hipError_t gemm_mfma_h(bool is_bf16, bool ta, bool tb, i64 m, i64 n, i64 k, float alpha,
                       const uint16_t* A, i64 lda, const uint16_t* B, i64 ldb, float beta,
                       uint16_t* C, i64 ldc, hipStream_t s);
// the 128x128-tile kernel every shape can take (edges, k tails, small problems)
hipError_t gemm_mfma_h_simple(bool is_bf16, bool ta, bool tb, i64 m, i64 n, i64 k, float alpha,
                              const uint16_t* A, i64 lda, const uint16_t* B, i64 ldb, float beta,
                              uint16_t* C, i64 ldc, hipStream_t s);

// One strided 2-D block move: dst(i,j) (=|+=) alpha*src(i,j),
// src(i,j) = src[i*scs + j*srs], dst(i,j) = dst[i*dcs + j*drs].
struct Copy2D {
    i64 m, n;
    const void* src; i64 scs, srs;
    void* dst; i64 dcs, drs;
};
constexpr int kMaxCopyBatch = 16;
// Executes up to any number of descriptors (chunks of kMaxCopyBatch per launch).
// axpy=false: plain copy (bit-exact, alpha ignored); axpy=true: dst += alpha*src.
// max_wgs > 0 caps the workgroups of the launch (grid-stride loops cover the rest)
hipError_t copy2d_batch(int dtype, const Copy2D* d, int nd, bool axpy, double alpha, hipStream_t s, int max_wgs = 0);

// Rank-ordered reduction of a ReduceScatter's contributions (AxpyContract,
// AxpyContract.hpp:462-478): for every (i,j) of the common destination
// pattern, dst(i,j) += alpha*src_q(i,j) for q = 0, 1, ... in order, rounded to
// the storage type after each source -- bit-identical to one copy2d_batch axpy
// launch per source, but dst is read and written once ((nsrc + 2) elements of
// traffic instead of 3 nsrc).
constexpr int kMaxContractSources = 16;
struct ContractSum {
    i64 m, n;
    void* dst; i64 dcs, drs;
    int nsrc;
    const void* src[kMaxContractSources];
    i64 scs[kMaxContractSources], srs[kMaxContractSources];
};
hipError_t contract_sum(int dtype, const ContractSum& c, double alpha, hipStream_t s, int max_wgs = 0);

// Type-converting strided copy: dst(i,j) = (dst type) src(i,j), one rounding (elem.hpp).
hipError_t convert2d(int src_dtype, int dst_dtype, const Copy2D& d, hipStream_t s);
hipError_t fill2d(int dtype, i64 m, i64 n, double v, void* A, i64 lda, hipStream_t s);
// Frobenius-norm partials (mode 0: max |a|, mode 1: sum (a/scale)^2) in double,
// at most kNormPartsMax of them written to out; *nparts says how many
constexpr int kNormPartsMax = 4096;
hipError_t norm_partials(int dtype, int mode, i64 m, i64 n, const void* A, i64 lda, double scale, double* out,
                         int* nparts, hipStream_t s);
hipError_t scale2d(int dtype, i64 m, i64 n, double alpha, void* A, i64 lda, hipStream_t s);
hipError_t hadamard2d(int dtype, i64 m, i64 n, const void* A, i64 lda, const void* B, i64 ldb,
                      void* C, i64 ldc, hipStream_t s);
hipError_t entrywise_map(int dtype, int fn, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb,
                         hipStream_t s);
hipError_t combine(int dtype, int fn, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb, hipStream_t s);
hipError_t fill_hash(int dtype, i64 m, i64 n, void* A, i64 lda, i64 i0, i64 istride, i64 j0,
                     i64 jstride, uint64_t seed, double center, double radius, hipStream_t s);

// Y(i,j) := beta*Y + alpha*X (X null: beta*Y) where global (i0+i*istride, j0+j*jstride)
// lies in the lower (gi >= gj - offset) or upper (gi <= gj - offset) trapezoid.
hipError_t trapezoid2d(int dtype, bool lower, i64 m, i64 n, double alpha, const void* X, i64 ldx, double beta,
                       void* Y, i64 ldy, i64 i0, i64 istride, i64 j0, i64 jstride, i64 offset, hipStream_t s);
// op(A) X = B in place (A m x m, uplo triangle, unit diagonal optional); f64/f32 only.
// ident: B (m x m) is output only and becomes op(A)^-1.
hipError_t trsm_local(int dtype, bool ident, bool lower, bool trans, bool unit, i64 m, i64 n, const void* A, i64 lda,
                      void* B, i64 ldb, hipStream_t s);
// W_b := op(A_bb)^-1 for every nb x nb diagonal block of A (m x m; the last may be
// ragged), W_b at W + b*nb*nb with leading dimension nb; one launch.  Dynamic LDS
// of one workgroup: nb x 65 elements, at most kTriInverseLdsMax (the caller
// falls back to 128-row blocks when the >64 KiB attribute cannot be set)
constexpr long kTriInverseLdsMax = 150 * 1024;
// can one workgroup get nb x 65 elements of dynamic LDS (sets the >64 KiB attribute)?
bool tri_inverse_lds_ok(int dtype, i64 nb);
hipError_t tri_inverse_batched(int dtype, bool lower, bool trans, bool unit, i64 nb, i64 m, const void* A, i64 lda,
                               void* W, hipStream_t s);
}  // namespace kern
}  // namespace elx
