// fp64 local panel update, LDS-DMA path for gfx950: C := alpha op(A) op(B) + beta C
// (column-major).  The hot kernel of configs C1-C3 (SUMMA's LocalGemm,
// src/blas_like/level3/Gemm.cpp:163-186 -> rocblas_dgemm in the reference,
// include/hydrogen/blas/GPU_BLAS_impl.hpp:397-423).
//
// Why a second fp64 kernel: ablating the register-staged kernel of
// gemm_mfma.hip (profiles/r01_sched_knobs.log) showed the slab staging
// (global_load -> VGPR -> select -> ds_write) costs ~12 % of the MFMA pipe,
// the barriers ~3 %.  Here the staging is global_load_lds (LDS DMA): no VGPR
// round trip, no ds_write issue, no selects, and the next slab is in flight
// across the MFMAs of the current one.
//
// Geometry: 128 x 128 tile, BK = 16, two LDS stages of 32 KiB -> two workgroups
// per CU.  Waves: 4 of 64 x 64 (4 x 4 accumulators of v_mfma_f64_16x16x4_f64,
// 0.5 ds_read per MFMA, 2 waves per SIMD) for NN/TN/TT; 8 of 32 x 64 (2 x 4
// accumulators, 4 waves per SIMD) for NT, where it measured faster
// (profiles/r01_f64_wave.log).  LDS images, 16-B chunk XOR swizzles applied to the
// glds SOURCE addresses (the DMA writes lane-linearly), conflict-free reads:
//   KC (k contiguous in HBM): [128 rows][16 k] (128-B rows), chunk c -> c ^ ((r>>1)&7)
//   RC (rows contiguous):     [16 k][128 rows] (1-KiB k-rows), chunk c -> c ^ 8(kk&1)
// Edges: rows past m/n are clamped (read, never stored); k is a multiple of 16
// here (the k tail goes to the general kernel); 16-B aligned operands.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include "kernels.hpp"
#include "lds_dma.hpp"

namespace elx {
namespace kern {

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 16, GROUP_M = 8;
constexpr bool RING64_DEFAULT = true;  // the 64 x 64 ring on grids of 64-tiles by default
// Tile shape: BM = 128 rows, slab depth SK = 16 (two 32-KiB stages: two
// workgroups per CU); wave tiles WTM x 64 with WTM = 32 (2 x 4 accumulators,
// 0.75 ds_read per MFMA) or 64 (4 x 4 accumulators, 0.5 ds_read per MFMA, half
// the waves).  (The template also admits BM = 256 and SK = 32, both measured
// slower and no longer launched.)
// BN_ x WTN_: the N side likewise (128 x 64 everywhere but the 64 x 64 tiles
// of grids with few 128 x 128 tiles).
template <int BM_, int WTM_ = 32, int SK_ = BK, int BN_ = 128, int WTN_ = 64>
struct Shape {
    static constexpr int BM = BM_, WTM = WTM_, MI = WTM_ / 16, WM = BM_ / WTM_, SK = SK_;
    static constexpr int BN = BN_, WTN = WTN_, NI = WTN_ / 16, WN = BN_ / WTN_, NW = WM * WN, NT = 64 * NW;
    static constexpr int IMGA = BM * SK * 8, IMGB = BN * SK * 8, STAGE = IMGA + IMGB;
    // waves resident per SIMD: two workgroups per CU at SK = 16 (BM 64 / 128), and
    // four of the 32-KiB 64 x 64 tiles
    static constexpr int WAVES_PER_EU = BM_ == 64 && BN_ == 64 ? 4 : NW * (BM_ <= 128 && SK_ == 16 ? 2 : 1) / 4;
};

// KC images: rows of SK doubles (128 B at SK 16, 256 B at SK 32); 16-B chunk c of
// row r stored at c ^ swz_kc(r): at SK 16 (r>>1)&7, at SK 32 r&15 (the 32 lanes of
// a ds_read_b64 half-wave read 16 rows x one chunk: 16 distinct chunks, 256 B).
template <int SK>
__device__ __forceinline__ int swz_kc(int r) { return SK == 16 ? (r >> 1) & 7 : r & 15; }

struct GParams {
    i64 m, n, k;  // k: multiple of BK
    double alpha, beta;
    const double* A; i64 lda;
    const double* B; i64 ldb;
    double* C; i64 ldc;
    int tiles_m, tiles_n;
    // split-k (gridDim.y chunks): chunk z covers k in [z*kchunk, min(k, (z+1)*kchunk))
    // and writes C + z*zstride (the caller passes a workspace, alpha = 1, beta = 0)
    i64 kchunk, zstride;
    int group_m;  // tile-order group height (L2 locality of the concurrently running tiles)
    int xcd_remap;
};

__device__ __forceinline__ void tile_of(int bid, int nwg, int tiles_m, int tiles_n, int group_m, int remap, int& tm,
                                        int& tn) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = remap ? (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3) : bid;
    const int per_group = group_m * tiles_n;
    const int group = wg / per_group;
    const int first_m = group * group_m;
    const int gsz = min(tiles_m - first_m, group_m);
    const int inner = wg - group * per_group;
    tm = first_m + inner % gsz;
    tn = inner / gsz;
}

// Stage one operand image (ROWS operand rows from global row R, SK k from k0):
// ROWS*SK/128 wave-instructions of 1 KiB dealt over NW waves.
template <bool BUF, bool KC, int ROWS, int NW, int SK>
__device__ __forceinline__ void stage_img(const double* X, i64 ld, i64 rows, i64 R, i64 k0, lds_char* img, int w,
                                          int l) {
    constexpr int NINS = ROWS * SK * 8 / 1024;
    constexpr int CPR = SK / 2, RPI = 64 / CPR;  // 16-B chunks per row, rows per instruction
    const DmaSrc<BUF, double> src(KC ? X + R * ld + k0 : X + R + k0 * ld, (KC ? ROWS : SK) * ld * 8);
#pragma unroll
    for (int q = 0; q < NINS / NW; ++q) {
        const int ins = w + NW * q;
        if (KC) {  // X(row, k) = X[k + row*ld]; RPI rows of SK*8 B per instruction
            const int r = ins * RPI + l / CPR;
            const int c = (l % CPR) ^ swz_kc<SK>(r);
            const i64 row = R + r < rows ? r : rows - 1 - R;  // rows past the edge: any valid data
            src.load(row * ld + 2 * c, img + ins * 1024);
        } else if constexpr (ROWS * 8 >= 1024) {  // X(row, k) = X[row + k*ld]; k-rows of ROWS*8 B
            constexpr int IPR = ROWS * 8 / 1024;  // instructions per k-row
            const int kk = ins / IPR;
            const int c = ((ins % IPR) * 64 + l) ^ ((kk & 1) << 3);
            const i64 col = R + 2 * c <= rows - 2 ? 2 * c : rows - 2 - R;
            src.load(col + kk * ld, img + ins * 1024);
        } else {  // short k-rows (ROWS = 64: 512 B): several k-rows per 1-KiB instruction
            constexpr int CPK = ROWS * 8 / 16, KPI = 1024 / (ROWS * 8);  // chunks per k-row, k-rows per instruction
            const int kk = ins * KPI + l / CPK;
            const int c = (l % CPK) ^ ((kk & 1) << 3);
            const i64 col = R + 2 * c <= rows - 2 ? 2 * c : rows - 2 - R;
            src.load(col + kk * ld, img + ins * 1024);
        }
    }
}

// Operand of one 16x16x4 MFMA: lane l holds X(R0 + (l&15), 4s + (l>>4)).
template <bool KC, int ROWS, int SK>
__device__ __forceinline__ double opnd(const lds_char* img, int R0, int s, int l) {
    const int r = R0 + (l & 15), k = 4 * s + (l >> 4);
    int off;
    if (KC) off = r * (SK * 8) + ((((k >> 1) ^ swz_kc<SK>(r))) << 4) + ((k & 1) << 3);
    else off = k * (ROWS * 8) + ((((r >> 1) ^ ((k & 1) << 3))) << 4) + ((r & 1) << 3);
    return *(const __attribute__((address_space(3))) double*)(img + off);
}

struct Frame {
    const double* A; i64 lda, m, m0;
    const double* B; i64 ldb, n, n0;
    int w, l, wr, wc;
};

// One slab: stage slab t+1 into `next` and run slab t's MFMAs from `cur`.  The
// __restrict__ LDS pointers give the inlined accesses alias scopes, so the
// waitcnt pass does not drain the in-flight DMA before the ds_reads.
template <typename SH, bool KCA, bool KCB, bool BUF>
__device__ __forceinline__ void slab(const Frame& f, i64 knext, bool more, lds_char* __restrict__ next,
                                     const lds_char* __restrict__ cur, f64x4 (&acc)[SH::MI][SH::NI]) {
    if (more) {
        stage_img<BUF, KCA, SH::BM, SH::NW, SH::SK>(f.A, f.lda, f.m, f.m0, knext, next, f.w, f.l);
        stage_img<BUF, KCB, SH::BN, SH::NW, SH::SK>(f.B, f.ldb, f.n, f.n0, knext, next + SH::IMGA, f.w, f.l);
    }
    const lds_char* Ai = cur;
    const lds_char* Bi = cur + SH::IMGA;
#pragma unroll
    for (int s = 0; s < SH::SK / 4; ++s) {
        double a[SH::MI], b[SH::NI];
#pragma unroll
        for (int mi = 0; mi < SH::MI; ++mi) a[mi] = opnd<KCA, SH::BM, SH::SK>(Ai, f.wr * SH::WTM + mi * 16, s, f.l);
#pragma unroll
        for (int ni = 0; ni < SH::NI; ++ni) b[ni] = opnd<KCB, SH::BN, SH::SK>(Bi, f.wc * SH::WTN + ni * 16, s, f.l);
#pragma unroll
        for (int mi = 0; mi < SH::MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < SH::NI; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
}

// BUF: stage through buffer descriptors (default where every lane offset of a
// slab image fits the descriptor's 31-bit range): +2.5 % over global_load_lds
// (profiles/r01_f64_buf.log).
template <typename SH, bool KCA, bool KCB, bool BETA0, bool BUF>
__global__ __launch_bounds__(SH::NT, SH::WAVES_PER_EU) void gemm_f64g_kernel(GParams p) {
    constexpr int BM = SH::BM, BN = SH::BN, STAGE = SH::STAGE;
    __shared__ __attribute__((aligned(1024))) char lds_raw[2 * STAGE];
    lds_char* lds = (lds_char*)lds_raw;
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w / SH::WN, wc = w % SH::WN;  // WM (M) x WN (N) waves of WTM x WTN
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, p.xcd_remap, tm, tn);
    const i64 m0 = (i64)tm * BM, n0 = (i64)tn * BN;
    {
        const i64 kz0 = (i64)blockIdx.y * p.kchunk;
        p.k = min(p.kchunk, p.k - kz0);
        p.A += KCA ? kz0 : kz0 * p.lda;
        p.B += KCB ? kz0 : kz0 * p.ldb;
        p.C += (i64)blockIdx.y * p.zstride;
    }
    const Frame f{p.A, p.lda, p.m, m0, p.B, p.ldb, p.n, n0, w, l, wr, wc};

    f64x4 acc[SH::MI][SH::NI];
#pragma unroll
    for (int a = 0; a < SH::MI; ++a)
#pragma unroll
        for (int b = 0; b < SH::NI; ++b) acc[a][b] = f64x4{0, 0, 0, 0};

    const int nt = (int)(p.k / SH::SK);
    stage_img<BUF, KCA, BM, SH::NW, SH::SK>(p.A, p.lda, p.m, m0, 0, lds, w, l);
    stage_img<BUF, KCB, BN, SH::NW, SH::SK>(p.B, p.ldb, p.n, n0, 0, lds + SH::IMGA, w, l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        const int cur = t & 1;
        slab<SH, KCA, KCB, BUF>(f, (i64)(t + 1) * SH::SK, t + 1 < nt, lds + (cur ^ 1) * STAGE, lds + cur * STAGE,
                                acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // next slab landed
        __syncthreads();                                    // and every wave is done with this one
    }

    // Epilogue: C/D map of v_mfma_f64_16x16x4_f64: row = (lane>>4) + 4*reg, col = lane&15
    const int g = l >> 4, c = l & 15;
    const i64 ib = m0 + wr * SH::WTM, jb = n0 + wc * SH::WTN;
    if (m0 + BM <= p.m && n0 + BN <= p.n) {
        // interior tile: every C load issued before the first store (the guarded
        // form below serializes load -> wait -> store per element)
#pragma unroll
        for (int mi = 0; mi < SH::MI; ++mi) {  // 16 loads in flight per 16-row block (VGPR budget: 4 waves per SIMD)
            double cv[SH::NI][4];
            if (!BETA0) {
#pragma unroll
                for (int ni = 0; ni < SH::NI; ++ni)
#pragma unroll
                    for (int r = 0; r < 4; ++r) cv[ni][r] = p.C[(jb + ni * 16 + c) * p.ldc + ib + mi * 16 + g + 4 * r];
            }
#pragma unroll
            for (int ni = 0; ni < SH::NI; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double v = p.alpha * acc[mi][ni][r];
                    p.C[(jb + ni * 16 + c) * p.ldc + ib + mi * 16 + g + 4 * r] = BETA0 ? v : v + p.beta * cv[ni][r];
                }
        }
        return;
    }
#pragma unroll
    for (int mi = 0; mi < SH::MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < SH::NI; ++ni) {
            const i64 j = jb + ni * 16 + c;
            if (j >= p.n) continue;
            double* col = p.C + j * p.ldc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 i = ib + mi * 16 + g + 4 * r;
                if (i < p.m) {
                    const double v = p.alpha * acc[mi][ni][r];
                    col[i] = BETA0 ? v : v + p.beta * col[i];
                }
            }
        }
}

// ---------------------------------------------------------------------------
// Ring kernel (round 5): the 16-bit four-wave loop (gemm_h16.hip) in fp64.
// 128 x 128 tile, four waves of 64 x 64 (4 x 4 accumulators of
// v_mfma_f64_16x16x4_f64, 64 cycles each), one wave per SIMD, one workgroup per
// CU.  Staging unit = one operand's K-tile image of RBK = 32 k (KC: 128 rows of
// 256 B; RC: 32 k-rows of 1 KiB): 32 KiB = 32 one-KiB pieces, 8 per wave; a ring
// of 5 slots (160 KiB): A_t is unit 2t, B_t unit 2t+1, unit u in slot u % 5.
// A K-tile is 8 k-steps of 16 MFMAs per wave (8192 cycles).  In K-tile t:
//   (t,0..3): two pieces of A_{t+2} per k-step, into B_{t-1}'s slot;
//   (t,0..6): each k-step's MFMAs and the next k-step's 8 operand reads from
//             A_t, B_t;
//   after (t,6): vmcnt(8) (A_{t+1}, B_{t+1} landed; A_{t+2} may be in
//             flight), lgkmcnt(0), barrier;
//   (t,7):    MFMAs; reads of (t+1,0) from A_{t+1}, B_{t+1}; the 8 pieces of
//             B_{t+2} into A_t's slot.
// RAW: A_{t+1}, B_{t+1} are read from (t,7) on, after every wave's wait and the
// barrier.  WAR: A_t's and B_t's last reads are issued in (t,6) and retired
// before that barrier; A_t's slot is restaged in (t,7), B_t's in (t+1,0..3),
// both after it.  No wave can pass a barrier another has not reached, so one
// barrier per K-tile (8192 MFMA cycles) suffices.  Units past the end re-stage
// the last K-tile into a slot nobody reads again (counted waits stay exact).
// Versus the two-stage slab kernel (one barrier and a full vmcnt(0) drain per
// 16-k slab, two workgroups per CU): no drain, one barrier per 32 k, 1.5 K-tiles
// of DMA lead.
// ---------------------------------------------------------------------------
namespace ring {
constexpr int NSLOT = 5;
// BT 128: the kernel above.  BT 64 (round 5, grids of 64-tiles): four waves of
// 32 x 32 (2 x 2 accumulators), K-tiles of 16 k (8 KiB per image, 40 KiB of
// ring), four workgroups per CU, 4 k-steps of 4 MFMAs per K-tile; the same
// schedule with 2 pieces per wave and image.
// UN: bytes of one operand image (32 KiB: one workgroup per CU; 8 KiB: the 64 x 64
// ring, four per CU).  (A 128 x 128 ring with 16 KiB images, two per CU, the
// fp32 kernel's choice, measured 32768^3 76.3 -> 70.9 TF, 16384^3 -0.3..-1.8 %,
// +0.5..1.3 % at 4096^2: not kept, profiles/r05ak_f64_ring129_ab.log.)
template <int BT, int UN>
struct RG {
    static constexpr int UNIT = UN, RBK = UN / 8 / BT, WT = BT / 2, MI = WT / 16;
    static constexpr int NKS = RBK / 4;                // k-steps per K-tile
    static constexpr int NPW = UNIT / 1024 / 4;        // pieces per wave and image
    static constexpr int NM = MI * MI, NR = 2 * MI;    // MFMAs and operand reads per k-step
    static constexpr int MINB = 32768 / UN;            // workgroups per CU
};

// per-lane element offset of piece `ins` of one operand's K-tile image
template <int BT, int UN, bool KC>
__device__ __forceinline__ i64 piece_off(int ins, int l, i64 R0, i64 rows, i64 ld) {
    constexpr int RBK = RG<BT, UN>::RBK;
    if (KC) {  // RPI rows of RBK doubles per piece; chunk c of row r at c ^ swz_kc(r)
        constexpr int CPR = RBK / 2, RPI = 64 / CPR;
        const int r = ins * RPI + l / CPR;
        const int c = (l % CPR) ^ swz_kc<RBK>(r);
        const i64 row = R0 + r < rows ? r : rows - 1 - R0;
        return row * ld + 2 * c;
    } else {   // blocked: piece = 4 k-rows 4 (ins / NSEG).. x one 256-B line (ins % NSEG)
               // of the BT rows; chunk c at c ^ 8 (kk & 1).  One 1-KiB k-row per piece instead
               // (the slab kernel's shape) ran NN / NT / TT 2.5 / 5.4 / 2.8 % slower at
               // 16384^3, 2048^3 NN 69.4 -> 70.9 TF (profiles/r05aa_f64_rcblk_ab.log)
        constexpr int NSEG = BT * 8 / 256;
        const int kk = (ins / NSEG) * 4 + (l >> 4);
        const int c = (l & 15) ^ ((kk & 1) << 3);
        const int col0 = (ins % NSEG) * 32 + 2 * c;
        const i64 col = R0 + col0 <= rows - 2 ? col0 : rows - 2 - R0;
        return col + kk * ld;
    }
}
// operand of k-step s for rows R0..R0+15 from a ring image (KC: opnd's layout;
// RC: the blocked layout above, 1-KiB block (s, r>>5), sub-row k & 3)
template <int BT, int UN, bool KC>
__device__ __forceinline__ double ropnd(const lds_char* img, int R0, int s, int l) {
    if (KC) return opnd<true, BT, RG<BT, UN>::RBK>(img, R0, s, l);
    constexpr int NSEG = BT * 8 / 256;
    const int r = R0 + (l & 15), g = l >> 4;
    const int off = (s * NSEG + (r >> 5)) * 1024 + g * 256 + ((((r & 31) >> 1) ^ ((g & 1) << 3)) << 4) + ((r & 1) << 3);
    return *(const __attribute__((address_space(3))) double*)(img + off);
}

template <int BT, int UN, bool BUF, bool KC>
__device__ __forceinline__ void piece(const double* X, i64 ld, i64 R0, i64 k0, int off, i64 goff, int ins,
                                      lds_char* img) {
    const double* base = KC ? X + R0 * ld + k0 : X + R0 + k0 * ld;
    if constexpr (BUF) {
        const BufferSrc<double> src(base, (KC ? BT : RG<BT, UN>::RBK) * ld * 8);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src.rs, (__attribute__((address_space(3))) void*)(img + ins * 1024),
                                                 16, off, 0, 0, 0);
    } else {
        __builtin_amdgcn_global_load_lds((const void*)(base + goff),
                                         (__attribute__((address_space(3))) void*)(img + ins * 1024), 16, 0, 0);
    }
}

template <int BT, int UN>
struct Ops { double a[RG<BT, UN>::MI], b[RG<BT, UN>::MI]; };
// this lane's buffer offsets (bytes) / element offsets of its pieces per operand
template <int BT, int UN>
struct Pieces { int offA[RG<BT, UN>::NPW], offB[RG<BT, UN>::NPW]; i64 gA[RG<BT, UN>::NPW], gB[RG<BT, UN>::NPW]; };

// acc += a b.  The builtin, not asm: hipcc's hazard recognizer then pads the
// operand hazards (an asm MFMA here gave wrong products on 1.4 % of the entries:
// the wait states around its operand registers are nobody's job), and with the
// placement pinned by sched_barrier it allocates the accumulators in place (no
// v_accvgpr moves in the loop).
__device__ __forceinline__ void mfma_acc(f64x4& acc, double a, double b) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
}

// one k-step: NM MFMAs on `cur`; the next k-step's NR operand reads (k-step
// `srd` of the K-tile in rdA / rdB) into `nxt` over the first half of them; NP
// pieces u0.. of one unit into `st` over the second half
template <int BT, int UN, bool KCA, bool KCB, bool BUF, bool SB, int NP>
__device__ __forceinline__ void kstep(const GParams& p, i64 m0, i64 n0, int w, int l, int wr, int wc,
                                      const Pieces<BT, UN>& pc, const lds_char* __restrict__ rdA,
                                      const lds_char* __restrict__ rdB, int srd, lds_char* __restrict__ st,
                                      int u0, i64 k0, f64x4 (&acc)[RG<BT, UN>::MI][RG<BT, UN>::MI], const Ops<BT, UN>& cur,
                                      Ops<BT, UN>& nxt) {
    constexpr int MI = RG<BT, UN>::MI, NM = RG<BT, UN>::NM, NR = RG<BT, UN>::NR, WT = RG<BT, UN>::WT, H = NM / 2;
    // BT 128: reads one per MFMA of the first half, pieces SP apart in the second
    // half from its second MFMA on (at 2 pieces); BT 64: two reads per MFMA
    constexpr int RPM = NR / H;
    constexpr int SP = NP > 0 ? H / NP : 1, OFF = (SP > 1 && BT == 128) ? 1 : 0;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        mfma_acc(acc[i / MI][i % MI], cur.b[i % MI], cur.a[i / MI]);  // D^T: C rows across lanes
        if (i < H) {
#pragma unroll
            for (int q = 0; q < RPM; ++q) {
                const int f = i * RPM + q;
                if (f < MI) nxt.a[f] = ropnd<BT, UN, KCA>(rdA, wr * WT + f * 16, srd, l);
                else nxt.b[f - MI] = ropnd<BT, UN, KCB>(rdB, wc * WT + (f - MI) * 16, srd, l);
            }
        }
        if constexpr (NP > 0) {
            if (i >= H + OFF && (i - H - OFF) % SP == 0 && (i - H - OFF) / SP < NP) {
                const int u = u0 + (i - H - OFF) / SP;
                if constexpr (SB) piece<BT, UN, BUF, KCB>(p.B, p.ldb, n0, k0, pc.offB[u], pc.gB[u], w + 4 * u, st);
                else piece<BT, UN, BUF, KCA>(p.A, p.lda, m0, k0, pc.offA[u], pc.gA[u], w + 4 * u, st);
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the placement as written
    }
}
}  // namespace ring

template <int BT, int UN, bool KCA, bool KCB, bool BETA0, bool BUF>
__global__ __launch_bounds__(256, (ring::RG<BT, UN>::MINB)) void gemm_f64r_kernel(GParams p) {
    using namespace ring;
    using G = RG<BT, UN>;
    constexpr int RBK = G::RBK, UNIT = G::UNIT, WT = G::WT, MI = G::MI, NKS = G::NKS, NPW = G::NPW;
    constexpr int NPA = NPW / (NKS / 2);  // pieces of A_{t+2} per k-step over the first half
    __shared__ __attribute__((aligned(1024))) char lds_raw[NSLOT * UNIT];
    lds_char* lds = (lds_char*)lds_raw;
    const int tid = threadIdx.x, l = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 1, wc = w & 1;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, p.group_m, p.xcd_remap, tm, tn);
    const i64 m0 = (i64)tm * BT, n0 = (i64)tn * BT;
    {
        const i64 kz0 = (i64)blockIdx.y * p.kchunk;
        p.k = min(p.kchunk, p.k - kz0);
        p.A += KCA ? kz0 : kz0 * p.lda;
        p.B += KCB ? kz0 : kz0 * p.ldb;
        p.C += (i64)blockIdx.y * p.zstride;
    }
    Pieces<BT, UN> pc;
#pragma unroll
    for (int u = 0; u < NPW; ++u) {
        pc.gA[u] = piece_off<BT, UN, KCA>(w + 4 * u, l, m0, p.m, p.lda);
        pc.gB[u] = piece_off<BT, UN, KCB>(w + 4 * u, l, n0, p.n, p.ldb);
        pc.offA[u] = (int)(pc.gA[u] * 8);
        pc.offB[u] = (int)(pc.gB[u] * 8);
    }
    f64x4 acc[MI][MI];
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
        for (int b = 0; b < MI; ++b) acc[a][b] = f64x4{0, 0, 0, 0};

    const int nt = (int)(p.k / RBK);
    auto kt = [&](int t) { return (i64)min(t, nt - 1) * RBK; };
    // prologue: A_0, B_0, A_1, B_1 into slots 0..3; wait for A_0, B_0; operands (0,0)
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
    for (int q = 0; q < MI; ++q) {
        X.a[q] = ropnd<BT, UN, KCA>(lds, wr * WT + q * 16, 0, l);
        X.b[q] = ropnd<BT, UN, KCB>(lds + UNIT, wc * WT + q * 16, 0, l);
    }
    wait_cnt<NOWAIT_VM, 0>();
    auto ktile = [&](auto jc, int t) {
        constexpr int J = decltype(jc)::value;
        constexpr int sA = 2 * J % NSLOT, sB = (2 * J + 1) % NSLOT, sA1 = (2 * J + 2) % NSLOT,
                      sB1 = (2 * J + 3) % NSLOT, st0 = (2 * J + 4) % NSLOT, st1 = (2 * J + 5) % NSLOT;
        lds_char* rA = lds + sA * UNIT;
        lds_char* rB = lds + sB * UNIT;
        const i64 k2 = kt(t + 2);
        // (t,0..NKS-2): operands of (t,1..NKS-1) from A_t, B_t; the pieces of A_{t+2}
        // over the first NKS/2 k-steps (operands alternate X -> Y -> X; NKS is even)
        auto ks = [&](auto sc) {
            constexpr int S = decltype(sc)::value;
            constexpr int NP = S < NKS / 2 ? NPA : 0;
            if constexpr (S % 2 == 0)
                ring::kstep<BT, UN, KCA, KCB, BUF, false, NP>(p, m0, n0, w, l, wr, wc, pc, rA, rB, S + 1,
                                                          lds + st0 * UNIT, S * NPA, k2, acc, X, Y);
            else
                ring::kstep<BT, UN, KCA, KCB, BUF, false, NP>(p, m0, n0, w, l, wr, wc, pc, rA, rB, S + 1,
                                                          lds + st0 * UNIT, S * NPA, k2, acc, Y, X);
            if constexpr (S < NKS - 2) wait_cnt<NOWAIT_VM, 0>();
        };
        ks(std::integral_constant<int, 0>{});
        ks(std::integral_constant<int, 1>{});
        ks(std::integral_constant<int, 2>{});
        if constexpr (NKS == 8) {
            ks(std::integral_constant<int, 3>{});
            ks(std::integral_constant<int, 4>{});
            ks(std::integral_constant<int, 5>{});
            ks(std::integral_constant<int, 6>{});
        }
        wait_cnt<NPW, 0>();  // A_{t+1}, B_{t+1} landed (A_{t+2} may fly); reads of A_t, B_t retired
        dma_barrier();
        // (t,NKS-1): operands of (t+1,0) from A_{t+1}, B_{t+1}; B_{t+2} into A_t's slot
        ring::kstep<BT, UN, KCA, KCB, BUF, true, NPW>(p, m0, n0, w, l, wr, wc, pc, lds + sA1 * UNIT, lds + sB1 * UNIT,
                                                  0, lds + st1 * UNIT, 0, k2, acc, Y, X);
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

    // Epilogue: the MFMAs computed (op(A) op(B))^T blocks (B fragments as the
    // first operand), so lane l, register r of accumulator (mi, ni) holds C row
    // mi*16 + (l & 15), column ni*16 + (l >> 4) + 4 r: 16 lanes write 128
    // contiguous bytes of a column (v_mfma_f64_16x16x4_f64's D map is row =
    // (lane>>4) + 4 reg, col = lane & 15)
    const int g = l >> 4, c = l & 15;
    const i64 ib = m0 + wr * WT + c, jb = n0 + wc * WT + g;
    if (m0 + BT <= p.m && n0 + BT <= p.n) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
            double cv[MI][4];
            if (!BETA0) {
#pragma unroll
                for (int ni = 0; ni < MI; ++ni)
#pragma unroll
                    for (int r = 0; r < 4; ++r) cv[ni][r] = p.C[(jb + ni * 16 + 4 * r) * p.ldc + ib + mi * 16];
            }
#pragma unroll
            for (int ni = 0; ni < MI; ++ni)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double v = p.alpha * acc[mi][ni][r];
                    p.C[(jb + ni * 16 + 4 * r) * p.ldc + ib + mi * 16] = BETA0 ? v : v + p.beta * cv[ni][r];
                }
        }
        return;
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < MI; ++ni) {
            const i64 i = ib + mi * 16;
            if (i >= p.m) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 j = jb + ni * 16 + 4 * r;
                if (j < p.n) {
                    const double v = p.alpha * acc[mi][ni][r];
                    double* cp = p.C + j * p.ldc + i;
                    *cp = BETA0 ? v : v + p.beta * *cp;
                }
            }
        }
}

template <typename K>
hipError_t launch(K kernel, dim3 grid, int nt, const GParams& p, hipStream_t s) {
    hipLaunchKernelGGL(kernel, grid, dim3(nt), 0, s, p);
    return hipGetLastError();
}


template <typename SH, bool KCA, bool KCB, bool BUF>
hipError_t launch_b(const GParams& p, dim3 grid, hipStream_t s) {
    if (p.beta == 0.0) return launch(gemm_f64g_kernel<SH, KCA, KCB, true, BUF>, grid, SH::NT, p, s);
    return launch(gemm_f64g_kernel<SH, KCA, KCB, false, BUF>, grid, SH::NT, p, s);
}

template <typename SH, bool KCA, bool KCB>
hipError_t launch_g(GParams p, hipStream_t s) {
    p.tiles_m = (int)((p.m + SH::BM - 1) / SH::BM);
    p.tiles_n = (int)((p.n + SH::BN - 1) / SH::BN);
    const dim3 grid(p.tiles_m * p.tiles_n, (unsigned)((p.k + p.kchunk - 1) / p.kchunk));
    static const bool global_only = [] { const char* v = getenv("ELX_F64G_STAGE"); return v && v[0] == 'g'; }();
    if (!global_only && dma_fits(KCA ? SH::BM : SH::SK, p.lda, 8) && dma_fits(KCB ? SH::BN : SH::SK, p.ldb, 8))
        return launch_b<SH, KCA, KCB, true>(p, grid, s);
    return launch_b<SH, KCA, KCB, false>(p, grid, s);
}

template <int BT, int UN, bool KCA, bool KCB>
hipError_t launch_r(GParams p, hipStream_t s) {
    constexpr int RBK = ring::RG<BT, UN>::RBK;
    p.tiles_m = (int)((p.m + BT - 1) / BT);
    p.tiles_n = (int)((p.n + BT - 1) / BT);
    const dim3 grid(p.tiles_m * p.tiles_n, (unsigned)((p.k + p.kchunk - 1) / p.kchunk));
    // buffer-descriptor DMA when every offset of an image fits 31 bits, else the
    // global (64-bit address) form; ELX_F64G_STAGE=g forces the latter (read per call:
    // the tests cover it without operands of 2^21+ elements per row)
    const char* stg = getenv("ELX_F64G_STAGE");
    const bool buf = !(stg && stg[0] == 'g') && dma_fits(KCA ? BT : RBK, p.lda, 8) &&
                     dma_fits(KCB ? BT : RBK, p.ldb, 8);
    if (p.beta == 0.0) {
        if (buf) return launch(gemm_f64r_kernel<BT, UN, KCA, KCB, true, true>, grid, 256, p, s);
        return launch(gemm_f64r_kernel<BT, UN, KCA, KCB, true, false>, grid, 256, p, s);
    }
    if (buf) return launch(gemm_f64r_kernel<BT, UN, KCA, KCB, false, true>, grid, 256, p, s);
    return launch(gemm_f64r_kernel<BT, UN, KCA, KCB, false, false>, grid, 256, p, s);
}

template <typename SH>
hipError_t launch_shape(bool kca, bool kcb, const GParams& p, hipStream_t s) {
    if (kca) return kcb ? launch_g<SH, true, true>(p, s) : launch_g<SH, true, false>(p, s);
    return kcb ? launch_g<SH, false, true>(p, s) : launch_g<SH, false, false>(p, s);
}

bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

// 64 x 64 tiles where prefer_t64 (kernels.hpp) says they balance the CUs
// better; ELX_F64G_T64 = 0 never, 2 always (tests).  A grid of exactly 256
// 128-tiles (2048^2) takes the 128 ring when k is long (2048^2 x 16384: 75.9 vs
// 72.0 TF with the 64 ring) and the 64 ring, four workgroups per CU, when it is
// short (2048^3 NN 70.7 -> 71.6, TN 70.7 -> 71.8; profiles/r05ag_f64_t64_rule_ab.log).
// k: the depth the launch covers, compared as k / 32 * 32 so that the plan (k)
// and the launch (its kmain) decide alike.
bool t64_tiles(i64 m, i64 n, i64 k) {
    static const int v = [] { const char* e = getenv("ELX_F64G_T64"); return e ? atoi(e) : 1; }();
    if (v == 1 && (m + 127) / 128 * ((n + 127) / 128) == 256 && k / 32 * 32 <= 4096) return true;
    return prefer_t64(v, m, n, 255);
}

// the ring kernel's tile edge for this grid (0: the slab kernel).  128: the
// ring on every grid of 128-tiles; measured against the slab kernel in one
// process (profiles/r05o_ring_ab.log): 32768^3 NN 73.7 -> 74.0 TF, 16384^3 NN /
// TN / NT / TT 73.8 / 68.7 / 71.9 / 73.1 -> 74.6 / 76.1 / 72.6 / 74.3, 4096^3
// 70.4 -> 72.1 (and with the RC images in 256-B lines 76.5-76.7 in every
// orientation, profiles/r05aa_f64_rcblk_ab.log).  64: the 64 x 64 ring on grids
// of 64-tiles (four workgroups per CU), where it measured ahead of the slab
// kernel (profiles/r05af_f64_ring64_ab.log).  ELX_F64G_RING (read per call, for
// the A/B and the tests): bit 0 the 128 ring, bit 1 the 64 ring, 0 neither.
int ring_bt(i64 m, i64 n, i64 k) {
    const char* e = getenv("ELX_F64G_RING");
    const int v = e ? atoi(e) : RING64_DEFAULT ? 3 : 1;
    if (t64_tiles(m, n, k)) return (v & 2) ? 64 : 0;
    return (v & 1) ? 128 : 0;
}

}  // namespace

DmaPlan gemm_f64_lds_dma_plan(bool ta, bool tb, i64 m, i64 n, i64 k, const double* A, i64 lda, const double* B,
                              i64 ldb) {
    const bool kca = ta, kcb = !tb;
    const bool ok = k >= BK && al16(A) && al16(B) && lda % 2 == 0 && ldb % 2 == 0 && (kca || (m % 2 == 0 && m >= 2)) &&
                    (kcb || (n % 2 == 0 && n >= 2)) && m < (1ll << 31) && n < (1ll << 31);
    const int bt = ring_bt(m, n, k);
    if (bt == 128) return dma_plan(ok && k >= 32, (m + 127) / 128 * ((n + 127) / 128), k, 32, 256);
    if (t64_tiles(m, n, k)) return dma_plan(ok, (m + 63) / 64 * ((n + 63) / 64), k, BK, bt == 64 ? 1024 : 512);
    return dma_plan(ok, (m + 127) / 128 * ((n + 127) / 128), k, BK);
}

// C = alpha op(A)(:, :kmain) op(B)(:kmain, :) + beta C (kmain a multiple of 16, split
// into kchunk pieces over gridDim.y); the caller adds the k tail.
hipError_t gemm_f64_lds_dma(bool ta, bool tb, i64 m, i64 n, i64 kmain, i64 kchunk, double alpha, const double* A,
                            i64 lda, const double* B, i64 ldb, double beta, double* C, i64 ldc, hipStream_t s) {
    static const int gm = [] {  // >= 1: tile_of divides by it
        const char* v = getenv("ELX_F64G_GROUP");
        const int g = v ? atoi(v) : GROUP_M;
        return g >= 1 ? g : 1;
    }();
    static const int rm = [] { const char* v = getenv("ELX_F64G_REMAP"); return v ? atoi(v) : 1; }();
    GParams p{m, n, kmain, alpha, beta, A, lda, B, ldb, C, ldc, 0, 0, kchunk, m * n, gm, rm};
    // 64 x 64 tiles: eight waves of 32 x 16 where A is rows-contiguous (NN / NT:
    // 2048^3 NN 64.4 -> 66.2 TF, 1536 x 2048^2 62.5 -> 64.6, 1024^2 x 2048 49.9 ->
    // 54.8), four of 32 x 32 where it is k-contiguous (TN 64.4 vs 60.3 with eight,
    // TT 65.0 vs 62.2); profiles/r04_t64_waves8_ab.log (the fp32 kernel measured
    // 4-13 % slower with eight and keeps four).  ELX_F64G_T64W = 4 / 8 forces one.
    static const int t64w = [] { const char* v = getenv("ELX_F64G_T64W"); return v ? atoi(v) : 0; }();
    const int bt = ring_bt(m, n, kmain);
    if (bt == 128 && kmain % 32 == 0 && kchunk % 32 == 0) {
        if (ta) return !tb ? launch_r<128, 32768, true, true>(p, s) : launch_r<128, 32768, true, false>(p, s);
        return !tb ? launch_r<128, 32768, false, true>(p, s) : launch_r<128, 32768, false, false>(p, s);
    }
    if (bt == 64 && kmain % 16 == 0 && kchunk % 16 == 0) {
        if (ta) return !tb ? launch_r<64, 8192, true, true>(p, s) : launch_r<64, 8192, true, false>(p, s);
        return !tb ? launch_r<64, 8192, false, true>(p, s) : launch_r<64, 8192, false, false>(p, s);
    }
    if (t64_tiles(m, n, kmain)) {
        if (t64w == 8 || (t64w != 4 && !ta)) return launch_shape<Shape<64, 32, BK, 64, 16>>(ta, !tb, p, s);
        return launch_shape<Shape<64, 32, BK, 64, 32>>(ta, !tb, p, s);
    }
    // wave tile: 64 x 64 (four waves) measured +1.5-2 % for NN/TN/TT; NT (both
    // operands rows-contiguous) runs faster with 32 x 64 (profiles/r01_f64_wave.log)
    static const int wtm_env = [] { const char* v = getenv("ELX_F64G_WTM"); return v ? atoi(v) : 0; }();
    // and with at most one workgroup per CU (a grid of <= 256 tiles x chunks) the
    // eight-wave 32 x 64 split keeps two waves per SIMD: 2048^3 NN 61.0 -> 64.0 TF
    // (4096^3 and up: the four-wave split stays ahead; profiles/r03_f64_small.log).
    // (Measured and removed in round 4: 256-row tiles, 68.6-72.6 vs 74.1 TF at
    // 16384^3; 32-deep slabs for one-workgroup-per-CU grids, 53.8 vs 60.6 TF at
    // 2048^3, profiles/r03_f64_small.log; 64 x 128 tiles, no gain,
    // profiles/r04_small_shapes_ab.log; an LDS ring of 3 / 4 slabs for one
    // workgroup per CU, -5 % at 2048^3, profiles/r04_f64_ring_ab.log.)
    const i64 grid_wgs = (m + 127) / 128 * ((n + 127) / 128) * ((kmain + kchunk - 1) / kchunk);
    const int wtm = wtm_env ? wtm_env : ((!ta && tb) || grid_wgs <= 256) ? 32 : 64;
    if (wtm == 64) return launch_shape<Shape<128, 64>>(ta, !tb, p, s);
    return launch_shape<Shape<128>>(ta, !tb, p, s);
}

}  // namespace kern
}  // namespace elx
