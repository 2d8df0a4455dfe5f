// BLAS-1 / data-movement kernels for gfx950 (HBM-bound).
//
// Replace the reference's per-op device kernels and rocBLAS geam fallbacks:
//   copy2d_batch : Copy_GPU_impl copy_1d/copy_2d (src/hydrogen/blas/gpu/Copy.cu:13-205),
//                  Transpose_GPU_impl (src/hydrogen/blas/gpu/Transpose.cu:17-127),
//                  Axpy_GPU_impl incl. the transpose-tiled form (src/hydrogen/blas/gpu/Axpy.cu:20-189),
//                  and every hipMemcpy2DAsync pack/unpack of Copy/util.hpp:233-355 —
//                  ONE launch moves all r or c portions of a redistribution.
//   fill2d       : Fill_GPU_impl (src/hydrogen/blas/gpu/Fill.cu:20-76)
//   scale2d      : Scale_GPU_impl (src/hydrogen/blas/gpu/Scale.cu:17-81)
//   hadamard2d   : Hadamard_GPU_impl (src/hydrogen/blas/gpu/Hadamard.cu:16-117)
//   entrywise_map: EntrywiseMapImpl (include/hydrogen/blas/gpu/EntrywiseMapImpl.hpp:46-104)
//
// Every kernel is a 256-thread (4-wave) workgroup; lanes always walk the
// unit-stride dimension of whatever they read or write (64 lanes x elem = one
// or more full cache lines); a transposing move stages a 64x64 tile in LDS
// (pitch 65: conflict-free both ways).
#include <hip/hip_runtime.h>
#include "kernels.hpp"
#include "elem.hpp"
#include "../../../include/elemental_amd.h"
#include <algorithm>
#include <cstdlib>
#include <initializer_list>
#include <utility>

namespace elx {
namespace kern {

namespace {

constexpr int TILE = 64;
constexpr int NT = 256;
constexpr int UNROLL = 4;  // vectors in flight per lane in the elementwise engine

struct CopyBatch {
    Copy2D d[kMaxCopyBatch];
};

template <typename S>
struct V16 {
    static constexpr int N = 16 / sizeof(S);
    S v[N];
};

template <typename T, bool AXPY>
__global__ __launch_bounds__(NT) void copy2d_kernel(CopyBatch b, double alpha) {
    using E = Elem<T>;
    using S = typename E::storage;
    using Cmp = typename E::compute;
    __shared__ S tile[TILE][TILE + 1];  // [j][i]
    const Copy2D& d = b.d[blockIdx.y];
    const i64 tiles_i = (d.m + TILE - 1) / TILE, tiles_j = (d.n + TILE - 1) / TILE;
    const i64 ntiles = tiles_i * tiles_j;
    const S* src = static_cast<const S*>(d.src);
    S* dst = static_cast<S*>(d.dst);
    const bool src_i = (d.scs == 1) || (d.srs != 1);
    const bool dst_i = (d.dcs == 1) || (d.drs != 1);
    const int t = threadIdx.x, fast = t & (TILE - 1), slow = t >> 6;
    const Cmp a = (Cmp)alpha;
    // vector transposition: both operands 16-B aligned along their unit-stride
    // dimension (base pointer and the other dimension's stride)
    const i64 es = (i64)sizeof(S);
    const bool tvec = src_i != dst_i && (reinterpret_cast<uintptr_t>(src) % 16 == 0) &&
                      (reinterpret_cast<uintptr_t>(dst) % 16 == 0) && (src_i ? d.scs == 1 && (d.srs * es) % 16 == 0
                                                                               : d.srs == 1 && (d.scs * es) % 16 == 0) &&
                      (dst_i ? d.dcs == 1 && (d.drs * es) % 16 == 0 : d.drs == 1 && (d.dcs * es) % 16 == 0);
    for (i64 tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
        const i64 i0 = (tile_id % tiles_i) * TILE, j0 = (tile_id / tiles_i) * TILE;
        if (src_i == dst_i) {
            // both sides walk the same dimension: no staging needed
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const i64 i = i0 + (src_i ? fast : slow + 4 * e);
                const i64 j = j0 + (src_i ? slow + 4 * e : fast);
                if (i < d.m && j < d.n) {
                    const S v = src[i * d.scs + j * d.srs];
                    S* o = dst + i * d.dcs + j * d.drs;
                    if (AXPY) *o = E::store(E::load(*o) + a * E::load(v));
                    else *o = v;
                }
            }
        } else if (tvec && i0 + TILE <= d.m && j0 + TILE <= d.n) {
            // transposing, whole tile, 16-B aligned unit-stride runs on both sides:
            // one 16-B global access per lane (N elements) in and out, the
            // transposition done element-wise through the LDS tile
            constexpr int N = V16<S>::N, CH = TILE / N;
            __syncthreads();
#pragma unroll
            for (int v = t; v < TILE * CH; v += NT) {
                const int c = (v % CH) * N, sl = v / CH;
                const int li = src_i ? c : sl, lj = src_i ? sl : c;
                const V16<S> x = *reinterpret_cast<const V16<S>*>(src + (i0 + li) * d.scs + (j0 + lj) * d.srs);
#pragma unroll
                for (int e = 0; e < N; ++e) {
                    if (src_i) tile[lj][li + e] = x.v[e];
                    else tile[lj + e][li] = x.v[e];
                }
            }
            __syncthreads();
#pragma unroll
            for (int v = t; v < TILE * CH; v += NT) {
                const int c = (v % CH) * N, sl = v / CH;
                const int li = dst_i ? c : sl, lj = dst_i ? sl : c;
                V16<S>* o = reinterpret_cast<V16<S>*>(dst + (i0 + li) * d.dcs + (j0 + lj) * d.drs);
                V16<S> x;
#pragma unroll
                for (int e = 0; e < N; ++e) x.v[e] = dst_i ? tile[lj][li + e] : tile[lj + e][li];
                if (AXPY) {
                    V16<S> y = *o;
#pragma unroll
                    for (int e = 0; e < N; ++e) y.v[e] = E::store(E::load(y.v[e]) + a * E::load(x.v[e]));
                    *o = y;
                } else {
                    *o = x;
                }
            }
        } else {
            __syncthreads();
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const int li = src_i ? fast : slow + 4 * e;
                const int lj = src_i ? slow + 4 * e : fast;
                const i64 i = i0 + li, j = j0 + lj;
                if (i < d.m && j < d.n) tile[lj][li] = src[i * d.scs + j * d.srs];
            }
            __syncthreads();
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const int li = dst_i ? fast : slow + 4 * e;
                const int lj = dst_i ? slow + 4 * e : fast;
                const i64 i = i0 + li, j = j0 + lj;
                if (i < d.m && j < d.n) {
                    S* o = dst + i * d.dcs + j * d.drs;
                    if (AXPY) *o = E::store(E::load(*o) + a * E::load(tile[lj][li]));
                    else *o = tile[lj][li];
                }
            }
        }
    }
}

// Rank-ordered contraction sum (kernels.hpp ContractSum): rows over the lanes
// of gridDim.x workgroups (N = 16 B / element per lane), columns over
// gridDim.y.  Every source is read once and dst once each way; with unit row
// stride and 16-B aligned columns on every operand each access is one 16-B
// vector.  The source loop is fully unrolled so the descriptor's arrays are
// indexed by constants (kernel arguments, never a private copy).
template <typename T>
__global__ __launch_bounds__(NT) void contract_sum_kernel(ContractSum c, double alpha) {
    using E = Elem<T>;
    using S = typename E::storage;
    constexpr int N = V16<S>::N;
    const auto a = (typename E::compute)alpha;
    S* dst = static_cast<S*>(c.dst);
    auto al16 = [](const void* p, i64 ld) {
        return reinterpret_cast<uintptr_t>(p) % 16 == 0 && (ld * (i64)sizeof(S)) % 16 == 0;
    };
    bool vec = c.dcs == 1 && al16(dst, c.n > 1 ? c.drs : 0);
#pragma unroll
    for (int q = 0; q < kMaxContractSources; ++q)
        if (q < c.nsrc) vec = vec && c.scs[q] == 1 && al16(c.src[q], c.n > 1 ? c.srs[q] : 0);
    const i64 mv = (c.m + N - 1) / N;
    for (i64 j = blockIdx.y; j < c.n; j += gridDim.y) {
        for (i64 iv = (i64)blockIdx.x * NT + threadIdx.x; iv < mv; iv += (i64)gridDim.x * NT) {
            const i64 i = iv * N;
            S* y = dst + j * c.drs + i * c.dcs;
            if (vec && i + N <= c.m) {
                V16<S> x[kMaxContractSources];
#pragma unroll
                for (int q = 0; q < kMaxContractSources; ++q)
                    if (q < c.nsrc) x[q] = *reinterpret_cast<const V16<S>*>(static_cast<const S*>(c.src[q]) + j * c.srs[q] + i);
                V16<S> acc = *reinterpret_cast<const V16<S>*>(y);
#pragma unroll
                for (int q = 0; q < kMaxContractSources; ++q)
                    if (q < c.nsrc) {
#pragma unroll
                        for (int e = 0; e < N; ++e) acc.v[e] = E::store(E::load(acc.v[e]) + a * E::load(x[q].v[e]));
                    }
                *reinterpret_cast<V16<S>*>(y) = acc;
            } else {
                for (int e = 0; e < N && i + e < c.m; ++e) {
                    S acc = y[e * c.dcs];
#pragma unroll
                    for (int q = 0; q < kMaxContractSources; ++q)
                        if (q < c.nsrc) {
                            const S xv = static_cast<const S*>(c.src[q])[j * c.srs[q] + (i + e) * c.scs[q]];
                            acc = E::store(E::load(acc) + a * E::load(xv));
                        }
                    y[e * c.dcs] = acc;
                }
            }
        }
    }
}

// Type-converting strided copy (Copy_GPU_impl<SrcT,DestT>, Copy.cu:93-205):
// the same two shapes as copy2d_kernel (direct when both sides walk the same
// unit-stride dimension, LDS-staged 64x64 tile otherwise); the tile holds the
// converted destination values.
template <typename TS, typename TD>
__global__ __launch_bounds__(NT) void convert2d_kernel(Copy2D d) {
    using SS = typename Elem<TS>::storage;
    using SD = typename Elem<TD>::storage;
    __shared__ SD tile[TILE][TILE + 1];  // [j][i]
    const i64 tiles_i = (d.m + TILE - 1) / TILE, tiles_j = (d.n + TILE - 1) / TILE;
    const SS* src = static_cast<const SS*>(d.src);
    SD* dst = static_cast<SD*>(d.dst);
    const bool src_i = (d.scs == 1) || (d.srs != 1);
    const bool dst_i = (d.dcs == 1) || (d.drs != 1);
    const int t = threadIdx.x, fast = t & (TILE - 1), slow = t >> 6;
    for (i64 tile_id = blockIdx.x; tile_id < tiles_i * tiles_j; tile_id += gridDim.x) {
        const i64 i0 = (tile_id % tiles_i) * TILE, j0 = (tile_id / tiles_i) * TILE;
        if (src_i == dst_i) {
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const i64 i = i0 + (src_i ? fast : slow + 4 * e);
                const i64 j = j0 + (src_i ? slow + 4 * e : fast);
                if (i < d.m && j < d.n) dst[i * d.dcs + j * d.drs] = convert_elem<TS, TD>(src[i * d.scs + j * d.srs]);
            }
        } else {
            __syncthreads();
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const int li = src_i ? fast : slow + 4 * e;
                const int lj = src_i ? slow + 4 * e : fast;
                const i64 i = i0 + li, j = j0 + lj;
                if (i < d.m && j < d.n) tile[lj][li] = convert_elem<TS, TD>(src[i * d.scs + j * d.srs]);
            }
            __syncthreads();
#pragma unroll 4
            for (int e = 0; e < TILE / 4; ++e) {
                const int li = dst_i ? fast : slow + 4 * e;
                const int lj = dst_i ? slow + 4 * e : fast;
                const i64 i = i0 + li, j = j0 + lj;
                if (i < d.m && j < d.n) dst[i * d.dcs + j * d.drs] = tile[lj][li];
            }
        }
    }
}

// Vectorized 2-D elementwise engine (HBM-bound ops).  Columns over gridDim.y,
// rows over gridDim.x*NT lanes, each lane moving VEC = 16 B / sizeof(S)
// elements per access (one global_load/store_dwordx4) when every operand's
// column starts are 16-B aligned (uniform per launch); otherwise element by
// element.  The host collapses contiguous operands (ld == m) into one column.

// Operand 0 is the output; RD0 says whether the op reads it (scale) or only
// writes it (fill, hadamard, map), so no HBM read is spent on a pure output.
template <typename S, int NOP, bool RD0, typename F>
__device__ __forceinline__ void ew_2d(i64 m, i64 n, S* const (&ptr)[NOP], const i64 (&ld)[NOP], bool vec, F&& f) {
    constexpr int N = V16<S>::N;
    constexpr i64 CHUNK = (i64)NT * UNROLL * N;  // elements per workgroup pass of a column
    for (i64 j = blockIdx.y; j < n; j += gridDim.y) {
        S* col[NOP];
#pragma unroll
        for (int q = 0; q < NOP; ++q) col[q] = ptr[q] + j * ld[q];
        for (i64 c0 = (i64)blockIdx.x * CHUNK; c0 < m; c0 += (i64)gridDim.x * CHUNK) {
            if (vec && c0 + CHUNK <= m) {
                // UNROLL independent 16-B accesses per operand in flight per lane,
                // the workgroup sweeping one contiguous CHUNK
                V16<S> x[NOP][UNROLL];
#pragma unroll
                for (int u = 0; u < UNROLL; ++u)
#pragma unroll
                    for (int q = RD0 ? 0 : 1; q < NOP; ++q)
                        x[q][u] = *reinterpret_cast<const V16<S>*>(col[q] + c0 + (u * NT + threadIdx.x) * N);
#pragma unroll
                for (int u = 0; u < UNROLL; ++u)
#pragma unroll
                    for (int e = 0; e < N; ++e) {
                        S r[NOP];
#pragma unroll
                        for (int q = RD0 ? 0 : 1; q < NOP; ++q) r[q] = x[q][u].v[e];
                        x[0][u].v[e] = f(r);
                    }
#pragma unroll
                for (int u = 0; u < UNROLL; ++u)
                    *reinterpret_cast<V16<S>*>(col[0] + c0 + (u * NT + threadIdx.x) * N) = x[0][u];
            } else {
                const i64 end = c0 + CHUNK < m ? c0 + CHUNK : m;
                for (i64 i = c0 + (i64)threadIdx.x * N; i < end; i += (i64)NT * N) {
                    if (vec && i + N <= end) {
                        V16<S> x[NOP];
#pragma unroll
                        for (int q = RD0 ? 0 : 1; q < NOP; ++q) x[q] = *reinterpret_cast<const V16<S>*>(col[q] + i);
#pragma unroll
                        for (int e = 0; e < N; ++e) {
                            S r[NOP];
#pragma unroll
                            for (int q = RD0 ? 0 : 1; q < NOP; ++q) r[q] = x[q].v[e];
                            x[0].v[e] = f(r);
                        }
                        *reinterpret_cast<V16<S>*>(col[0] + i) = x[0];
                    } else {
                        for (i64 e = i; e < i + N && e < end; ++e) {
                            S r[NOP];
#pragma unroll
                            for (int q = RD0 ? 0 : 1; q < NOP; ++q) r[q] = col[q][e];
                            col[0][e] = f(r);
                        }
                    }
                }
            }
        }
    }
}

// Batched column-contiguous moves (scs == dcs == 1: axpy, copy, and every
// pack/unpack whose portions are whole column runs): the descriptor's
// n x ceil(m/VEC) vectors are dealt over the workgroups of its blockIdx.y row.
template <typename T, bool AXPY>
__global__ __launch_bounds__(NT) void copy_cols_kernel(CopyBatch b, double alpha) {
    using E = Elem<T>;
    using S = typename E::storage;
    constexpr int N = V16<S>::N;
    const Copy2D& d = b.d[blockIdx.y];
    const S* src = static_cast<const S*>(d.src);
    S* dst = static_cast<S*>(d.dst);
    const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16 == 0) &&
                     ((d.srs * (i64)sizeof(S)) % 16 == 0 || d.n == 1) && ((d.drs * (i64)sizeof(S)) % 16 == 0 || d.n == 1);
    const auto a = (typename E::compute)alpha;
    const i64 mv = (d.m + N - 1) / N, total = mv * d.n;
    // column of a vector id: 32-bit division when the ids fit (64-bit division is
    // a long emulated sequence), none at all for a single column
    const bool one_col = d.n == 1, narrow = total < (1ll << 31);
    auto col_of = [&](i64 id) -> i64 {
        return one_col ? 0 : narrow ? (i64)((uint32_t)id / (uint32_t)mv) : id / mv;
    };
    auto one = [&](i64 id) {
        const i64 j = col_of(id), i = (id - j * mv) * N;
        const S* x = src + j * d.srs + i;
        S* y = dst + j * d.drs + i;
        if (vec && i + N <= d.m) {
            const V16<S> xv = *reinterpret_cast<const V16<S>*>(x);
            if (AXPY) {
                V16<S> yv = *reinterpret_cast<const V16<S>*>(y);
#pragma unroll
                for (int e = 0; e < N; ++e) yv.v[e] = E::store(E::load(yv.v[e]) + a * E::load(xv.v[e]));
                *reinterpret_cast<V16<S>*>(y) = yv;
            } else {
                *reinterpret_cast<V16<S>*>(y) = xv;
            }
        } else {
            for (i64 e = 0; e < N && i + e < d.m; ++e) {
                if (AXPY) y[e] = E::store(E::load(y[e]) + a * E::load(x[e]));
                else y[e] = x[e];
            }
        }
    };
    constexpr i64 CHUNK = (i64)NT * UNROLL;  // vectors per workgroup pass
    for (i64 c0 = (i64)blockIdx.x * CHUNK; c0 < total; c0 += (i64)gridDim.x * CHUNK) {
        if (vec && d.m % N == 0 && c0 + CHUNK <= total) {
            // every vector whole: UNROLL independent loads in flight before any store
            V16<S> xv[UNROLL], yv[UNROLL];
            S* y[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const i64 k = c0 + u * NT + threadIdx.x, j = col_of(k), i = (k - j * mv) * N;
                xv[u] = *reinterpret_cast<const V16<S>*>(src + j * d.srs + i);
                y[u] = dst + j * d.drs + i;
                if (AXPY) yv[u] = *reinterpret_cast<const V16<S>*>(y[u]);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                if (AXPY) {
#pragma unroll
                    for (int e = 0; e < N; ++e) yv[u].v[e] = E::store(E::load(yv[u].v[e]) + a * E::load(xv[u].v[e]));
                    *reinterpret_cast<V16<S>*>(y[u]) = yv[u];
                } else {
                    *reinterpret_cast<V16<S>*>(y[u]) = xv[u];
                }
            }
        } else {
            for (i64 k = c0 + threadIdx.x; k < c0 + CHUNK && k < total; k += NT) one(k);
        }
    }
}

// Transposing moves with 16-B aligned unit-stride runs on both sides (the
// `tvec` case of copy2d_kernel), without LDS: each lane owns R blocks of N x N
// elements (N = 16 B / element, R = 16 / N, so 16 vectors in flight per lane),
// reads each as N 16-B vectors along the source's unit-stride dimension,
// transposes it in registers and writes N 16-B vectors along the
// destination's.  A wave tile is 8N (source unit-stride) x 8NR elements: lane
// (bu, bv) = (l & 7, l >> 3) owns the blocks (bu, bv + 8r), so every load and
// every store instruction touches 8 full 128-B runs.  Wave tiles are dealt
// over all waves of the grid; ragged ones move element by element.  For
// 16-bit data this replaces 16 two-byte LDS accesses per 16 B moved.
template <typename T, bool AXPY>
__global__ __launch_bounds__(NT) void transpose_vec_kernel(CopyBatch b, double alpha) {
    using E = Elem<T>;
    using S = typename E::storage;
    constexpr int N = V16<S>::N, R = 16 / N, WU = 8 * N, WV = 8 * N * R;
    const Copy2D& d = b.d[blockIdx.y];
    const S* src = static_cast<const S*>(d.src);
    S* dst = static_cast<S*>(d.dst);
    const bool src_i = d.scs == 1;  // source unit stride along i (then the destination's along j)
    // (u, v) = (source unit-stride index, the other); element (u, v) of source / destination
    const i64 su = src_i ? d.m : d.n, sv = src_i ? d.n : d.m;
    const i64 s_v = src_i ? d.srs : d.scs;        // source stride of v
    const i64 d_u = src_i ? d.dcs : d.drs;        // destination stride of u
    const auto a = (typename E::compute)alpha;
    const int l = threadIdx.x & 63, bu = l & 7, bv = l >> 3;
    const i64 tu = (su + WU - 1) / WU, ntiles = tu * ((sv + WV - 1) / WV);
    const i64 wave = (i64)blockIdx.x * (NT / 64) + (threadIdx.x >> 6), nwaves = (i64)gridDim.x * (NT / 64);
    for (i64 t = wave; t < ntiles; t += nwaves) {
        const i64 u0 = (t % tu) * WU, v0 = (t / tu) * WV;
        if (u0 + WU <= su && v0 + WV <= sv) {
            const i64 u = u0 + N * bu;
            V16<S> x[R][N];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int e = 0; e < N; ++e)
                    x[r][e] = *reinterpret_cast<const V16<S>*>(src + u + (v0 + N * (bv + 8 * r) + e) * s_v);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const i64 v = v0 + N * (bv + 8 * r);
#pragma unroll
                for (int g = 0; g < N; ++g) {
                    V16<S>* o = reinterpret_cast<V16<S>*>(dst + v + (u + g) * d_u);
                    V16<S> y;
#pragma unroll
                    for (int e = 0; e < N; ++e) y.v[e] = x[r][e].v[g];
                    if (AXPY) {
                        V16<S> z = *o;
#pragma unroll
                        for (int e = 0; e < N; ++e) z.v[e] = E::store(E::load(z.v[e]) + a * E::load(y.v[e]));
                        *o = z;
                    } else {
                        *o = y;
                    }
                }
            }
        } else {
            for (int q = l; q < WU * WV; q += 64) {
                const i64 u = u0 + (q % WU), v = v0 + (q / WU);
                if (u < su && v < sv) {
                    const S xv = src[u + v * s_v];
                    S* o = dst + v + u * d_u;
                    if (AXPY) *o = E::store(E::load(*o) + a * E::load(xv));
                    else *o = xv;
                }
            }
        }
    }
}

// 2-D elementwise driver (fill_hash): columns over gridDim.y, rows over gridDim.x*NT.
template <typename F>
__device__ __forceinline__ void for_each_2d(i64 m, i64 n, F&& f) {
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        for (i64 i = (i64)blockIdx.x * NT + threadIdx.x; i < m; i += (i64)gridDim.x * NT) f(i, j);
}

// operand 0 is the output (read too by scale; for fill/hadamard/map its value is ignored)
template <typename T>
__global__ __launch_bounds__(NT) void fill_kernel(i64 m, i64 n, double v, typename Elem<T>::storage* A, i64 lda,
                                                  bool vec) {
    using E = Elem<T>;
    using S = typename E::storage;
    const S s = E::store((typename E::compute)v);
    S* const p[1] = {A};
    const i64 l[1] = {lda};
    ew_2d<S, 1, false>(m, n, p, l, vec, [&](const S(&)[1]) { return s; });
}

template <typename T>
__global__ __launch_bounds__(NT) void scale_kernel(i64 m, i64 n, double alpha, typename Elem<T>::storage* A, i64 lda,
                                                   bool vec) {
    using E = Elem<T>;
    using S = typename E::storage;
    const auto a = (typename E::compute)alpha;
    S* const p[1] = {A};
    const i64 l[1] = {lda};
    ew_2d<S, 1, true>(m, n, p, l, vec, [&](const S(&x)[1]) { return E::store(a * E::load(x[0])); });
}

template <typename T>
__global__ __launch_bounds__(NT) void hadamard_kernel(i64 m, i64 n, const typename Elem<T>::storage* A, i64 lda,
                                                      const typename Elem<T>::storage* B, i64 ldb,
                                                      typename Elem<T>::storage* C, i64 ldc, bool vec) {
    using E = Elem<T>;
    using S = typename E::storage;
    // in-place aliasing (C==A or C==B) is safe: each element is read before its own write
    S* const p[3] = {C, const_cast<S*>(A), const_cast<S*>(B)};
    const i64 l[3] = {ldc, lda, ldb};
    ew_2d<S, 3, false>(m, n, p, l, vec, [&](const S(&x)[3]) { return E::store(E::load(x[1]) * E::load(x[2])); });
}

template <typename C>
__device__ __forceinline__ C apply_map(int fn, C x) {
    switch (fn) {
    case ELX_MAP_IDENTITY: return x;
    case ELX_MAP_NEGATE: return -x;
    case ELX_MAP_ABS: return x < C(0) ? -x : x;
    case ELX_MAP_SQUARE: return x * x;
    case ELX_MAP_SQRT: return sqrt(x);
    case ELX_MAP_EXP: return exp(x);
    case ELX_MAP_LOG: return log(x);
    case ELX_MAP_RELU: return x > C(0) ? x : C(0);
    case ELX_MAP_SIGMOID: return C(1) / (C(1) + exp(-x));
    case ELX_MAP_RECIP: return C(1) / x;
    case ELX_MAP_TANH: return tanh(x);
    default: return x;
    }
}

template <typename T, int FN>
__global__ __launch_bounds__(NT) void map_kernel(i64 m, i64 n, const typename Elem<T>::storage* A, i64 lda,
                                                 typename Elem<T>::storage* B, i64 ldb, bool vec) {
    using E = Elem<T>;
    using S = typename E::storage;
    S* const p[2] = {B, const_cast<S*>(A)};
    const i64 l[2] = {ldb, lda};
    ew_2d<S, 2, false>(m, n, p, l, vec, [&](const S(&x)[2]) { return E::store(apply_map(FN, E::load(x[1]))); });
}

template <typename C>
__device__ __forceinline__ C apply_combine(int fn, C a, C b) {
    switch (fn) {
    case ELX_COMBINE_ADD: return a + b;
    case ELX_COMBINE_SUB: return b - a;
    case ELX_COMBINE_MUL: return a * b;
    case ELX_COMBINE_DIV: return b / a;
    case ELX_COMBINE_MAX: return a > b ? a : b;
    case ELX_COMBINE_MIN: return a < b ? a : b;
    case ELX_COMBINE_RELU_GRAD: return a > C(0) ? b : C(0);
    default: return b;
    }
}

// B := f(A, B) (CombineImpl.hpp:47-213): operand 0 is B, read and written
template <typename T, int FN>
__global__ __launch_bounds__(NT) void combine_kernel(i64 m, i64 n, const typename Elem<T>::storage* A, i64 lda,
                                                     typename Elem<T>::storage* B, i64 ldb, bool vec) {
    using E = Elem<T>;
    using S = typename E::storage;
    S* const p[2] = {B, const_cast<S*>(A)};
    const i64 l[2] = {ldb, lda};
    ew_2d<S, 2, true>(m, n, p, l, vec,
                      [&](const S(&x)[2]) { return E::store(apply_combine(FN, E::load(x[1]), E::load(x[0]))); });
}

template <typename T>
__global__ __launch_bounds__(NT) void hash_kernel(i64 m, i64 n, typename Elem<T>::storage* A, i64 lda, i64 i0,
                                                  i64 istride, i64 j0, i64 jstride, uint64_t seed,
                                                  double center, double radius) {
    using E = Elem<T>;
    for_each_2d(m, n, [&](i64 i, i64 j) {
#pragma clang fp contract(off)
        const double u = hash_unit(seed, i0 + i * istride, j0 + j * jstride);
        // explicit roundings: no FMA contraction, so host and device agree bit for bit
        // plain operators under `contract(off)`: the instructions are created in
        // this scope, so no fused multiply-add can merge them (host == device)
        const double v = center + radius * (2.0 * u - 1.0);
        A[i + j * lda] = E::store((typename E::compute)v);  // double -> compute (RNE) -> storage (RNE)
    });
}

// Trapezoid update (ScaleTrapezoid.hpp:47-88, AxpyTrapezoid, LocalTrrk's
// diagonal blocks in Trrk/Local.hpp:155-210).  Element (i,j) of the local block
// is global (i0 + i*istride, j0 + j*jstride); inside the trapezoid
// (lower: gi >= gj - offset, upper: gi <= gj - offset) it becomes
// beta*Y + alpha*X (X may be null: beta*Y; with X and beta == 0, alpha*X without
// reading Y), outside it is neither read nor written.
template <typename T>
__global__ __launch_bounds__(NT) void trapezoid_kernel(bool lower, i64 m, i64 n, double alpha,
                                                       const typename Elem<T>::storage* X, i64 ldx, double beta,
                                                       typename Elem<T>::storage* Y, i64 ldy, i64 i0, i64 istride,
                                                       i64 j0, i64 jstride, i64 offset) {
    using E = Elem<T>;
    using Cm = typename E::compute;
    const Cm a = (Cm)alpha, b = (Cm)beta;
    for_each_2d(m, n, [&](i64 i, i64 j) {
        const i64 gi = i0 + i * istride, gj = j0 + j * jstride - offset;
        if (lower ? gi < gj : gi > gj) return;
        // with X and beta == 0, Y is not read (a trapezoid copy: NaNs there do not survive)
        Cm y = (X && beta == 0.0) ? Cm(0) : b * E::load(Y[i + j * ldy]);
        if (X) y = y + a * E::load(X[i + j * ldx]);
        Y[i + j * ldy] = E::store(y);
    });
}

// Launch geometry of ew_2d: collapse to one column when every operand is
// contiguous (ld == m), and decide the 16-B vector path.
struct EwShape {
    i64 m, n;
    bool vec;
    dim3 grid;
};
template <typename S>
EwShape ew_shape(i64 m, i64 n, std::initializer_list<std::pair<const void*, i64>> ops) {
    bool contig = true, vec = true;
    for (auto& o : ops) {
        contig = contig && (o.second == m || n == 1);
        vec = vec && (reinterpret_cast<uintptr_t>(o.first) % 16 == 0);
    }
    if (contig) { m *= n; n = 1; }
    for (auto& o : ops) vec = vec && (n == 1 || (o.second * (i64)sizeof(S)) % 16 == 0);
    constexpr int N = 16 / sizeof(S);
    // one pass: every workgroup sweeps one CHUNK of one column
    i64 gx = (m + (i64)NT * N * UNROLL - 1) / ((i64)NT * N * UNROLL);
    const i64 gy = n < 1 ? 1 : (n > 65535 ? 65535 : n);
    gx = std::max<i64>(1, std::min<i64>(gx, (1ll << 31) - 1));
    return EwShape{m, n, vec, dim3((unsigned)gx, (unsigned)gy)};
}

dim3 grid2d(i64 m, i64 n) {
    i64 gx = (m + NT - 1) / NT;
    if (gx > 64) gx = 64;
    if (gx < 1) gx = 1;
    i64 gy = n < 1 ? 1 : n;
    if (gy > 4096) gy = 4096;
    return dim3((unsigned)gx, (unsigned)gy);
}

#define ELX_DTYPE_SWITCH(dtype, T, ...)                 \
    switch (dtype) {                                    \
    case ELX_F64: { using T = double; __VA_ARGS__; break; } \
    case ELX_F32: { using T = float; __VA_ARGS__; break; }  \
    case ELX_F16: { using T = f16_t; __VA_ARGS__; break; }  \
    case ELX_BF16: { using T = bf16_t; __VA_ARGS__; break; } \
    default: return hipErrorInvalidValue;               \
    }

// A transposing descriptor whose unit-stride runs are 16-B aligned on both
// sides (the condition of copy2d_kernel's `tvec` branch): transpose_vec_kernel.
bool TransposeVec(const Copy2D& x, int es) {
    const bool src_i = x.scs == 1, dst_i = x.dcs == 1;
    if (src_i == dst_i || (src_i ? false : x.srs != 1) || (dst_i ? false : x.drs != 1)) return false;
    if (((reinterpret_cast<uintptr_t>(x.src) | reinterpret_cast<uintptr_t>(x.dst)) % 16) != 0) return false;
    const i64 sother = src_i ? x.srs : x.scs, dother = dst_i ? x.drs : x.dcs;
    return (sother * es) % 16 == 0 && (dother * es) % 16 == 0;
}

// ELX_TRANSPOSE_LDS=1: the LDS-tile transposition of copy2d_kernel for 16-bit data too (A/B timing)
bool TransposeViaLds() {
    static const bool v = [] { const char* e = getenv("ELX_TRANSPOSE_LDS"); return e && e[0] == '1'; }();
    return v;
}

// Frobenius-norm partials in double, one per workgroup: MODE 0 the largest
// |a| (NaN wins), MODE 1 the sum of (a / scale)^2 (El::FrobeniusNorm's scaled
// sum of squares, src/lapack_like/props/Norm/Frobenius.cpp:37-44, with the
// grid-wide max as the one scale)
__device__ __forceinline__ double norm_max(double a, double b) { return a != a ? a : b != b ? b : (a > b ? a : b); }

template <typename T, int MODE>
__global__ __launch_bounds__(NT) void norm_partial_kernel(i64 m, i64 n, const typename Elem<T>::storage* A, i64 lda,
                                                          double scale, double* out) {
    using E = Elem<T>;
    double acc = 0.0;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        for (i64 i = (i64)blockIdx.x * NT + threadIdx.x; i < m; i += (i64)gridDim.x * NT) {
            const double x = (double)E::load(A[i + j * lda]);
            if (MODE == 0) {
                acc = norm_max(acc, x < 0 ? -x : x);
            } else {
                const double y = x / scale;
                acc += y * y;
            }
        }
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_xor(acc, off, 64);
        acc = MODE == 0 ? norm_max(acc, o) : acc + o;
    }
    __shared__ double wave[NT / 64];
    if ((threadIdx.x & 63) == 0) wave[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = wave[0];
        for (int w = 1; w < NT / 64; ++w) r = MODE == 0 ? norm_max(r, wave[w]) : r + wave[w];
        out[(i64)blockIdx.y * gridDim.x + blockIdx.x] = r;
    }
}

}  // namespace

hipError_t copy2d_batch(int dtype, const Copy2D* d, int nd, bool axpy, double alpha, hipStream_t s, int max_wgs) {
    for (int base = 0; base < nd; base += kMaxCopyBatch) {
        CopyBatch b{};
        const int cnt = (nd - base) < kMaxCopyBatch ? (nd - base) : kMaxCopyBatch;
        i64 maxtiles = 0, maxvec = 0, maxwt = 0;
        int used = 0;
        bool cols = true, tvec_all = true;
        const int es = dtype == ELX_F64 ? 8 : dtype == ELX_F32 ? 4 : 2;
        for (int q = 0; q < cnt; ++q) {
            Copy2D x = d[base + q];
            if (x.m <= 0 || x.n <= 0) continue;
            if (x.scs == 1 && x.dcs == 1 && x.srs == x.m && x.drs == x.m && x.n > 1) {
                x.m *= x.n;  // both sides contiguous: one long column
                x.n = 1;
                x.srs = x.drs = x.m;
            }
            b.d[used++] = x;
            const i64 t = ((x.m + TILE - 1) / TILE) * ((x.n + TILE - 1) / TILE);
            if (t > maxtiles) maxtiles = t;
            const i64 v = (x.m + 16 / es - 1) / (16 / es) * x.n;
            if (v > maxvec) maxvec = v;
            cols = cols && x.scs == 1 && x.dcs == 1;
            tvec_all = tvec_all && TransposeVec(x, es);
            const i64 w = 8 * (16 / es);  // wave tile: w x 128 elements
            const i64 wt = ((x.m + w - 1) / w) * ((x.n + 127) / 128);
            if (wt > maxwt) maxwt = wt;
        }
        if (used == 0) continue;
        // workgroups per descriptor row of the grid under the caller's cap
        const i64 cap = max_wgs > 0 ? std::max<i64>(1, max_wgs / used) : (i64)1 << 30;
        // 16-bit: register blocks (4.08 vs 3.59 TB/s at 16384 x 8192); f32 / f64
        // keep the LDS tile, which measured faster for them (4.71 vs 4.19, 5.04
        // vs 4.93 TB/s; profiles/r02_transpose_ab.log)
        if (!cols && tvec_all && es == 2 && !TransposeViaLds()) {
            // ~8 workgroups per CU: 32 waves per CU over the batch's wave tiles
            const unsigned gx = (unsigned)std::max<i64>(1, std::min<i64>(std::min<i64>((maxwt + 3) / 4, 2048), cap));
            dim3 grid(gx, used);
            ELX_DTYPE_SWITCH(dtype, T,
                if (axpy) hipLaunchKernelGGL((transpose_vec_kernel<T, true>), grid, dim3(NT), 0, s, b, alpha);
                else hipLaunchKernelGGL((transpose_vec_kernel<T, false>), grid, dim3(NT), 0, s, b, alpha));
        } else if (cols) {
            // ~16 workgroups per CU across the batch
            const i64 gx = std::max<i64>(1, std::min<i64>(std::min<i64>((maxvec + NT * UNROLL - 1) / (NT * UNROLL), 1 << 20), cap));
            dim3 grid((unsigned)gx, used);
            ELX_DTYPE_SWITCH(dtype, T,
                if (axpy) hipLaunchKernelGGL((copy_cols_kernel<T, true>), grid, dim3(NT), 0, s, b, alpha);
                else hipLaunchKernelGGL((copy_cols_kernel<T, false>), grid, dim3(NT), 0, s, b, alpha));
        } else {
            const unsigned gx = (unsigned)std::max<i64>(1, std::min<i64>(maxtiles > 4096 ? 4096 : maxtiles, cap));
            dim3 grid(gx, used);
            ELX_DTYPE_SWITCH(dtype, T,
                if (axpy) hipLaunchKernelGGL((copy2d_kernel<T, true>), grid, dim3(NT), 0, s, b, alpha);
                else hipLaunchKernelGGL((copy2d_kernel<T, false>), grid, dim3(NT), 0, s, b, alpha));
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t contract_sum(int dtype, const ContractSum& c, double alpha, hipStream_t s, int max_wgs) {
    if (c.m <= 0 || c.n <= 0 || c.nsrc <= 0) return hipSuccess;
    if (c.nsrc > kMaxContractSources) return hipErrorInvalidValue;
    const int es = dtype == ELX_F64 ? 8 : dtype == ELX_F32 ? 4 : 2;
    const i64 mv = (c.m + 16 / es - 1) / (16 / es);
    // ~8 workgroups per CU in total, under the caller's cap
    const i64 gy = std::min<i64>(c.n, 4096);
    i64 gx = std::max<i64>(1, std::min<i64>((mv + NT - 1) / NT, std::max<i64>(1, 2048 / gy)));
    if (max_wgs > 0) gx = std::max<i64>(1, std::min<i64>(gx, max_wgs / gy));
    const dim3 grid((unsigned)gx, (unsigned)gy);
    ELX_DTYPE_SWITCH(dtype, T, hipLaunchKernelGGL((contract_sum_kernel<T>), grid, dim3(NT), 0, s, c, alpha));
    return hipGetLastError();
}

hipError_t convert2d(int sdt, int ddt, const Copy2D& d, hipStream_t s) {
    if (d.m <= 0 || d.n <= 0) return hipSuccess;
    if (sdt == ddt) return copy2d_batch(sdt, &d, 1, false, 0.0, s);
    const i64 tiles = ((d.m + TILE - 1) / TILE) * ((d.n + TILE - 1) / TILE);
    const dim3 grid((unsigned)(tiles > 8192 ? 8192 : tiles));
    ELX_DTYPE_SWITCH(sdt, TS, ELX_DTYPE_SWITCH(ddt, TD, hipLaunchKernelGGL((convert2d_kernel<TS, TD>), grid, dim3(NT), 0, s, d)));
    return hipGetLastError();
}

hipError_t fill2d(int dtype, i64 m, i64 n, double v, void* A, i64 lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T, {
        const EwShape g = ew_shape<typename Elem<T>::storage>(m, n, {{A, lda}});
        hipLaunchKernelGGL((fill_kernel<T>), g.grid, dim3(NT), 0, s, g.m, g.n, v,
                           static_cast<typename Elem<T>::storage*>(A), lda, g.vec);
    });
    return hipGetLastError();
}

hipError_t norm_partials(int dtype, int mode, i64 m, i64 n, const void* A, i64 lda, double scale, double* out,
                         int* nparts, hipStream_t s) {
    *nparts = 0;
    if (m <= 0 || n <= 0) return hipSuccess;
    const dim3 grid((unsigned)std::min<i64>((m + NT - 1) / NT, 32), (unsigned)std::min<i64>(n, kNormPartsMax / 32));
    *nparts = (int)(grid.x * grid.y);
    ELX_DTYPE_SWITCH(dtype, T, {
        using S = typename Elem<T>::storage;
        if (mode == 0)
            hipLaunchKernelGGL((norm_partial_kernel<T, 0>), grid, dim3(NT), 0, s, m, n, static_cast<const S*>(A), lda,
                               scale, out);
        else
            hipLaunchKernelGGL((norm_partial_kernel<T, 1>), grid, dim3(NT), 0, s, m, n, static_cast<const S*>(A), lda,
                               scale, out);
    });
    return hipGetLastError();
}

hipError_t scale2d(int dtype, i64 m, i64 n, double alpha, void* A, i64 lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T, {
        const EwShape g = ew_shape<typename Elem<T>::storage>(m, n, {{A, lda}});
        hipLaunchKernelGGL((scale_kernel<T>), g.grid, dim3(NT), 0, s, g.m, g.n, alpha,
                           static_cast<typename Elem<T>::storage*>(A), lda, g.vec);
    });
    return hipGetLastError();
}

hipError_t hadamard2d(int dtype, i64 m, i64 n, const void* A, i64 lda, const void* B, i64 ldb, void* C,
                      i64 ldc, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T, {
        using S = typename Elem<T>::storage;
        const EwShape g = ew_shape<S>(m, n, {{A, lda}, {B, ldb}, {C, ldc}});
        hipLaunchKernelGGL((hadamard_kernel<T>), g.grid, dim3(NT), 0, s, g.m, g.n,
                           static_cast<const S*>(A), lda, static_cast<const S*>(B), ldb,
                           static_cast<S*>(C), ldc, g.vec);
    });
    return hipGetLastError();
}

template <typename T, int FN>
static void launch_map(hipStream_t s, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb) {
    using S = typename Elem<T>::storage;
    const EwShape g = ew_shape<S>(m, n, {{A, lda}, {B, ldb}});
    hipLaunchKernelGGL((map_kernel<T, FN>), g.grid, dim3(NT), 0, s, g.m, g.n, static_cast<const S*>(A), lda,
                       static_cast<S*>(B), ldb, g.vec);
}

hipError_t entrywise_map(int dtype, int fn, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb,
                         hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
#define ELX_MAP_CASE(F) case F: launch_map<T, F>(s, m, n, A, lda, B, ldb); break;
    ELX_DTYPE_SWITCH(dtype, T, switch (fn) {
        ELX_MAP_CASE(ELX_MAP_IDENTITY) ELX_MAP_CASE(ELX_MAP_NEGATE) ELX_MAP_CASE(ELX_MAP_ABS)
        ELX_MAP_CASE(ELX_MAP_SQUARE) ELX_MAP_CASE(ELX_MAP_SQRT) ELX_MAP_CASE(ELX_MAP_EXP)
        ELX_MAP_CASE(ELX_MAP_LOG) ELX_MAP_CASE(ELX_MAP_RELU) ELX_MAP_CASE(ELX_MAP_SIGMOID)
        ELX_MAP_CASE(ELX_MAP_RECIP) ELX_MAP_CASE(ELX_MAP_TANH)
        default: return hipErrorInvalidValue;
    });
#undef ELX_MAP_CASE
    return hipGetLastError();
}

template <typename T, int FN>
static void launch_combine(hipStream_t s, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb) {
    using S = typename Elem<T>::storage;
    const EwShape g = ew_shape<S>(m, n, {{A, lda}, {B, ldb}});
    hipLaunchKernelGGL((combine_kernel<T, FN>), g.grid, dim3(NT), 0, s, g.m, g.n, static_cast<const S*>(A), lda,
                       static_cast<S*>(B), ldb, g.vec);
}

hipError_t combine(int dtype, int fn, i64 m, i64 n, const void* A, i64 lda, void* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
#define ELX_COMBINE_CASE(F) case F: launch_combine<T, F>(s, m, n, A, lda, B, ldb); break;
    ELX_DTYPE_SWITCH(dtype, T, switch (fn) {
        ELX_COMBINE_CASE(ELX_COMBINE_ADD) ELX_COMBINE_CASE(ELX_COMBINE_SUB) ELX_COMBINE_CASE(ELX_COMBINE_MUL)
        ELX_COMBINE_CASE(ELX_COMBINE_DIV) ELX_COMBINE_CASE(ELX_COMBINE_MAX) ELX_COMBINE_CASE(ELX_COMBINE_MIN)
        ELX_COMBINE_CASE(ELX_COMBINE_RELU_GRAD)
        default: return hipErrorInvalidValue;
    });
#undef ELX_COMBINE_CASE
    return hipGetLastError();
}

hipError_t fill_hash(int dtype, i64 m, i64 n, void* A, i64 lda, i64 i0, i64 istride, i64 j0, i64 jstride,
                     uint64_t seed, double center, double radius, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T,
        hipLaunchKernelGGL((hash_kernel<T>), grid2d(m, n), dim3(NT), 0, s, m, n,
                           static_cast<typename Elem<T>::storage*>(A), lda, i0, istride, j0, jstride,
                           seed, center, radius));
    return hipGetLastError();
}

hipError_t trapezoid2d(int dtype, bool lower, i64 m, i64 n, double alpha, const void* X, i64 ldx, double beta,
                       void* Y, i64 ldy, i64 i0, i64 istride, i64 j0, i64 jstride, i64 offset, hipStream_t s) {
    if (m <= 0 || n <= 0) return hipSuccess;
    ELX_DTYPE_SWITCH(dtype, T,
        hipLaunchKernelGGL((trapezoid_kernel<T>), grid2d(m, n), dim3(NT), 0, s, lower, m, n, alpha,
                           static_cast<const typename Elem<T>::storage*>(X), ldx, beta,
                           static_cast<typename Elem<T>::storage*>(Y), ldy, i0, istride, j0, jstride, offset));
    return hipGetLastError();
}

}  // namespace kern
}  // namespace elx
