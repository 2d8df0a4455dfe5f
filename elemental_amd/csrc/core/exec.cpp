#include <cstdlib>
#include "exec.hpp"
#include "../kernels/elem.hpp"
#include <cmath>
#include <vector>

namespace elx {
namespace exec {

namespace {

// Host element access in the compute type of each dtype (f16/bf16 -> float).
template <typename S> struct H;
template <> struct H<double> {
    using C = double;
    static C ld(const double* p) { return *p; }
    static void st(double* p, C v) { *p = v; }
};
template <> struct H<float> {
    using C = float;
    static C ld(const float* p) { return *p; }
    static void st(float* p, C v) { *p = v; }
};
struct Half16 { uint16_t b; };
struct Brain16 { uint16_t b; };
template <> struct H<Half16> {
    using C = float;
    static C ld(const Half16* p) { return HalfToFloat(p->b); }
    static void st(Half16* p, C v) { p->b = FloatToHalf(v); }
};
template <> struct H<Brain16> {
    using C = float;
    static C ld(const Brain16* p) { return BF16ToFloat(p->b); }
    static void st(Brain16* p, C v) { p->b = FloatToBF16(v); }
};

#define HOST_DTYPE_SWITCH(t, S, ...)                                   \
    switch (t) {                                                       \
    case DType::F64: { using S = double; __VA_ARGS__; break; }         \
    case DType::F32: { using S = float; __VA_ARGS__; break; }          \
    case DType::F16: { using S = Half16; __VA_ARGS__; break; }         \
    case DType::BF16: { using S = Brain16; __VA_ARGS__; break; }       \
    default: throw LogicError(Cat("dtype ", DTypeName(t), " is not a matrix type")); \
    }

template <typename S>
void cpu_copy(const Copy2D& d, bool axpy, double alpha) {
    const S* src = static_cast<const S*>(d.src);
    S* dst = static_cast<S*>(d.dst);
    using C = typename H<S>::C;
    const C a = (C)alpha;
    for (Int j = 0; j < d.n; ++j)
        for (Int i = 0; i < d.m; ++i) {
            const S* x = src + i * d.scs + j * d.srs;
            S* y = dst + i * d.dcs + j * d.drs;
            if (axpy) H<S>::st(y, H<S>::ld(y) + a * H<S>::ld(x));
            else *y = *x;
        }
}

template <typename S>
void cpu_gemm(bool ta, bool tb, Int m, Int n, Int k, double alpha, const S* A, Int lda, const S* B,
              Int ldb, double beta, S* C, Int ldc) {
    using Cm = typename H<S>::C;
    std::vector<Cm> acc(static_cast<size_t>(m));
    for (Int j = 0; j < n; ++j) {
        std::fill(acc.begin(), acc.end(), Cm(0));
        for (Int l = 0; l < k; ++l) {
            const Cm b = H<S>::ld(tb ? B + j + l * ldb : B + l + j * ldb);
            if (b == Cm(0)) continue;
            if (!ta) {
                const S* acol = A + l * lda;
                for (Int i = 0; i < m; ++i) acc[i] += H<S>::ld(acol + i) * b;
            } else {
                for (Int i = 0; i < m; ++i) acc[i] += H<S>::ld(A + l + i * lda) * b;
            }
        }
        for (Int i = 0; i < m; ++i) {
            S* c = C + i + j * ldc;
            const Cm v = (Cm)alpha * acc[i];
            H<S>::st(c, beta == 0.0 ? v : v + (Cm)beta * H<S>::ld(c));
        }
    }
}

template <typename Cm>
Cm cpu_map(int fn, Cm x) {
    switch (fn) {
    case ELX_MAP_IDENTITY: return x;
    case ELX_MAP_NEGATE: return -x;
    case ELX_MAP_ABS: return std::fabs(x);
    case ELX_MAP_SQUARE: return x * x;
    case ELX_MAP_SQRT: return std::sqrt(x);
    case ELX_MAP_EXP: return std::exp(x);
    case ELX_MAP_LOG: return std::log(x);
    case ELX_MAP_RELU: return x > Cm(0) ? x : Cm(0);
    case ELX_MAP_SIGMOID: return Cm(1) / (Cm(1) + std::exp(-x));
    case ELX_MAP_RECIP: return Cm(1) / x;
    case ELX_MAP_TANH: return std::tanh(x);
    default: throw LogicError(Cat("unknown entrywise functor ", fn));
    }
}

void check(hipError_t e, const char* what) {
    if (e != hipSuccess)
        throw HIPError(Cat(what, ": ", hipGetErrorName(e), " (", hipGetErrorString(e), ")"));
}

}  // namespace

// Pack / unpack launches on the comm stream run beside full-machine MFMA
// updates, so they are capped at ELX_COMM_COPY_WGS workgroups (default 256, one
// per CU): uncapped launches of thousands of workgroups at the comm stream's
// priority slowed the MFMA updates by 5-10 %, caps of 256-512 by 0-2 %
// (profiles/r02_comm_copy_cap.log; 0 = uncapped)
int CommCopyWGs() {
    static const int v = [] { const char* e = getenv("ELX_COMM_COPY_WGS"); return e ? atoi(e) : 256; }();
    return v;
}

void Copy2DBatch(Device dev, DType t, const Copy2D* d, int nd, bool axpy, double alpha, hipStream_t s) {
    if (nd <= 0) return;
    if (dev == Device::GPU) {
        const int cap = s != nullptr && s == Runtime::Get().CommStream() ? CommCopyWGs() : 0;
        check(kern::copy2d_batch(static_cast<int>(t), d, nd, axpy, alpha, s, cap), "copy2d_batch");
        return;
    }
    for (int q = 0; q < nd; ++q) HOST_DTYPE_SWITCH(t, S, cpu_copy<S>(d[q], axpy, alpha));
}

void ContractSum(Device dev, DType t, Int m, Int n, void* dst, Int dcs, Int drs, const ContractSource* src,
                 int nsrc, double alpha, hipStream_t s) {
    if (m <= 0 || n <= 0 || nsrc <= 0) return;
    if (dev == Device::GPU) {
        const int cap = s != nullptr && s == Runtime::Get().CommStream() ? CommCopyWGs() : 0;
        for (int q0 = 0; q0 < nsrc; q0 += kern::kMaxContractSources) {
            kern::ContractSum c{};
            c.m = m; c.n = n; c.dst = dst; c.dcs = dcs; c.drs = drs;
            c.nsrc = std::min(nsrc - q0, kern::kMaxContractSources);
            for (int q = 0; q < c.nsrc; ++q) {
                c.src[q] = src[q0 + q].p;
                c.scs[q] = src[q0 + q].cs;
                c.srs[q] = src[q0 + q].rs;
            }
            check(kern::contract_sum(static_cast<int>(t), c, alpha, s, cap), "contract_sum");
        }
        return;
    }
    // host: the same per-source axpys, in order
    for (int q = 0; q < nsrc; ++q) {
        const Copy2D d{m, n, src[q].p, src[q].cs, src[q].rs, dst, dcs, drs};
        HOST_DTYPE_SWITCH(t, S, cpu_copy<S>(d, true, alpha));
    }
}

namespace {
template <typename TS, typename TD>
void cpu_convert(const Copy2D& d) {
    using SS = typename kern::Elem<TS>::storage;
    using SD = typename kern::Elem<TD>::storage;
    const SS* src = static_cast<const SS*>(d.src);
    SD* dst = static_cast<SD*>(d.dst);
    for (Int j = 0; j < d.n; ++j)
        for (Int i = 0; i < d.m; ++i)
            dst[i * d.dcs + j * d.drs] = kern::convert_elem<TS, TD>(src[i * d.scs + j * d.srs]);
}
#define KERN_DTYPE_SWITCH(t, T, ...)                                     \
    switch (t) {                                                         \
    case DType::F64: { using T = double; __VA_ARGS__; break; }           \
    case DType::F32: { using T = float; __VA_ARGS__; break; }            \
    case DType::F16: { using T = kern::f16_t; __VA_ARGS__; break; }      \
    case DType::BF16: { using T = kern::bf16_t; __VA_ARGS__; break; }    \
    default: throw LogicError(Cat("dtype ", DTypeName(t), " is not a matrix type")); \
    }
}  // namespace

void Convert2D(Device dev, DType src_t, DType dst_t, const Copy2D& d, hipStream_t s) {
    if (d.m <= 0 || d.n <= 0) return;
    if (src_t == dst_t) { Copy2DBatch(dev, src_t, &d, 1, false, 0.0, s); return; }
    if (dev == Device::GPU) {
        check(kern::convert2d(static_cast<int>(src_t), static_cast<int>(dst_t), d, s), "convert2d");
        return;
    }
    KERN_DTYPE_SWITCH(src_t, TS, KERN_DTYPE_SWITCH(dst_t, TD, cpu_convert<TS, TD>(d)));
}

void Gemm(Device dev, DType t, bool ta, bool tb, Int m, Int n, Int k, double alpha, const void* A, Int lda,
          const void* B, Int ldb, double beta, void* C, Int ldc, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) {
        hipError_t e = hipSuccess;
        switch (t) {
        case DType::F64:
            e = kern::gemm_mfma<double>(ta, tb, m, n, k, alpha, static_cast<const double*>(A), lda,
                                        static_cast<const double*>(B), ldb, beta, static_cast<double*>(C), ldc, s);
            break;
        case DType::F32:
            e = kern::gemm_mfma<float>(ta, tb, m, n, k, (float)alpha, static_cast<const float*>(A), lda,
                                       static_cast<const float*>(B), ldb, (float)beta, static_cast<float*>(C),
                                       ldc, s);
            break;
        case DType::F16:
        case DType::BF16:
            e = kern::gemm_mfma_h(t == DType::BF16, ta, tb, m, n, k, (float)alpha,
                                  static_cast<const uint16_t*>(A), lda, static_cast<const uint16_t*>(B), ldb,
                                  (float)beta, static_cast<uint16_t*>(C), ldc, s);
            break;
        default:
            throw LogicError(Cat("dtype ", DTypeName(t), " is not a matrix type"));
        }
        check(e, "gemm_mfma");
        return;
    }
    HOST_DTYPE_SWITCH(t, S,
        cpu_gemm<S>(ta, tb, m, n, k, alpha, static_cast<const S*>(A), lda, static_cast<const S*>(B), ldb, beta,
                    static_cast<S*>(C), ldc));
}

void Fill(Device dev, DType t, Int m, Int n, double v, void* A, Int lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) { check(kern::fill2d((int)t, m, n, v, A, lda, s), "fill2d"); return; }
    HOST_DTYPE_SWITCH(t, S, {
        S* a = static_cast<S*>(A);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i) H<S>::st(a + i + j * lda, (typename H<S>::C)v);
    });
}

void Scale(Device dev, DType t, Int m, Int n, double alpha, void* A, Int lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) { check(kern::scale2d((int)t, m, n, alpha, A, lda, s), "scale2d"); return; }
    HOST_DTYPE_SWITCH(t, S, {
        S* a = static_cast<S*>(A);
        using Cm = typename H<S>::C;
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i) H<S>::st(a + i + j * lda, (Cm)alpha * H<S>::ld(a + i + j * lda));
    });
}

namespace {
double NormMax(double a, double b) { return a != a ? a : b != b ? b : std::max(a, b); }
// mode 0: max |a|; mode 1: sum (a / scale)^2 — device partials reduced on the host
double NormReduce(Device dev, DType t, int mode, Int m, Int n, const void* A, Int lda, double scale, hipStream_t s) {
    double r = 0.0;
    if (m <= 0 || n <= 0) return r;
    if (dev == Device::GPU) {
        Buffer parts(Device::GPU, sizeof(double) * kern::kNormPartsMax, s);
        int np = 0;
        check(kern::norm_partials((int)t, mode, m, n, A, lda, scale, static_cast<double*>(parts.data()), &np, s),
              "norm_partials");
        std::vector<double> h(np);
        ELX_CHECK_HIP(hipMemcpyAsync(h.data(), parts.data(), sizeof(double) * np, hipMemcpyDeviceToHost, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
        for (double v : h) r = mode == 0 ? NormMax(r, v) : r + v;
        return r;
    }
    HOST_DTYPE_SWITCH(t, S, {
        const S* a = static_cast<const S*>(A);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i) {
                const double x = (double)H<S>::ld(a + i + j * lda);
                if (mode == 0) r = NormMax(r, std::fabs(x));
                else { const double y = x / scale; r += y * y; }
            }
    });
    return r;
}
}  // namespace

double AbsMax(Device dev, DType t, Int m, Int n, const void* A, Int lda, hipStream_t s) {
    return NormReduce(dev, t, 0, m, n, A, lda, 1.0, s);
}
double ScaledSumSq(Device dev, DType t, Int m, Int n, const void* A, Int lda, double scale, hipStream_t s) {
    return NormReduce(dev, t, 1, m, n, A, lda, scale, s);
}

void Hadamard(Device dev, DType t, Int m, Int n, const void* A, Int lda, const void* B, Int ldb, void* C,
              Int ldc, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) { check(kern::hadamard2d((int)t, m, n, A, lda, B, ldb, C, ldc, s), "hadamard2d"); return; }
    HOST_DTYPE_SWITCH(t, S, {
        const S* a = static_cast<const S*>(A);
        const S* b = static_cast<const S*>(B);
        S* c = static_cast<S*>(C);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i)
                H<S>::st(c + i + j * ldc, H<S>::ld(a + i + j * lda) * H<S>::ld(b + i + j * ldb));
    });
}

void Map(Device dev, DType t, int fn, Int m, Int n, const void* A, Int lda, void* B, Int ldb, hipStream_t s) {
    if (fn < ELX_MAP_IDENTITY || fn > ELX_MAP_TANH) throw LogicError(Cat("unknown entrywise functor ", fn));
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) { check(kern::entrywise_map((int)t, fn, m, n, A, lda, B, ldb, s), "entrywise_map"); return; }
    HOST_DTYPE_SWITCH(t, S, {
        const S* a = static_cast<const S*>(A);
        S* b = static_cast<S*>(B);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i) H<S>::st(b + i + j * ldb, cpu_map(fn, H<S>::ld(a + i + j * lda)));
    });
}

template <typename Cm>
Cm cpu_combine(int fn, Cm a, Cm b) {
    switch (fn) {
    case ELX_COMBINE_ADD: return a + b;
    case ELX_COMBINE_SUB: return b - a;
    case ELX_COMBINE_MUL: return a * b;
    case ELX_COMBINE_DIV: return b / a;
    case ELX_COMBINE_MAX: return a > b ? a : b;
    case ELX_COMBINE_MIN: return a < b ? a : b;
    case ELX_COMBINE_RELU_GRAD: return a > Cm(0) ? b : Cm(0);
    default: throw LogicError(Cat("unknown combine functor ", fn));
    }
}

void Combine(Device dev, DType t, int fn, Int m, Int n, const void* A, Int lda, void* B, Int ldb, hipStream_t s) {
    if (fn < ELX_COMBINE_ADD || fn > ELX_COMBINE_RELU_GRAD) throw LogicError(Cat("unknown combine functor ", fn));
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) { check(kern::combine((int)t, fn, m, n, A, lda, B, ldb, s), "combine"); return; }
    HOST_DTYPE_SWITCH(t, S, {
        const S* a = static_cast<const S*>(A);
        S* b = static_cast<S*>(B);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i)
                H<S>::st(b + i + j * ldb, cpu_combine(fn, H<S>::ld(a + i + j * lda), H<S>::ld(b + i + j * ldb)));
    });
}

void Trapezoid(Device dev, DType t, bool lower, Int m, Int n, double alpha, const void* X, Int ldx, double beta,
               void* Y, Int ldy, Int i0, Int is, Int j0, Int js, Int offset, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) {
        check(kern::trapezoid2d((int)t, lower, m, n, alpha, X, ldx, beta, Y, ldy, i0, is, j0, js, offset, s),
              "trapezoid2d");
        return;
    }
    HOST_DTYPE_SWITCH(t, S, {
        using Cm = typename H<S>::C;
        const S* x = static_cast<const S*>(X);
        S* y = static_cast<S*>(Y);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i) {
                const Int gi = i0 + i * is, gj = j0 + j * js - offset;
                if (lower ? gi < gj : gi > gj) continue;
                Cm v = (x && beta == 0.0) ? Cm(0) : (Cm)beta * H<S>::ld(y + i + j * ldy);
                if (x) v = v + (Cm)alpha * H<S>::ld(x + i + j * ldx);
                H<S>::st(y + i + j * ldy, v);
            }
    });
}

template <typename S>
void cpu_trsm(bool lower, bool trans, bool unit, Int m, Int n, const S* A, Int lda, S* B, Int ldb) {
    const bool forward = lower != trans;
    auto opA = [&](Int r, Int c) { return trans ? A[c + r * lda] : A[r + c * lda]; };
    for (Int j = 0; j < n; ++j) {
        S* x = B + j * ldb;
        for (Int s = 0; s < m; ++s) {
            const Int i = forward ? s : m - 1 - s;
            S xi = x[i];
            if (!unit) xi = xi / opA(i, i);
            x[i] = xi;
            if (forward)
                for (Int r = i + 1; r < m; ++r) x[r] = x[r] - opA(r, i) * xi;
            else
                for (Int r = 0; r < i; ++r) x[r] = x[r] - opA(r, i) * xi;
        }
    }
}

void Trsm(Device dev, DType t, bool lower, bool trans, bool unit, Int m, Int n, const void* A, Int lda, void* B,
          Int ldb, hipStream_t s) {
    if (t != DType::F64 && t != DType::F32) throw LogicError("Trsm: only float and double are supported");
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) {
        const size_t es = DTypeSize(t);
        if (m <= 256 && n >= 4 * m) {
            // many right-hand sides: W = op(A)^-1 (m lanes of substitution), then
            // B := W B as one MFMA GEMM through a workspace (the inverted-diagonal-
            // block scheme of vendor trsm), instead of n/64 waves each running an
            // m^2/2-long dependent chain
            Buffer W(dev, (size_t)m * m * es, s);
            check(kern::trsm_local((int)t, true, lower, trans, unit, m, m, A, lda, W.data(), m, s), "trsm_local");
            ApplyInverse(dev, t, m, n, W.data(), m, B, ldb, s);
            return;
        }
        check(kern::trsm_local((int)t, false, lower, trans, unit, m, n, A, lda, B, ldb, s), "trsm_local");
        return;
    }
    if (t == DType::F64)
        cpu_trsm(lower, trans, unit, m, n, static_cast<const double*>(A), lda, static_cast<double*>(B), ldb);
    else
        cpu_trsm(lower, trans, unit, m, n, static_cast<const float*>(A), lda, static_cast<float*>(B), ldb);
}

void TriInverseBatched(DType t, bool lower, bool trans, bool unit, Int nb, Int m, const void* A, Int lda, void* W,
                       hipStream_t s) {
    check(kern::tri_inverse_batched((int)t, lower, trans, unit, nb, m, A, lda, W, s), "tri_inverse_batched");
}

void ApplyInverse(Device dev, DType t, Int m, Int n, const void* W, Int ldw, void* B, Int ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    Buffer T(dev, (size_t)m * n * DTypeSize(t), s);
    Gemm(dev, t, false, false, m, n, m, 1.0, W, ldw, B, ldb, 0.0, T.data(), m, s);
    const Copy2D d{m, n, T.data(), 1, m, B, 1, ldb};
    Copy2DBatch(dev, t, &d, 1, false, 0.0, s);
}

void FillHash(Device dev, DType t, Int m, Int n, void* A, Int lda, Int i0, Int is, Int j0, Int js,
              uint64_t seed, double center, double radius, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (dev == Device::GPU) {
        check(kern::fill_hash((int)t, m, n, A, lda, i0, is, j0, js, seed, center, radius, s), "fill_hash");
        return;
    }
    HOST_DTYPE_SWITCH(t, S, {
        S* a = static_cast<S*>(A);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i) {
                const double u = kern::hash_unit(seed, i0 + i * is, j0 + j * js);
                H<S>::st(a + i + j * lda, (typename H<S>::C)(center + radius * (2.0 * u - 1.0)));
            }
    });
}

double LoadScalar(DType t, const void* p) {
    double v = 0;
    HOST_DTYPE_SWITCH(t, S, v = (double)H<S>::ld(static_cast<const S*>(p)));
    return v;
}
void StoreScalar(DType t, void* p, double v) {
    HOST_DTYPE_SWITCH(t, S, H<S>::st(static_cast<S*>(p), (typename H<S>::C)v));
}

}  // namespace exec
}  // namespace elx
