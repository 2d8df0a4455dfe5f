// extern "C" boundary (include/elemental_amd.h).  Every entry point runs
// inside Guard(), which turns the C++ exceptions into ELX_ERR_* codes.
#include "common.hpp"
#include "runtime/runtime.hpp"
#include "comm/comm.hpp"
#include "core/distmatrix.hpp"
#include "core/redist.hpp"
#include "core/gemm.hpp"
#include "core/random.hpp"
#include "core/io.hpp"
#include "core/exec.hpp"
#include <string>

struct elx_comm_s { std::shared_ptr<elx::Comm> c; };
struct elx_grid_s { std::shared_ptr<elx::Grid> g; };
struct elx_dm_s { std::shared_ptr<elx::DistMatrix> m; };

namespace elx {
namespace {
thread_local std::string g_last_error;

Dist ToDist(int d) {
    if (d < ELX_MC || d > ELX_CIRC) throw LogicError(Cat("invalid dist ", d));
    return static_cast<Dist>(d);
}
Device ToDevice(int d) {
    if (d != ELX_DEVICE_CPU && d != ELX_DEVICE_GPU) throw LogicError(Cat("invalid device ", d));
    return static_cast<Device>(d);
}
DistMatrix& M(elx_dm_t h) {
    if (!h || !h->m) throw LogicError("null DistMatrix handle");
    return *h->m;
}
void CheckOp(int o) {
    if (o != ELX_NORMAL && o != ELX_TRANSPOSE && o != ELX_ADJOINT) throw LogicError(Cat("invalid orientation ", o));
}
hipStream_t S(void* s) { return Runtime::Get().Resolve(s); }
// the handle elx_comm_world lends out (never freed)
elx_comm_s& WorldHandle() {
    static elx_comm_s* h = new elx_comm_s{};
    return *h;
}
}  // namespace

void SetLastError(const std::string& msg) { g_last_error = msg; }
}  // namespace elx

using namespace elx;

extern "C" {

const char* elx_last_error(void) { return g_last_error.c_str(); }
int elx_version(void) { return 10000; }

int elx_device_count(int* count) {
    return Guard([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        *count = n;
    });
}
int elx_set_device(int device) { return Guard([&] { Runtime::Get().SetDevice(device); Runtime::Get().EnsureGPU(); }); }
int elx_get_device(int* device) { return Guard([&] { Runtime::Get().EnsureGPU(); *device = Runtime::Get().DeviceId(); }); }
int elx_device_synchronize(void) {
    return Guard([&] { Runtime::Get().EnsureGPU(); ELX_CHECK_HIP(hipDeviceSynchronize()); });
}
int elx_default_stream(void** stream) { return Guard([&] { *stream = Runtime::Get().ComputeStream(); }); }
int elx_comm_stream(void** stream) { return Guard([&] { *stream = Runtime::Get().CommStream(); }); }
int elx_reserved_cus(int* cus) { return Guard([&] { *cus = Runtime::Get().ReservedCUs(); }); }
int elx_stream_create(void** stream) {
    return Guard([&] {
        Runtime::Get().EnsureGPU();
        hipStream_t s;
        ELX_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        *stream = s;
    });
}
int elx_stream_destroy(void* stream) { return Guard([&] { ELX_CHECK_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream))); }); }
int elx_stream_synchronize(void* stream) { return Guard([&] { ELX_CHECK_HIP(hipStreamSynchronize(S(stream))); }); }
int elx_default_event(void** event) {
    return Guard([&] {
        Runtime::Get().EnsureGPU();
        static hipEvent_t ev = [] {
            hipEvent_t e;
            ELX_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            return e;
        }();
        *event = ev;
    });
}
int elx_event_create(void** event) {
    return Guard([&] {
        Runtime::Get().EnsureGPU();
        hipEvent_t e;
        ELX_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        *event = e;
    });
}
int elx_event_destroy(void* event) { return Guard([&] { ELX_CHECK_HIP(hipEventDestroy(static_cast<hipEvent_t>(event))); }); }
int elx_event_record(void* event, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(event, "null event");
        ELX_CHECK_HIP(hipEventRecord(static_cast<hipEvent_t>(event), S(stream)));
    });
}
int elx_stream_wait_event(void* stream, void* event) {
    return Guard([&] {
        ELX_REQUIRE(event, "null event");
        ELX_CHECK_HIP(hipStreamWaitEvent(S(stream), static_cast<hipEvent_t>(event), 0));
    });
}
int elx_event_synchronize(void* event) {
    return Guard([&] {
        ELX_REQUIRE(event, "null event");
        ELX_CHECK_HIP(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    });
}

int elx_pool_alloc(void** ptr, size_t bytes, void* stream) {
    return Guard([&] { *ptr = Runtime::Get().Alloc(bytes, S(stream)); });
}
int elx_pool_free(void* ptr, void* stream) { return Guard([&] { Runtime::Get().Free(ptr, S(stream)); }); }
int elx_pool_trim(size_t keep) { return Guard([&] { Runtime::Get().Trim(keep); }); }
int elx_pool_stats(size_t* reserved, size_t* in_use) { return Guard([&] { Runtime::Get().Stats(*reserved, *in_use); }); }
int elx_pool_set_max_cached(size_t bytes) { return Guard([&] { Runtime::Get().SetMaxCached(bytes); }); }
int elx_pool_max_cached(size_t* bytes) { return Guard([&] { *bytes = Runtime::Get().MaxCached(); }); }
size_t elx_pool_bin_bytes(size_t bytes) { return Runtime::BinBytes(bytes); }
int elx_pool_bin_cacheable(size_t bytes) {
    bool c = true;
    (void)Runtime::BinBytes(bytes, &c);
    return c ? 1 : 0;
}
int elx_pool_backing_reserved(size_t* bytes) { return Guard([&] { *bytes = Runtime::Get().BackingReserved(); }); }
int elx_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    return Guard([&] {
        hipStream_t s = S(stream);
        ELX_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
    });
}
int elx_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    return Guard([&] {
        hipStream_t s = S(stream);
        ELX_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
    });
}
int elx_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
    return Guard([&] { ELX_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, S(stream))); });
}

// ---- local GEMM ----------------------------------------------------------
#define ELX_GEMM_ENTRY(NAME, DT, ST, SC)                                                              \
    int NAME(int opA, int opB, int64_t m, int64_t n, int64_t k, SC alpha, const ST* A, int64_t lda,    \
             const ST* B, int64_t ldb, SC beta, ST* C, int64_t ldc, void* stream) {                  \
        return Guard([&] {                                                                             \
            CheckOp(opA);                                                                              \
            CheckOp(opB);                                                                              \
            ELX_REQUIRE(m >= 0 && n >= 0 && k >= 0, "negative GEMM dimension");                       \
            const bool ta = opA != ELX_NORMAL, tb = opB != ELX_NORMAL;                                 \
            ELX_REQUIRE(ldc >= (m > 1 ? m : 1), "ldc too small");                                     \
            ELX_REQUIRE(lda >= ((ta ? k : m) > 1 ? (ta ? k : m) : 1), "lda too small");               \
            ELX_REQUIRE(ldb >= ((tb ? n : k) > 1 ? (tb ? n : k) : 1), "ldb too small");               \
            if (m == 0 || n == 0) return;                                                              \
            exec::Gemm(Device::GPU, DT, ta, tb, m, n, k, (double)alpha, A, lda, B, ldb, (double)beta, C, \
                       ldc, S(stream));                                                                \
        });                                                                                            \
    }
ELX_GEMM_ENTRY(elx_gemm_f64, DType::F64, double, double)
ELX_GEMM_ENTRY(elx_gemm_f32, DType::F32, float, float)
ELX_GEMM_ENTRY(elx_gemm_f16, DType::F16, uint16_t, float)
ELX_GEMM_ENTRY(elx_gemm_bf16, DType::BF16, uint16_t, float)
#undef ELX_GEMM_ENTRY

// ---- El::Matrix<T,D> (either device) ------------------------------------------
namespace {
hipStream_t DevStream(Device d, void* stream) { return d == Device::GPU ? S(stream) : nullptr; }
void CheckLd(int64_t ld, int64_t rows, const char* what) {
    ELX_REQUIRE(ld >= (rows > 1 ? rows : 1), what, " leading dimension ", ld, " < ", rows);
}
}  // namespace
int elx_matrix_gemm(int dtype, int device, int opA, int opB, int64_t m, int64_t n, int64_t k, double alpha,
                    const void* A, int64_t lda, const void* B, int64_t ldb, double beta, void* C, int64_t ldc,
                    void* stream) {
    return Guard([&] {
        CheckOp(opA);
        CheckOp(opB);
        ELX_REQUIRE(m >= 0 && n >= 0 && k >= 0, "negative GEMM dimension");
        const bool ta = opA != ELX_NORMAL, tb = opB != ELX_NORMAL;
        CheckLd(ldc, m, "C");
        CheckLd(lda, ta ? k : m, "A");
        CheckLd(ldb, tb ? n : k, "B");
        if (m == 0 || n == 0) return;
        const Device d = ToDevice(device);
        if (k == 0) {  // Gemm.cpp:240-248: C := beta C (beta == 0 clears NaNs)
            if (beta == 0.0) exec::Fill(d, ToDType(dtype), m, n, 0.0, C, ldc, DevStream(d, stream));
            else if (beta != 1.0) exec::Scale(d, ToDType(dtype), m, n, beta, C, ldc, DevStream(d, stream));
            return;
        }
        exec::Gemm(d, ToDType(dtype), ta, tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, DevStream(d, stream));
    });
}
int elx_matrix_fill(int dtype, int device, int64_t m, int64_t n, double value, void* A, int64_t lda, void* stream) {
    return Guard([&] {
        CheckLd(lda, m, "A");
        if (m == 0 || n == 0) return;
        const Device d = ToDevice(device);
        exec::Fill(d, ToDType(dtype), m, n, value, A, lda, DevStream(d, stream));
    });
}
int elx_matrix_scale(int dtype, int device, int64_t m, int64_t n, double alpha, void* A, int64_t lda, void* stream) {
    return Guard([&] {
        CheckLd(lda, m, "A");
        if (m == 0 || n == 0) return;
        const Device d = ToDevice(device);
        if (alpha == 0.0) exec::Fill(d, ToDType(dtype), m, n, 0.0, A, lda, DevStream(d, stream));
        else if (alpha != 1.0) exec::Scale(d, ToDType(dtype), m, n, alpha, A, lda, DevStream(d, stream));
    });
}
int elx_matrix_axpy(int dtype, int device, int64_t m, int64_t n, double alpha, const void* X, int64_t ldx, void* Y,
                    int64_t ldy, void* stream) {
    return Guard([&] {
        CheckLd(ldx, m, "X");
        CheckLd(ldy, m, "Y");
        if (m == 0 || n == 0) return;
        const Device d = ToDevice(device);
        kern::Copy2D c{m, n, X, 1, ldx, Y, 1, ldy};
        exec::Copy2DBatch(d, ToDType(dtype), &c, 1, true, alpha, DevStream(d, stream));
    });
}
int elx_matrix_copy(int dtype, int device, int64_t m, int64_t n, const void* A, int64_t lda, void* B, int64_t ldb,
                    void* stream) {
    return Guard([&] {
        CheckLd(lda, m, "A");
        CheckLd(ldb, m, "B");
        if (m == 0 || n == 0) return;
        const Device d = ToDevice(device);
        kern::Copy2D c{m, n, A, 1, lda, B, 1, ldb};
        exec::Copy2DBatch(d, ToDType(dtype), &c, 1, false, 0.0, DevStream(d, stream));
    });
}

// ---- BLAS-1 --------------------------------------------------------------
int elx_axpy2d(int dtype, int64_t m, int64_t n, double alpha, const void* X, int64_t xcs, int64_t xrs, void* Y,
               int64_t ycs, int64_t yrs, void* stream) {
    return Guard([&] {
        kern::Copy2D d{m, n, X, xcs, xrs, Y, ycs, yrs};
        exec::Copy2DBatch(Device::GPU, ToDType(dtype), &d, 1, true, alpha, S(stream));
    });
}
int elx_copy2d(int dtype, int64_t m, int64_t n, const void* A, int64_t acs, int64_t ars, void* B, int64_t bcs,
               int64_t brs, void* stream) {
    return Guard([&] {
        kern::Copy2D d{m, n, A, acs, ars, B, bcs, brs};
        exec::Copy2DBatch(Device::GPU, ToDType(dtype), &d, 1, false, 0.0, S(stream));
    });
}
int elx_copy2d_convert(int src_dtype, int dst_dtype, int64_t m, int64_t n, const void* A, int64_t acs, int64_t ars,
                       void* B, int64_t bcs, int64_t brs, void* stream) {
    return Guard([&] {
        kern::Copy2D d{m, n, A, acs, ars, B, bcs, brs};
        exec::Convert2D(Device::GPU, ToDType(src_dtype), ToDType(dst_dtype), d, S(stream));
    });
}
// ---- pack / unpack for redistributions (Copy/util.hpp) ---------------------------
// Each call is ONE batched strided-copy launch over all portions (the reference
// issues one InterleaveMatrix per portion).  Portion k of a colStride-way split
// holds the rows colShift(k) = Shift_(k, colAlign, colStride), colShift+colStride, ...
// (indexing/impl.hpp:33-36,244-245), stored column-major with ld = its height.
}  // extern "C"
namespace {
Device PackDev(int device) {
    ELX_REQUIRE(device == ELX_DEVICE_CPU || device == ELX_DEVICE_GPU, "pack: bad device ", device);
    return device == ELX_DEVICE_GPU ? Device::GPU : Device::CPU;
}
void RunCopies(int device, int dtype, const std::vector<kern::Copy2D>& d, bool axpy, double alpha, void* stream) {
    if (d.empty()) return;
    const Device dev = PackDev(device);
    exec::Copy2DBatch(dev, ToDType(dtype), d.data(), (int)d.size(), axpy, alpha, dev == Device::GPU ? S(stream) : nullptr);
}
// StridedPack / StridedUnpack (util.hpp:667-718): portion k + l*colStride holds
// the (colShift(k), rowShift(l)) sub-lattice; col/row-only forms are stride 1
std::vector<kern::Copy2D> StridedPlan(int dtype, Int h, Int w, Int colAlign, Int colStride, Int rowAlign,
                                      Int rowStride, const void* M, Int ldm, const void* P, Int portionSize,
                                      bool pack) {
    ELX_REQUIRE(h >= 0 && w >= 0 && colStride > 0 && rowStride > 0 && portionSize >= 0 && ldm >= std::max<Int>(1, h),
                "pack: bad sizes");
    const size_t es = DTypeSize(ToDType(dtype));
    std::vector<kern::Copy2D> d;
    for (Int l = 0; l < rowStride; ++l) {
        const Int rs = Shift(l, rowAlign, rowStride), lw = Length(w, rs, rowStride);
        for (Int k = 0; k < colStride; ++k) {
            const Int cs = Shift(k, colAlign, colStride), lh = Length(h, cs, colStride);
            ELX_REQUIRE(lh * lw <= portionSize, "pack: portion ", k + l * colStride, " needs ", lh * lw,
                        " elements, portionSize is ", portionSize);
            if (lh == 0 || lw == 0) continue;
            char* m = (char*)M + (cs + rs * ldm) * es;
            char* q = (char*)P + (k + l * colStride) * portionSize * es;
            if (pack) d.push_back({lh, lw, m, colStride, rowStride * ldm, q, 1, lh});
            else d.push_back({lh, lw, q, 1, lh, m, colStride, rowStride * ldm});
        }
    }
    return d;
}
// PartialColStridedPack / Unpack (util.hpp:460-552) and the row forms
// (:186-230, :308-355): portion k holds the rows of partial rank
// colRankPart + k*colStridePart, read from a matrix whose own rows start at shift0
// with stride colStridePart (so those rows sit colStrideUnion apart in it)
std::vector<kern::Copy2D> PartialPlan(int dtype, bool cols, Int h, Int w, Int align, Int stride, Int strideUnion,
                                      Int stridePart, Int rankPart, Int shift0, const void* M, Int ldm,
                                      const void* P, Int portionSize, bool pack) {
    // (cols: `height` is the global height and M holds the rows of the partial
    // lattice from shift0, so its own height is Length_(h, shift0, stridePart))
    ELX_REQUIRE(h >= 0 && w >= 0 && stride > 0 && strideUnion > 0 && stridePart > 0 && portionSize >= 0 &&
                    ldm >= std::max<Int>(1, cols ? Length(h, shift0, stridePart) : h),
                "partial pack: bad sizes");
    ELX_REQUIRE(strideUnion * stridePart == stride, "partial pack: strideUnion * stridePart != stride");
    const size_t es = DTypeSize(ToDType(dtype));
    std::vector<kern::Copy2D> d;
    for (Int k = 0; k < strideUnion; ++k) {
        const Int sh = Shift(rankPart + k * stridePart, align, stride);
        ELX_REQUIRE((sh - shift0) % stridePart == 0, "partial pack: shift ", sh, " not on the partial lattice of ", shift0);
        const Int off = (sh - shift0) / stridePart;
        const Int len = Length(cols ? h : w, sh, stride);
        const Int lh = cols ? len : h, lw = cols ? w : len;
        ELX_REQUIRE(lh * lw <= portionSize, "partial pack: portion ", k, " needs ", lh * lw, " elements");
        if (lh == 0 || lw == 0) continue;
        char* m = (char*)M + (cols ? off : off * ldm) * es;
        char* q = (char*)P + k * portionSize * es;
        const Int mcs = cols ? strideUnion : 1, mrs = cols ? ldm : strideUnion * ldm;
        if (pack) d.push_back({lh, lw, m, mcs, mrs, q, 1, lh});
        else d.push_back({lh, lw, q, 1, lh, m, mcs, mrs});
    }
    return d;
}
}  // namespace
extern "C" {

int elx_pack_strided(int device, int dtype, int64_t height, int64_t width, int64_t colAlign, int64_t colStride,
                     int64_t rowAlign, int64_t rowStride, const void* A, int64_t lda, void* portions,
                     int64_t portionSize, void* stream) {
    return Guard([&] {
        RunCopies(device, dtype,
                  StridedPlan(dtype, height, width, colAlign, colStride, rowAlign, rowStride, A, lda, portions,
                              portionSize, true),
                  false, 0.0, stream);
    });
}
int elx_unpack_strided(int device, int dtype, int64_t height, int64_t width, int64_t colAlign, int64_t colStride,
                       int64_t rowAlign, int64_t rowStride, const void* portions, int64_t portionSize, void* B,
                       int64_t ldb, void* stream) {
    return Guard([&] {
        RunCopies(device, dtype,
                  StridedPlan(dtype, height, width, colAlign, colStride, rowAlign, rowStride, B, ldb, portions,
                              portionSize, false),
                  false, 0.0, stream);
    });
}
int elx_pack_partial_strided(int device, int dtype, int cols, int64_t height, int64_t width, int64_t align,
                             int64_t stride, int64_t strideUnion, int64_t stridePart, int64_t rankPart,
                             int64_t shiftA, const void* A, int64_t lda, void* portions, int64_t portionSize,
                             void* stream) {
    return Guard([&] {
        RunCopies(device, dtype,
                  PartialPlan(dtype, cols != 0, height, width, align, stride, strideUnion, stridePart, rankPart,
                              shiftA, A, lda, portions, portionSize, true),
                  false, 0.0, stream);
    });
}
int elx_unpack_partial_strided(int device, int dtype, int cols, int64_t height, int64_t width, int64_t align,
                               int64_t stride, int64_t strideUnion, int64_t stridePart, int64_t rankPart,
                               int64_t shiftB, const void* portions, int64_t portionSize, void* B, int64_t ldb,
                               void* stream) {
    return Guard([&] {
        RunCopies(device, dtype,
                  PartialPlan(dtype, cols != 0, height, width, align, stride, strideUnion, stridePart, rankPart,
                              shiftB, B, ldb, portions, portionSize, false),
                  false, 0.0, stream);
    });
}
int elx_unpack_axpy_strided(int device, int dtype, int64_t height, int64_t width, double alpha, int64_t colAlign,
                            int64_t colStride, int64_t rowAlign, int64_t rowStride, const void* portions,
                            int64_t portionSize, void* B, int64_t ldb, void* stream) {
    return Guard([&] {  // the fused reduce-scatter epilogue: B(lattice k,l) += alpha * portion (Axpy/util.hpp:23-50)
        RunCopies(device, dtype,
                  StridedPlan(dtype, height, width, colAlign, colStride, rowAlign, rowStride, B, ldb, portions,
                              portionSize, false),
                  true, alpha, stream);
    });
}
int elx_transpose(int dtype, int64_t m, int64_t n, const void* A, int64_t lda, void* B, int64_t ldb, void* stream) {
    return Guard([&] {  // B (n x m) = A^T
        kern::Copy2D d{n, m, A, lda, 1, B, 1, ldb};
        exec::Copy2DBatch(Device::GPU, ToDType(dtype), &d, 1, false, 0.0, S(stream));
    });
}
int elx_scale2d(int dtype, int64_t m, int64_t n, double alpha, void* A, int64_t lda, void* stream) {
    return Guard([&] { exec::Scale(Device::GPU, ToDType(dtype), m, n, alpha, A, lda, S(stream)); });
}
int elx_fill2d(int dtype, int64_t m, int64_t n, double value, void* A, int64_t lda, void* stream) {
    return Guard([&] { exec::Fill(Device::GPU, ToDType(dtype), m, n, value, A, lda, S(stream)); });
}
int elx_hadamard2d(int dtype, int64_t m, int64_t n, const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                   int64_t ldc, void* stream) {
    return Guard([&] { exec::Hadamard(Device::GPU, ToDType(dtype), m, n, A, lda, B, ldb, C, ldc, S(stream)); });
}
int elx_entrywise_map(int dtype, int fn, int64_t m, int64_t n, const void* A, int64_t lda, void* B, int64_t ldb,
                      void* stream) {
    return Guard([&] { exec::Map(Device::GPU, ToDType(dtype), fn, m, n, A, lda, B, ldb, S(stream)); });
}
int elx_combine(int dtype, int fn, int64_t m, int64_t n, const void* A, int64_t lda, void* B, int64_t ldb,
                void* stream) {
    return Guard([&] { exec::Combine(Device::GPU, ToDType(dtype), fn, m, n, A, lda, B, ldb, S(stream)); });
}
int elx_fill_hash(int dtype, int64_t m, int64_t n, void* A, int64_t lda, int64_t i0, int64_t istride, int64_t j0,
                  int64_t jstride, uint64_t seed, double center, double radius, void* stream) {
    return Guard([&] {
        exec::FillHash(Device::GPU, ToDType(dtype), m, n, A, lda, i0, istride, j0, jstride, seed, center, radius,
                       S(stream));
    });
}

// ---- communication ---------------------------------------------------------
int elx_comm_unique_id(unsigned char id[128]) {
    return Guard([&] {
        ncclUniqueId uid;
        ncclResult_t r = ncclGetUniqueId(&uid);
        if (r != ncclSuccess) throw CommError(Cat("ncclGetUniqueId: ", ncclGetErrorString(r)));
        std::memcpy(id, uid.internal, 128);
    });
}
int elx_comm_init_rccl(elx_comm_t* world, int rank, int size, const unsigned char id[128]) {
    return Guard([&] { *world = new elx_comm_s{Comm::InitRCCL(rank, size, id)}; });
}
int elx_comm_init_host(elx_comm_t* world, int rank, int size, elx_host_coll_fn coll, elx_host_split_fn split,
                       void* ctx) {
    return Guard([&] {
        *world = new elx_comm_s{size == 1 && !coll ? Comm::Self() : Comm::InitHost(rank, size, coll, split, ctx)};
    });
}
int elx_comm_wrap_rccl(elx_comm_t* comm, void* nccl_comm) {
    return Guard([&] { *comm = new elx_comm_s{Comm::WrapRCCL(static_cast<ncclComm_t>(nccl_comm))}; });
}
int elx_comm_rank(elx_comm_t c, int* rank) { return Guard([&] { *rank = c->c->Rank(); }); }
int elx_comm_size(elx_comm_t c, int* size) { return Guard([&] { *size = c->c->Size(); }); }
int elx_comm_destroy(elx_comm_t c) { return Guard([&] { delete c; }); }
int elx_comm_world(elx_comm_t* comm) {
    return Guard([&] {
        WorldHandle().c = WorldComm();
        *comm = &WorldHandle();
    });
}
int elx_comm_set_world(elx_comm_t comm) {
    return Guard([&] {
        ELX_REQUIRE(comm && comm->c, "null comm");
        WorldComm() = comm->c;
        WorldHandle().c = comm->c;
    });
}
int elx_rendezvous_bcast(void* data, size_t bytes, int rank, int size, const char* addr, int port, double timeout_s) {
    return Guard([&] { RendezvousBcast(data, bytes, rank, size, addr, port, timeout_s); });
}
int elx_watchdog_stage(const char* name, double seconds) { return Guard([&] { WatchdogStage(name, seconds); }); }
int elx_watchdog_epitaph(const char* text, int exit_code) { return Guard([&] { WatchdogEpitaph(text, exit_code); }); }
int elx_comm_allgather(elx_comm_t c, int dtype, const void* send, void* recv, int64_t count, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "allgather: negative count ", count);
        const Device d = c->c->kind() == Comm::Kind::RCCL ? Device::GPU : Device::CPU;
        c->c->AllGather(ToDType(dtype), send, recv, count, d, d == Device::GPU ? S(stream) : nullptr);
    });
}
int elx_comm_reduce_scatter(elx_comm_t c, int dtype, const void* send, void* recv, int64_t count, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "reduce_scatter: negative count ", count);
        const Device d = c->c->kind() == Comm::Kind::RCCL ? Device::GPU : Device::CPU;
        c->c->ReduceScatter(ToDType(dtype), send, recv, count, d, d == Device::GPU ? S(stream) : nullptr);
    });
}
int elx_comm_barrier(elx_comm_t c) { return Guard([&] { c->c->Barrier(); }); }
// the rest of El::mpi's typed collectives (src/core/imports/mpi/*.hpp); counts in
// elements, device from the communicator's kind, as above
namespace {
Device CommDev(elx_comm_t c) { return c->c->kind() == Comm::Kind::RCCL ? Device::GPU : Device::CPU; }
hipStream_t CommStream(elx_comm_t c, void* stream) { return CommDev(c) == Device::GPU ? S(stream) : nullptr; }
}  // namespace
int elx_comm_split(elx_comm_t c, int color, int key, elx_comm_t* out) {
    return Guard([&] { *out = new elx_comm_s{c->c->Split(color, key)}; });
}
int elx_comm_allreduce(elx_comm_t c, int dtype, const void* send, void* recv, int64_t count, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "allreduce: negative count ", count);
        c->c->AllReduce(ToDType(dtype), send, recv, count, CommDev(c), CommStream(c, stream));
    });
}
int elx_comm_bcast(elx_comm_t c, int dtype, void* buf, int64_t count, int root, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "bcast: negative count ", count);
        ELX_REQUIRE(root >= 0 && root < c->c->Size(), "bcast: root ", root, " outside the communicator");
        c->c->Bcast(ToDType(dtype), buf, count, root, CommDev(c), CommStream(c, stream));
    });
}
int elx_comm_alltoall(elx_comm_t c, int dtype, const void* send, void* recv, int64_t count, void* stream) {
    return Guard([&] {
        // El::mpi::AllToAll (AllToAll.hpp:11-105): `count` elements to and from every rank
        ELX_REQUIRE(count >= 0, "alltoall: negative count ", count);
        const int p = c->c->Size();
        std::vector<Int> cnt(p, count), dsp(p);
        for (int q = 0; q < p; ++q) dsp[q] = (Int)q * count;
        c->c->AllToAllV(ToDType(dtype), send, cnt, dsp, recv, cnt, dsp, CommDev(c), CommStream(c, stream));
    });
}
int elx_comm_sendrecv(elx_comm_t c, int dtype, const void* send, int dest, void* recv, int src, int64_t count,
                      void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "sendrecv: negative count ", count);
        ELX_REQUIRE(dest >= 0 && dest < c->c->Size() && src >= 0 && src < c->c->Size(), "sendrecv: peer outside the communicator");
        c->c->SendRecv(ToDType(dtype), send, dest, recv, src, count, CommDev(c), CommStream(c, stream));
    });
}
extern "C++" {
namespace {
// El::mpi on explicit-device buffers.  Host buffers over an RCCL communicator of
// size > 1 go through device copies on the comm stream (RCCL reads device
// memory only) and the call is synchronous, as the reference's MPI path on
// Device::CPU is.  `inplace`: send and recv are one buffer (Broadcast).
template <class F>
void MpiRun(elx_comm_t c, int device, void* stream, const void* send, size_t sbytes, void* recv, size_t rbytes,
            bool inplace, F&& f) {
    ELX_REQUIRE(c && c->c, "null comm");
    ELX_REQUIRE(device == ELX_DEVICE_CPU || device == ELX_DEVICE_GPU, "unknown device ", device);
    const Device d = device == ELX_DEVICE_GPU ? Device::GPU : Device::CPU;
    if (c->c->kind() == Comm::Kind::RCCL && d == Device::CPU && c->c->Size() > 1) {
        hipStream_t s = Runtime::Get().CommStream();
        Buffer ds(Device::GPU, inplace ? 0 : std::max<size_t>(sbytes, 1), s);
        Buffer dr(Device::GPU, std::max<size_t>(rbytes, 1), s);
        if (inplace) {
            if (rbytes) ELX_CHECK_HIP(hipMemcpyAsync(dr.data(), recv, rbytes, hipMemcpyHostToDevice, s));
        } else if (sbytes) {
            ELX_CHECK_HIP(hipMemcpyAsync(ds.data(), send, sbytes, hipMemcpyHostToDevice, s));
        }
        f(inplace ? dr.data() : ds.data(), dr.data(), Device::GPU, s);
        if (rbytes) ELX_CHECK_HIP(hipMemcpyAsync(recv, dr.data(), rbytes, hipMemcpyDeviceToHost, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
        return;
    }
    f(send, recv, d, d == Device::GPU ? S(stream) : nullptr);
}
ReduceOp ToOp(int op) {
    ELX_REQUIRE(op >= ELX_OP_SUM && op <= ELX_OP_MIN, "unknown reduction op ", op);
    return static_cast<ReduceOp>(op);
}
}  // namespace
}  // extern "C++"
int elx_mpi_allgather(elx_comm_t c, int dtype, int device, const void* send, void* recv, int64_t count,
                      void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "allgather: negative count ", count);
        const DType t = ToCommDType(dtype);
        const size_t b = static_cast<size_t>(count) * DTypeSize(t);
        MpiRun(c, device, stream, send, b, recv, b * c->c->Size(), false,
               [&](const void* sb, void* rb, Device d, hipStream_t s) { c->c->AllGather(t, sb, rb, count, d, s); });
    });
}
int elx_mpi_reduce_scatter(elx_comm_t c, int dtype, int device, int op, const void* send, void* recv,
                           int64_t count, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "reduce_scatter: negative count ", count);
        const DType t = ToCommDType(dtype);
        const ReduceOp o = ToOp(op);
        const size_t b = static_cast<size_t>(count) * DTypeSize(t);
        MpiRun(c, device, stream, send, b * c->c->Size(), recv, b, false,
               [&](const void* sb, void* rb, Device d, hipStream_t s) { c->c->ReduceScatter(t, sb, rb, count, d, s, o); });
    });
}
int elx_mpi_allreduce(elx_comm_t c, int dtype, int device, int op, const void* send, void* recv, int64_t count,
                      void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "allreduce: negative count ", count);
        const DType t = ToCommDType(dtype);
        const ReduceOp o = ToOp(op);
        const size_t b = static_cast<size_t>(count) * DTypeSize(t);
        MpiRun(c, device, stream, send, b, recv, b, false,
               [&](const void* sb, void* rb, Device d, hipStream_t s) { c->c->AllReduce(t, sb, rb, count, d, s, o); });
    });
}
int elx_mpi_alltoall(elx_comm_t c, int dtype, int device, const void* send, void* recv, int64_t count,
                     void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "alltoall: negative count ", count);
        const DType t = ToCommDType(dtype);
        const int p = c->c->Size();
        const size_t b = static_cast<size_t>(count) * DTypeSize(t) * p;
        std::vector<Int> cnt(p, count), dsp(p);
        for (int q = 0; q < p; ++q) dsp[q] = (Int)q * count;
        MpiRun(c, device, stream, send, b, recv, b, false, [&](const void* sb, void* rb, Device d, hipStream_t s) {
            c->c->AllToAllV(t, sb, cnt, dsp, rb, cnt, dsp, d, s);
        });
    });
}
int elx_mpi_bcast(elx_comm_t c, int dtype, int device, void* buf, int64_t count, int root, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(count >= 0, "bcast: negative count ", count);
        ELX_REQUIRE(root >= 0 && root < c->c->Size(), "bcast: root ", root, " outside the communicator");
        const DType t = ToCommDType(dtype);
        const size_t b = static_cast<size_t>(count) * DTypeSize(t);
        MpiRun(c, device, stream, buf, b, buf, b, true,
               [&](const void*, void* rb, Device d, hipStream_t s) { c->c->Bcast(t, rb, count, root, d, s); });
    });
}
int elx_mpi_sendrecv(elx_comm_t c, int dtype, int device, const void* send, int64_t scount, int dest, void* recv,
                     int64_t rcount, int src, void* stream) {
    return Guard([&] {
        ELX_REQUIRE(scount >= 0 && rcount >= 0, "sendrecv: negative count");
        const DType t = ToCommDType(dtype);
        const size_t es = DTypeSize(t);
        MpiRun(c, device, stream, send, static_cast<size_t>(scount) * es, recv, static_cast<size_t>(rcount) * es,
               false, [&](const void* sb, void* rb, Device d, hipStream_t s) {
                   c->c->SendRecv(t, sb, scount, dest, rb, rcount, src, d, s);
               });
    });
}
int elx_comm_stats(int64_t* bytes, double* seconds, int64_t* calls) {
    return Guard([&] {
        auto& s = GlobalCommStats();
        *bytes = s.bytes;
        *seconds = s.seconds;
        *calls = s.calls;
    });
}
int elx_comm_stats_reset(void) { return Guard([&] { GlobalCommStats() = CommStats{}; }); }

// ---- grid ----------------------------------------------------------------------
int elx_grid_default_height(int size) { return size > 0 ? Grid::DefaultHeight(size) : 0; }
int elx_grid_create(elx_grid_t* grid, elx_comm_t world, int height, int order) {
    return Guard([&] {
        ELX_REQUIRE(world && world->c, "null comm");
        ELX_REQUIRE(order == ELX_ROW_MAJOR || order == ELX_COLUMN_MAJOR, "bad grid order");
        *grid = new elx_grid_s{std::make_shared<Grid>(world->c, height, order)};
    });
}
int elx_grid_info(elx_grid_t g, int* info) {
    return Guard([&] {
        const Grid& G = *g->g;
        int v[8] = {G.Height(), G.Width(), G.Size(), G.Rank(), G.MCRank(), G.MRRank(), G.VCRank(), G.VRRank()};
        std::memcpy(info, v, sizeof(v));
    });
}
int elx_grid_destroy(elx_grid_t g) { return Guard([&] { delete g; }); }

// ---- DistMatrix ------------------------------------------------------------------
int elx_dm_create(elx_dm_t* A, elx_grid_t g, int dtype, int coldist, int rowdist, int device, int root) {
    return Guard([&] {
        ELX_REQUIRE(g && g->g, "null grid");
        *A = new elx_dm_s{std::make_shared<DistMatrix>(g->g, ToDType(dtype), ToDist(coldist), ToDist(rowdist),
                                                       ToDevice(device), root)};
    });
}
int elx_dm_destroy(elx_dm_t A) { return Guard([&] { delete A; }); }
int elx_dm_align(elx_dm_t A, int ca, int ra, int constrain) { return Guard([&] { M(A).Align(ca, ra, constrain != 0); }); }
int elx_dm_align_with(elx_dm_t A, elx_dm_t B, int constrain) { return Guard([&] { M(A).AlignWith(M(B), constrain != 0); }); }
int elx_dm_resize(elx_dm_t A, int64_t h, int64_t w) { return Guard([&] { M(A).Resize(h, w); }); }
int elx_dm_info(elx_dm_t A, int64_t* info) {
    return Guard([&] {
        const DistMatrix& X = M(A);
        const bool p = X.Participating();
        int64_t v[13] = {X.Height(), X.Width(), X.LocalHeight(), X.LocalWidth(), X.LDim(), X.ColAlign(),
                         X.RowAlign(), p ? X.ColShift() : 0, p ? X.RowShift() : 0, X.ColStride(), X.RowStride(),
                         p ? 1 : 0, X.Viewing() ? 1 : 0};
        std::memcpy(info, v, sizeof(v));
    });
}
int elx_dm_buffer(elx_dm_t A, void** ptr) { return Guard([&] { *ptr = M(A).Buffer(); }); }
int elx_dm_set_local(elx_dm_t A, const void* host, int64_t ld) { return Guard([&] { M(A).SetLocal(host, ld); }); }
int elx_dm_get_local(elx_dm_t A, void* host, int64_t ld) { return Guard([&] { M(A).GetLocal(host, ld); }); }
int elx_dm_frobenius_norm(elx_dm_t A, double* out) { return Guard([&] { *out = FrobeniusNorm(M(A)); }); }
int elx_dm_view(elx_dm_t* V, elx_dm_t A, int64_t i0, int64_t i1, int64_t j0, int64_t j1) {
    return Guard([&] { *V = new elx_dm_s{DistMatrix::View(M(A), i0, i1, j0, j1)}; });
}
int elx_dm_attach(elx_dm_t A, int64_t height, int64_t width, int colAlign, int rowAlign, void* buffer,
                  int64_t ldim, int root) {
    return Guard([&] { M(A).Attach(height, width, colAlign, rowAlign, buffer, ldim, root); });
}
int elx_dm_copy(elx_dm_t B, elx_dm_t A) { return Guard([&] { Copy(M(A), M(B)); }); }
int elx_dm_transpose(elx_dm_t A, elx_dm_t B) { return Guard([&] { Transpose(M(A), M(B)); }); }
int elx_dm_fill_hash(elx_dm_t A, uint64_t seed, double center, double radius) {
    return Guard([&] { M(A).FillHash(seed, center, radius); });
}
int elx_initialize_random(int deterministic, int world_rank) {
    return Guard([&] { InitializeRandom(deterministic != 0, world_rank); });
}
int elx_dm_uniform(elx_dm_t A, int64_t height, int64_t width, double center, double radius) {
    return Guard([&] { Uniform(M(A), height, width, center, radius); });
}
int elx_dm_make_uniform(elx_dm_t A, double center, double radius) {
    return Guard([&] { MakeUniform(M(A), center, radius); });
}
int elx_dm_synchronize(elx_dm_t A) { return Guard([&] { M(A).Synchronize(); }); }
int elx_dm_set_stream(elx_dm_t A, void* stream) {
    return Guard([&] { M(A).SetStream(stream ? static_cast<hipStream_t>(stream) : Runtime::Get().ComputeStream()); });
}
int elx_dm_stream(elx_dm_t A, void** stream) { return Guard([&] { *stream = M(A).Stream(); }); }
int elx_dm_write(elx_dm_t A, const char* basename, int format, int int_bytes) {
    return Guard([&] {
        ELX_REQUIRE(basename != nullptr, "null file name");
        Write(M(A), basename, format, int_bytes);
    });
}
int elx_dm_read(elx_dm_t A, const char* filename, int format, int int_bytes) {
    return Guard([&] {
        ELX_REQUIRE(filename != nullptr, "null file name");
        Read(M(A), filename, format, int_bytes);
    });
}

int elx_dm_get(elx_dm_t A, int64_t i, int64_t j, double* value) { return Guard([&] { *value = Get(M(A), i, j); }); }
int elx_dm_set(elx_dm_t A, int64_t i, int64_t j, double value) { return Guard([&] { Set(M(A), i, j, value); }); }
int elx_dm_update(elx_dm_t A, int64_t i, int64_t j, double value) { return Guard([&] { Update(M(A), i, j, value); }); }
int elx_dm_fill(elx_dm_t A, double value) { return Guard([&] { Fill(M(A), value); }); }

int elx_dm_axpy(double alpha, elx_dm_t X, elx_dm_t Y) { return Guard([&] { Axpy(alpha, M(X), M(Y)); }); }
int elx_dm_scale(double alpha, elx_dm_t A) { return Guard([&] { Scale(alpha, M(A)); }); }
int elx_dm_zero(elx_dm_t A) { return Guard([&] { Zero(M(A)); }); }
int elx_dm_hadamard(elx_dm_t A, elx_dm_t B, elx_dm_t C) { return Guard([&] { Hadamard(M(A), M(B), M(C)); }); }
int elx_dm_entrywise_map(int fn, elx_dm_t A, elx_dm_t B) { return Guard([&] { EntrywiseMap(fn, M(A), M(B)); }); }
int elx_dm_combine(int fn, elx_dm_t A, elx_dm_t B) { return Guard([&] { Combine(fn, M(A), M(B)); }); }
int elx_dm_axpy_contract(double alpha, elx_dm_t A, elx_dm_t B) { return Guard([&] { AxpyContract(alpha, M(A), M(B)); }); }

int elx_gemm(int oA, int oB, double alpha, elx_dm_t A, elx_dm_t B, double beta, elx_dm_t C, int alg) {
    return Guard([&] {
        CheckOp(oA);
        CheckOp(oB);
        ELX_REQUIRE(alg >= ELX_GEMM_DEFAULT && alg <= ELX_GEMM_CANNON, "invalid GemmAlgorithm ", alg);
        Gemm(oA, oB, alpha, M(A), M(B), beta, M(C), alg);
    });
}
int elx_local_gemm(int oA, int oB, double alpha, elx_dm_t A, elx_dm_t B, double beta, elx_dm_t C) {
    return Guard([&] {
        CheckOp(oA);
        CheckOp(oB);
        LocalGemm(oA == ELX_NORMAL ? ELX_NORMAL : ELX_TRANSPOSE, oB == ELX_NORMAL ? ELX_NORMAL : ELX_TRANSPOSE, alpha,
                  M(A), M(B), beta, M(C));
    });
}
int elx_syrk(int uplo, int orient, double alpha, elx_dm_t A, double beta, elx_dm_t C, int conjugate) {
    (void)conjugate;  // real types: Herk == Syrk
    return Guard([&] {
        CheckOp(orient);
        Syrk(uplo, orient, alpha, M(A), beta, M(C));
    });
}
int elx_trrk(int uplo, int oA, int oB, double alpha, elx_dm_t A, elx_dm_t B, double beta, elx_dm_t C) {
    return Guard([&] {
        CheckOp(oA);
        CheckOp(oB);
        Trrk(uplo, oA, oB, alpha, M(A), M(B), beta, M(C));
    });
}
int elx_syr2k(int uplo, int orient, double alpha, elx_dm_t A, elx_dm_t B, double beta, elx_dm_t C, int conjugate) {
    (void)conjugate;  // real types: Her2k == Syr2k
    return Guard([&] {
        CheckOp(orient);
        Syr2k(uplo, orient, alpha, M(A), M(B), beta, M(C));
    });
}
int elx_trsm(int side, int uplo, int orient, int diag, double alpha, elx_dm_t A, elx_dm_t B, int checkIfSingular) {
    return Guard([&] {
        CheckOp(orient);
        Trsm(side, uplo, orient, diag, alpha, M(A), M(B), checkIfSingular != 0);
    });
}
int elx_symm(int side, int uplo, double alpha, elx_dm_t A, elx_dm_t B, double beta, elx_dm_t C, int conjugate) {
    (void)conjugate;  // real types: Hemm == Symm
    return Guard([&] { Symm(side, uplo, alpha, M(A), M(B), beta, M(C)); });
}
int elx_dm_scale_trapezoid(double alpha, int uplo, elx_dm_t A, int64_t offset) {
    return Guard([&] { ScaleTrapezoid(alpha, uplo, M(A), offset); });
}
int elx_set_blocksize(int64_t nb) { return Guard([&] { SetBlocksize(nb); }); }
int64_t elx_blocksize(void) {
    int64_t nb = -1;
    (void)Guard([&] { nb = Blocksize(); });
    return nb;
}
int elx_push_blocksize(int64_t nb) { return Guard([&] { PushBlocksizeStack(nb); }); }
int elx_pop_blocksize(void) { return Guard([&] { PopBlocksizeStack(); }); }
int elx_empty_blocksize_stack(void) { return Guard([&] { EmptyBlocksizeStack(); }); }
int elx_initialize(void) {
    return Guard([&] {
        InitWorldFromEnv();
        EmptyBlocksizeStack();
        PushBlocksizeStack(128);
        InitializeRandom(true, WorldComm()->Rank());
    });
}
int elx_finalize(void) {
    return Guard([&] {
        WorldComm() = Comm::Self();
        if (WorldHandle().c) WorldHandle().c = WorldComm();
        EmptyBlocksizeStack();
    });
}
int elx_set_compute_panel(int64_t kc) { return Guard([&] { SetComputePanel(kc); }); }
int elx_last_gemm_algorithm(void) { return LastGemmAlgorithm(); }
int elx_set_stream_pool_size(int n) { return Guard([&] { SetStreamPoolSize(n); }); }
int elx_stream_pool_size(void) { return StreamPoolSize(); }
int elx_set_profiling(int on) { return Guard([&] { SetProfiling(on != 0); }); }
int elx_profile_stats(double* gemm_ms, int64_t* launches, double* flops, double* comm_ms, int64_t* bytes) {
    return Guard([&] { ProfileStats(*gemm_ms, *launches, *flops, *comm_ms, *bytes); });
}
int elx_profile_transfers(double* transfer_ms, int64_t* bytes, int64_t* transfers) {
    return Guard([&] { CommProfileStats(*transfer_ms, *bytes, *transfers); });
}
int elx_profile_pipeline(double* gap_ms, int64_t* gaps) { return Guard([&] { PipelineStats(*gap_ms, *gaps); }); }

}  // extern "C"
