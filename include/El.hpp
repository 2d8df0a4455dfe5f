// El.hpp — drop-in C++ surface of the El::Gemm path (header-only, over the C-ABI
// in elemental_amd.h).  Names, signatures, enum ordinals and exception types
// follow the reference (include/El/core/types.hpp, include/El/core/Grid.hpp,
// include/El/core/DistMatrix/*, include/El/blas_like/level3.hpp:20-90,
// include/El/blas_like/level1/*) so LBANN-style callers recompile against it:
//
//   El::Initialize(argc, argv);                  // RCCL world from RANK / WORLD_SIZE (torchrun)
//   El::Grid g(El::mpi::COMM_WORLD);              // or a communicator over RCCL / a host bridge
//   El::DistMatrix<double, El::MC, El::MR, El::ELEMENT, El::Device::GPU> A(m, k, g), B(k, n, g), C(m, n, g);
//   El::Gemm(El::NORMAL, El::NORMAL, 1.0, A, B, 0.0, C);
//
// Link with -lelemental_amd (elemental_amd/libelemental_amd.so).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <exception>
#include <initializer_list>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "elemental_amd.h"

// HIP's handle types, declared exactly as hip_runtime_api.h does, so this
// header needs no HIP include and mixes with one.
typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;

// ---- hydrogen: devices, SyncInfo, MultiSync ------------------------------------
// include/hydrogen/Device.hpp, SyncInfoBase.hpp, SynchronizeAPI.hpp,
// MultiSync.hpp:33-78, device/gpu/rocm/SyncInfo.hpp:15-81, device/GPU.hpp:130-160
namespace hydrogen {

enum class Device : unsigned char { CPU = ELX_DEVICE_CPU, GPU = ELX_DEVICE_GPU };

// 16-bit element types: gpu_half_type (rocblas_half in the reference,
// include/hydrogen/utils/HalfPrecision.hpp:123) and bfloat16 (new).
struct gpu_half_type { std::uint16_t x; };
struct bfloat16 { std::uint16_t x; };

struct GPUError : std::runtime_error { using std::runtime_error::runtime_error; };  // hydrogen::GPUError

namespace detail {
[[noreturn]] inline void ThrowGPU() { throw GPUError(elx_last_error()); }
inline void CheckGPU(int rc) { if (rc != ELX_OK) ThrowGPU(); }
}  // namespace detail

template <Device D> class SyncInfo;

// CPU work is synchronous with the host: nothing to carry
template <> class SyncInfo<Device::CPU> {
public:
    SyncInfo() noexcept = default;
};

// a HIP stream and an event recorded on it to mark sync points
template <> class SyncInfo<Device::GPU> {
public:
    SyncInfo();  // the library's default stream and event
    SyncInfo(hipStream_t stream, hipEvent_t event) noexcept : stream_(stream), event_(event) {}
    // take the other's non-null parts (SyncInfo.hpp:27-33)
    void Merge(SyncInfo const& si) noexcept {
        if (si.stream_) stream_ = si.stream_;
        if (si.event_) event_ = si.event_;
    }
    hipStream_t Stream() const noexcept { return stream_; }
    hipEvent_t Event() const noexcept { return event_; }

private:
    friend void DestroySyncInfo(SyncInfo<Device::GPU>&);
    hipStream_t stream_ = nullptr;
    hipEvent_t event_ = nullptr;
};

inline bool operator==(SyncInfo<Device::CPU> const&, SyncInfo<Device::CPU> const&) { return true; }
inline bool operator!=(SyncInfo<Device::CPU> const&, SyncInfo<Device::CPU> const&) { return false; }
inline bool operator==(SyncInfo<Device::GPU> const& a, SyncInfo<Device::GPU> const& b) {
    return a.Stream() == b.Stream() && a.Event() == b.Event();
}
inline bool operator!=(SyncInfo<Device::GPU> const& a, SyncInfo<Device::GPU> const& b) { return !(a == b); }
template <Device D1, Device D2> bool operator==(SyncInfo<D1> const&, SyncInfo<D2> const&) { return false; }
template <Device D1, Device D2> bool operator!=(SyncInfo<D1> const&, SyncInfo<D2> const&) { return true; }

namespace gpu {
// the SyncInfo Hydrogen uses by default: the library's compute stream (not the
// HIP null stream) and its event (GPU.hpp:130-144)
inline SyncInfo<Device::GPU> const& DefaultSyncInfo() {
    static const SyncInfo<Device::GPU> si = [] {
        void* s = nullptr;
        void* e = nullptr;
        detail::CheckGPU(elx_default_stream(&s));
        detail::CheckGPU(elx_default_event(&e));
        return SyncInfo<Device::GPU>(static_cast<hipStream_t>(s), static_cast<hipEvent_t>(e));
    }();
    return si;
}
}  // namespace gpu

inline SyncInfo<Device::GPU>::SyncInfo() : SyncInfo(gpu::DefaultSyncInfo()) {}

// a new non-blocking stream and a new event (CPU: empty)
template <Device D> SyncInfo<D> CreateNewSyncInfo();
template <> inline SyncInfo<Device::CPU> CreateNewSyncInfo<Device::CPU>() { return SyncInfo<Device::CPU>{}; }
template <> inline SyncInfo<Device::GPU> CreateNewSyncInfo<Device::GPU>() {
    void* s = nullptr;
    void* e = nullptr;
    detail::CheckGPU(elx_stream_create(&s));
    if (elx_event_create(&e) != ELX_OK) {
        (void)elx_stream_destroy(s);
        detail::ThrowGPU();
    }
    return SyncInfo<Device::GPU>(static_cast<hipStream_t>(s), static_cast<hipEvent_t>(e));
}
inline void DestroySyncInfo(SyncInfo<Device::CPU>&) noexcept {}
inline void DestroySyncInfo(SyncInfo<Device::GPU>& si) {
    if (si.stream_) detail::CheckGPU(elx_stream_destroy(si.stream_));
    if (si.event_) detail::CheckGPU(elx_event_destroy(si.event_));
    si.stream_ = nullptr;
    si.event_ = nullptr;
}

// block the host until the SyncInfo's queued work is done
inline void Synchronize(SyncInfo<Device::CPU> const&) {}
inline void Synchronize(SyncInfo<Device::GPU> const& si) { detail::CheckGPU(elx_stream_synchronize(si.Stream())); }

// mark this point of the SyncInfo's stream
inline void AddSynchronizationPoint(SyncInfo<Device::CPU> const&) {}
inline void AddSynchronizationPoint(SyncInfo<Device::GPU> const& si) {
    detail::CheckGPU(elx_event_record(si.Event(), si.Stream()));
}

namespace details {
// `dependent` waits for the work captured at master's last sync point
inline void AddSyncPoint(SyncInfo<Device::CPU> const&, SyncInfo<Device::CPU> const&) {}
inline void AddSyncPoint(SyncInfo<Device::CPU> const&, SyncInfo<Device::GPU> const&) {}
inline void AddSyncPoint(SyncInfo<Device::GPU> const& master, SyncInfo<Device::CPU> const&) { Synchronize(master); }
inline void AddSyncPoint(SyncInfo<Device::GPU> const& master, SyncInfo<Device::GPU> const& other) {
    if (master.Stream() != other.Stream()) detail::CheckGPU(elx_stream_wait_event(other.Stream(), master.Event()));
}
}  // namespace details

// the "others" wait for the master (SynchronizeAPI.hpp)
template <Device D, Device... Ds>
void AddSynchronizationPoint(SyncInfo<D> const& master, SyncInfo<Ds> const&... others) {
    AddSynchronizationPoint(master);
    int dummy[] = {0, (details::AddSyncPoint(master, others), 0)...};
    (void)dummy;
}
template <Device D, Device... Ds>
void AllWaitOnMaster(SyncInfo<D> const& master, SyncInfo<Ds> const&... others) {
    AddSynchronizationPoint(master, others...);
}
template <Device D, Device... Ds>
void MasterWaitOnAll(SyncInfo<D> const& master, SyncInfo<Ds> const&... others) {
    int dummy[] = {0, (AddSynchronizationPoint(others, master), 0)...};
    (void)dummy;
}

// RAII: construction makes the first (master) SyncInfo wait on the others,
// destruction makes the others wait on the master (MultiSync.hpp:33-78)
template <Device... Ds>
class MultiSync {
    using tuple_type = std::tuple<SyncInfo<Ds>...>;
    using master_type = typename std::tuple_element<0, tuple_type>::type;

public:
    explicit MultiSync(SyncInfo<Ds> const&... sis) : sis_{sis...} { MasterWaitOnAll(sis...); }
    ~MultiSync() { Release(std::make_index_sequence<sizeof...(Ds)>{}); }
    MultiSync(MultiSync&& o) noexcept : sis_(o.sis_) { o.moved_ = true; }
    MultiSync(MultiSync const&) = delete;
    MultiSync& operator=(MultiSync const&) = delete;
    operator master_type const&() const noexcept { return std::get<0>(sis_); }

private:
    template <std::size_t... Is>
    void Release(std::index_sequence<Is...>) {
        if (!moved_) AllWaitOnMaster(std::get<Is>(sis_)...);
    }
    tuple_type sis_;
    bool moved_ = false;
};
template <Device... Ds>
MultiSync<Ds...> MakeMultiSync(SyncInfo<Ds> const&... sis) {
    return MultiSync<Ds...>(sis...);
}

}  // namespace hydrogen

namespace El {

using Int = std::int64_t;
// the reference brings hydrogen's names into El (include/El/core.hpp:74-79)
using hydrogen::Device;
using hydrogen::SyncInfo;
using hydrogen::MultiSync;
using hydrogen::MakeMultiSync;
using hydrogen::CreateNewSyncInfo;
using hydrogen::DestroySyncInfo;
using hydrogen::Synchronize;
using hydrogen::AddSynchronizationPoint;
using hydrogen::gpu_half_type;
using hydrogen::bfloat16;
namespace gpu = hydrogen::gpu;

// ---- enums (ordinals match the reference) --------------------------------
enum Dist { MC = ELX_MC, MD = ELX_MD, MR = ELX_MR, VC = ELX_VC, VR = ELX_VR, STAR = ELX_STAR, CIRC = ELX_CIRC };
enum DistWrap { ELEMENT = 0, BLOCK = 1 };
enum Orientation { NORMAL = ELX_NORMAL, TRANSPOSE = ELX_TRANSPOSE, ADJOINT = ELX_ADJOINT };
enum UpperOrLower { LOWER = ELX_LOWER, UPPER = ELX_UPPER };
enum LeftOrRight { LEFT = ELX_LEFT, RIGHT = ELX_RIGHT };
enum UnitOrNonUnit { NON_UNIT = ELX_NON_UNIT, UNIT = ELX_UNIT };
enum GridOrder { ROW_MAJOR = ELX_ROW_MAJOR, COLUMN_MAJOR = ELX_COLUMN_MAJOR };
enum GemmAlgorithm {
    GEMM_DEFAULT = ELX_GEMM_DEFAULT, GEMM_SUMMA_A_MS = ELX_GEMM_SUMMA_A_MS, GEMM_SUMMA_A = ELX_GEMM_SUMMA_A,
    GEMM_SUMMA_B_MS = ELX_GEMM_SUMMA_B_MS, GEMM_SUMMA_B = ELX_GEMM_SUMMA_B, GEMM_SUMMA_C_MS = ELX_GEMM_SUMMA_C_MS,
    GEMM_SUMMA_C = ELX_GEMM_SUMMA_C, GEMM_SUMMA_DOT = ELX_GEMM_SUMMA_DOT, GEMM_CANNON = ELX_GEMM_CANNON
};
// include/El/core/types.hpp:543-559 (the formats of the GEMM path's fixtures)
enum FileFormat { AUTO = ELX_FILE_AUTO, BINARY = ELX_FILE_BINARY, BINARY_FLAT = ELX_FILE_BINARY_FLAT };

// ---- errors: the reference's exception types ------------------------------
struct LogicError : std::logic_error { using std::logic_error::logic_error; };
struct RuntimeError : std::runtime_error { using std::runtime_error::runtime_error; };
struct UnsupportedError : LogicError { using LogicError::LogicError; };
namespace hydrogen_errors {
using hydrogen::GPUError;  // the round-2 spelling
}
// include/El/core/environment/decl.hpp:209-214
struct SingularMatrixException : std::runtime_error {
    explicit SingularMatrixException(const char* msg = "Matrix was singular") : std::runtime_error(msg) {}
};

namespace detail {
// rc's exception; `msg` when the library's last error was overwritten since
inline void Check(int rc, const std::string& saved = std::string()) {
    if (rc == ELX_OK) return;
    const std::string msg = saved.empty() ? std::string(elx_last_error()) : saved;
    switch (rc) {
    case ELX_ERR_LOGIC: throw LogicError(msg);
    case ELX_ERR_UNSUPPORTED: throw UnsupportedError(msg);
    case ELX_ERR_HIP:
    case ELX_ERR_NO_DEVICE: throw hydrogen::GPUError(msg);
    case ELX_ERR_SINGULAR: throw SingularMatrixException(msg.c_str());
    default: throw RuntimeError(msg);
    }
}
template <typename T> struct TypeCode;
template <> struct TypeCode<float> { static constexpr int value = ELX_F32; };
template <> struct TypeCode<double> { static constexpr int value = ELX_F64; };
template <> struct TypeCode<gpu_half_type> { static constexpr int value = ELX_F16; };
template <> struct TypeCode<bfloat16> { static constexpr int value = ELX_BF16; };
// communication-only element types (El::mpi on Int / int / byte buffers)
template <> struct TypeCode<std::int32_t> { static constexpr int value = ELX_I32; };
template <> struct TypeCode<std::int64_t> { static constexpr int value = ELX_I64; };
template <> struct TypeCode<unsigned char> { static constexpr int value = ELX_U8; };
template <typename T> double ToDouble(T x) { return static_cast<double>(x); }
template <typename T> T FromDouble(double v) { return static_cast<T>(v); }
// 16-bit values cross the boundary as their exact double widening
inline double HalfBitsToDouble(std::uint16_t h) {
    const int e = (h >> 10) & 0x1f, m = h & 0x3ff;
    const double mag = e == 0 ? std::ldexp(m, -24) : e == 31 ? (m ? NAN : INFINITY) : std::ldexp(1024 + m, e - 25);
    return (h & 0x8000) ? -mag : mag;
}
inline double BF16BitsToDouble(std::uint16_t b) {
    const std::uint32_t u = static_cast<std::uint32_t>(b) << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
template <> inline double ToDouble(gpu_half_type x) { return HalfBitsToDouble(x.x); }
template <> inline double ToDouble(bfloat16 x) { return BF16BitsToDouble(x.x); }
// double -> 16-bit with one round-to-nearest-even (through float is exact for
// the values Get returns, which are 16-bit already)
inline std::uint16_t FloatToBF16Bits(float f) {
    std::uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<std::uint16_t>((u >> 16) | 0x40);
    return static_cast<std::uint16_t>((u + 0x7fffu + ((u >> 16) & 1)) >> 16);
}
inline std::uint16_t FloatToHalfBits(float f) {
    std::uint32_t u;
    std::memcpy(&u, &f, 4);
    const std::uint32_t sign = (u >> 16) & 0x8000u, a = u & 0x7fffffffu;
    if (a >= 0x7f800000u) return static_cast<std::uint16_t>(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0));
    if (a >= 0x477ff000u) return static_cast<std::uint16_t>(sign | 0x7c00u);
    if (a < 0x33000001u) return static_cast<std::uint16_t>(sign);
    const int e = static_cast<int>(a >> 23);
    std::uint32_t man = (a & 0x7fffffu) | 0x800000u;
    const int shift = e < 113 ? 126 - e : 13;
    std::uint32_t mm = man >> shift;
    const std::uint32_t rem = man & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (mm & 1))) ++mm;
    if (e < 113) return static_cast<std::uint16_t>(sign | mm);
    return static_cast<std::uint16_t>(sign | (((e - 112) << 10) + (mm - 1024)));
}
template <> inline gpu_half_type FromDouble(double v) { return gpu_half_type{FloatToHalfBits(static_cast<float>(v))}; }
template <> inline bfloat16 FromDouble(double v) { return bfloat16{FloatToBF16Bits(static_cast<float>(v))}; }
}  // namespace detail

// ---- Range / views ---------------------------------------------------------
struct Range { Int beg, end; };
inline Range IR(Int beg, Int end) { return Range{beg, end}; }
inline Range IR(Int i) { return Range{i, i + 1}; }
struct AllRange {};
static constexpr AllRange ALL{};

// ---- communicator ----------------------------------------------------------
namespace mpi {
class Comm {
public:
    Comm() = default;
    explicit Comm(elx_comm_t c) : c_(c, [](elx_comm_s* p) { if (p) elx_comm_destroy(p); }) {}
    // size-1 communicator (COMM_SELF)
    static Comm Self() {
        elx_comm_t c = nullptr;
        detail::Check(elx_comm_init_host(&c, 0, 1, nullptr, nullptr, nullptr));
        return Comm(c);
    }
    // RCCL world: every rank passes the same 128-byte id (elx_comm_unique_id on one rank)
    static Comm RCCL(int rank, int size, const unsigned char id[128]) {
        elx_comm_t c = nullptr;
        detail::Check(elx_comm_init_rccl(&c, rank, size, id));
        return Comm(c);
    }
    // a communicator the caller already owns (e.g. LBANN's ncclComm_t); borrowed, not destroyed
    static Comm FromRCCL(void* ncclComm) {
        elx_comm_t c = nullptr;
        detail::Check(elx_comm_wrap_rccl(&c, ncclComm));
        return Comm(c);
    }
    // the world communicator (what COMM_WORLD names), resolved when used
    struct WorldTag {};
    explicit Comm(WorldTag) noexcept : world_(true) {}
    int Rank() const { int r = 0; detail::Check(elx_comm_rank(Handle(), &r)); return r; }
    int Size() const { int s = 1; detail::Check(elx_comm_size(Handle(), &s)); return s; }
    elx_comm_t Handle() const {
        if (!world_) return c_.get();
        elx_comm_t w = nullptr;  // borrowed from the library
        detail::Check(elx_comm_world(&w));
        return w;
    }
    // make this communicator the world (what COMM_WORLD and Grid() then use)
    void InstallAsWorld() const { detail::Check(elx_comm_set_world(Handle())); }
private:
    std::shared_ptr<elx_comm_s> c_;
    bool world_ = false;
};
// El::mpi::COMM_WORLD / COMM_SELF (include/El/core/imports/mpi.hpp:84-86): the
// world is the library's (El::Initialize builds it; Comm::InstallAsWorld
// replaces it), COMM_SELF a size-1 communicator
inline const Comm COMM_WORLD{Comm::WorldTag{}};
inline Comm COMM_SELF() { return Comm::Self(); }
inline int Rank(const Comm& comm = COMM_WORLD) { return comm.Rank(); }
inline int Size(const Comm& comm = COMM_WORLD) { return comm.Size(); }
inline void Barrier(const Comm& comm = COMM_WORLD) { detail::Check(elx_comm_barrier(comm.Handle())); }

// ---- typed collectives on SyncInfo-tagged buffers (include/El/core/imports/mpi.hpp) ----
// Device::GPU: device buffers, enqueued on the SyncInfo's stream after its
// queued work (RCCL; the host backend stages and synchronizes), as the
// reference's Aluminum path does; Device::CPU: host buffers, returns when done.
// El::mpi::Op (mpi.hpp:88-99): the reductions RCCL runs natively.
struct Op { int code; };
inline constexpr Op SUM{ELX_OP_SUM};
inline constexpr Op PROD{ELX_OP_PROD};
inline constexpr Op MAX{ELX_OP_MAX};
inline constexpr Op MIN{ELX_OP_MIN};
namespace detail_ {
inline void* StreamOf(SyncInfo<Device::CPU> const&) noexcept { return nullptr; }
inline void* StreamOf(SyncInfo<Device::GPU> const& si) noexcept { return si.Stream(); }
template <Device D> constexpr int DevCode() noexcept { return static_cast<int>(D); }
}  // namespace detail_

// Broadcast (mpi.hpp:675-720)
template <typename T, Device D>
void Broadcast(T* buffer, int count, int root, Comm const& comm, SyncInfo<D> const& si) {
    detail::Check(elx_mpi_bcast(comm.Handle(), detail::TypeCode<T>::value, detail_::DevCode<D>(), buffer, count, root,
                                detail_::StreamOf(si)));
}
template <typename T, Device D>
void Broadcast(T& b, int root, Comm const& comm, SyncInfo<D> const& si) { Broadcast(&b, 1, root, comm, si); }

// AllGather (mpi.hpp:861-930): rbuf holds rc * Size(comm) entries, sc == rc
template <typename T, Device D>
void AllGather(T const* sbuf, int sc, T* rbuf, int rc, Comm const& comm, SyncInfo<D> const& si) {
    if (sc != rc) throw LogicError("AllGather: send and receive counts must match");
    detail::Check(elx_mpi_allgather(comm.Handle(), detail::TypeCode<T>::value, detail_::DevCode<D>(), sbuf, rbuf, sc,
                                    detail_::StreamOf(si)));
}

// AllToAll (mpi.hpp:1006-1075): sc entries to and rc entries from every rank, sc == rc
template <typename T, Device D>
void AllToAll(T const* sbuf, int sc, T* rbuf, int rc, Comm const& comm, SyncInfo<D> const& si) {
    if (sc != rc) throw LogicError("AllToAll: send and receive counts must match");
    detail::Check(elx_mpi_alltoall(comm.Handle(), detail::TypeCode<T>::value, detail_::DevCode<D>(), sbuf, rbuf, sc,
                                   detail_::StreamOf(si)));
}

// AllReduce (mpi.hpp:1248-1351): out-of-place, in-place, default SUM, scalar
template <typename T, Device D>
void AllReduce(T const* sbuf, T* rbuf, int count, Op op, Comm const& comm, SyncInfo<D> const& si) {
    detail::Check(elx_mpi_allreduce(comm.Handle(), detail::TypeCode<T>::value, detail_::DevCode<D>(), op.code, sbuf,
                                    rbuf, count, detail_::StreamOf(si)));
}
template <typename T, Device D>
void AllReduce(T const* sbuf, T* rbuf, int count, Comm const& comm, SyncInfo<D> const& si) {
    AllReduce(sbuf, rbuf, count, SUM, comm, si);
}
template <typename T, Device D>
void AllReduce(T* buf, int count, Op op, Comm const& comm, SyncInfo<D> const& si) {
    AllReduce(static_cast<T const*>(buf), buf, count, op, comm, si);
}
template <typename T, Device D>
void AllReduce(T* buf, int count, Comm const& comm, SyncInfo<D> const& si) { AllReduce(buf, count, SUM, comm, si); }
// the scalar forms take host values (the reference's one-element overloads)
template <typename T, Device D>
T AllReduce(T sb, Op op, Comm const& comm, SyncInfo<D> const&) {
    T rb = sb;
    AllReduce(&sb, &rb, 1, op, comm, SyncInfo<Device::CPU>{});
    return rb;
}
template <typename T, Device D>
T AllReduce(T sb, Comm const& comm, SyncInfo<D> const& si) { return AllReduce(sb, SUM, comm, si); }

// ReduceScatter (mpi.hpp:1361-): sbuf holds rc * Size(comm) entries, rbuf rc
template <typename T, Device D>
void ReduceScatter(T const* sbuf, T* rbuf, int rc, Op op, Comm const& comm, SyncInfo<D> const& si) {
    detail::Check(elx_mpi_reduce_scatter(comm.Handle(), detail::TypeCode<T>::value, detail_::DevCode<D>(), op.code,
                                         sbuf, rbuf, rc, detail_::StreamOf(si)));
}
template <typename T, Device D>
void ReduceScatter(T const* sbuf, T* rbuf, int rc, Comm const& comm, SyncInfo<D> const& si) {
    ReduceScatter(sbuf, rbuf, rc, SUM, comm, si);
}

// SendRecv (mpi.hpp:593-633): send sc entries to `to` while receiving rc from `from`
template <typename T, Device D>
void SendRecv(T const* sbuf, int sc, int to, T* rbuf, int rc, int from, Comm const& comm, SyncInfo<D> const& si) {
    detail::Check(elx_mpi_sendrecv(comm.Handle(), detail::TypeCode<T>::value, detail_::DevCode<D>(), sbuf, sc, to,
                                   rbuf, rc, from, detail_::StreamOf(si)));
}
// in place: buf's count entries go to `to` and are replaced by `from`'s (the
// outgoing entries are first copied aside, on the SyncInfo's stream on the GPU)
template <typename T, Device D>
void SendRecv(T* buf, int count, int to, int from, Comm const& comm, SyncInfo<D> const& si) {
    if (count <= 0) return;
    const int dt = detail::TypeCode<T>::value;
    if (D == Device::CPU) {
        std::vector<T> tmp(buf, buf + count);
        SendRecv(static_cast<T const*>(tmp.data()), count, to, buf, count, from, comm, si);
        return;
    }
    void* tmp = nullptr;
    detail::Check(elx_pool_alloc(&tmp, sizeof(T) * count, detail_::StreamOf(si)));
    // a byte copy: any communication type (Int, int, byte as well as the
    // matrix types), stream-ordered before the exchange
    int rc = elx_memcpy_d2d(tmp, buf, sizeof(T) * static_cast<size_t>(count), detail_::StreamOf(si));
    if (rc == ELX_OK)
        rc = elx_mpi_sendrecv(comm.Handle(), dt, ELX_DEVICE_GPU, tmp, count, to, buf, count, from, detail_::StreamOf(si));
    const std::string err = rc == ELX_OK ? std::string() : std::string(elx_last_error());
    (void)elx_pool_free(tmp, detail_::StreamOf(si));
    if (rc != ELX_OK) detail::Check(rc, err);
}
}  // namespace mpi

// ---- El::Grid (src/core/Grid.cpp) --------------------------------------------
class Grid {
public:
    Grid() : Grid(mpi::COMM_WORLD) {}  // Grid.hpp:18 (over COMM_WORLD)
    explicit Grid(const mpi::Comm& comm, int height = 0, GridOrder order = COLUMN_MAJOR)
        : comm_(comm) {
        elx_grid_t g = nullptr;
        detail::Check(elx_grid_create(&g, comm.Handle(), height, order));
        g_.reset(g, [](elx_grid_s* p) { if (p) elx_grid_destroy(p); });
        detail::Check(elx_grid_info(g, info_));
    }
    Grid(const mpi::Comm& comm, GridOrder order) : Grid(comm, 0, order) {}
    static int DefaultHeight(int size) { return elx_grid_default_height(size); }
    int Height() const { return info_[0]; }
    int Width() const { return info_[1]; }
    int Size() const { return info_[2]; }
    int Rank() const { return info_[3]; }
    int MCRank() const { return info_[4]; }
    int MRRank() const { return info_[5]; }
    int VCRank() const { return info_[6]; }
    int VRRank() const { return info_[7]; }
    elx_grid_t Handle() const { return g_.get(); }
private:
    mpi::Comm comm_;
    std::shared_ptr<elx_grid_s> g_;
    int info_[8] = {};
};

// ---- El::Matrix<T,D> (include/El/core/Matrix/decl.hpp:299-540) -------------------
// Column-major local matrix on one device: owns its buffer (host memory, or the
// library's stream-ordered device pool) or views caller storage (Attach /
// LockedAttach, and the local block a DistMatrix hands out through Matrix()).
template <typename T>
class AbstractMatrix {
public:
    virtual ~AbstractMatrix() = default;
    virtual Device GetDevice() const noexcept = 0;
    virtual void Resize(Int height, Int width) = 0;
    Int Height() const noexcept { return h_; }
    Int Width() const noexcept { return w_; }
    Int LDim() const noexcept { return ld_; }
    bool Viewing() const noexcept { return !owned_; }
    bool Locked() const noexcept { return locked_; }
    T* Buffer() {
        if (locked_) throw LogicError("Cannot return non-const buffer of locked Matrix");
        return buf_;
    }
    const T* LockedBuffer() const noexcept { return buf_; }
    T* Buffer(Int i, Int j) { return Buffer() + i + j * ld_; }
    const T* LockedBuffer(Int i, Int j) const noexcept { return buf_ + i + j * ld_; }
    // the HIP stream the matrix's device work is ordered on (null on the CPU);
    // SyncInfoFromMatrix(M).Stream()
    void* Stream() const noexcept { return stream_; }
    // SyncInfoFromMatrix(M) as a GPU SyncInfo (null stream and event on the CPU)
    SyncInfo<Device::GPU> GPUSyncInfo() const noexcept {
        return SyncInfo<Device::GPU>(static_cast<hipStream_t>(stream_), static_cast<hipEvent_t>(event_));
    }

protected:
    T* buf_ = nullptr;
    Int h_ = 0, w_ = 0, ld_ = 1;
    bool owned_ = true, locked_ = false;
    void* stream_ = nullptr;
    void* event_ = nullptr;
};

namespace detail {
// MultiSync over local matrices (Gemm.cpp:178-180 MakeMultiSync(C, A, B)): the
// master's stream waits for the operands' queued work on entry, the operands'
// streams wait for the master's on exit; nothing on the CPU or on one stream.
template <typename T>
class LocalFence {
public:
    LocalFence(const AbstractMatrix<T>& master, std::initializer_list<const AbstractMatrix<T>*> others)
        : gpu_(master.GetDevice() == Device::GPU), m_(master.GPUSyncInfo()) {
        if (!gpu_) return;
        for (const AbstractMatrix<T>* o : others)
            if (o && o->Stream() != master.Stream()) o_.push_back(o->GPUSyncInfo());
        for (const auto& o : o_) {
            if (o.Event()) AddSynchronizationPoint(o, m_);
            else Synchronize(o);  // no event to record (moved-from shell): drain its stream
        }
    }
    // Never throws (a destructor is noexcept): skipped while an exception from
    // the fenced call unwinds (the stream may hold a sticky error) or when the
    // master has no event; a failure to record or wait here is dropped, and the
    // next checked call on the stream reports it.
    ~LocalFence() {
        if (!gpu_ || o_.empty() || !m_.Event() || std::uncaught_exceptions() > uncaught_) return;
        if (elx_event_record(m_.Event(), m_.Stream()) != ELX_OK) return;
        for (const auto& o : o_)
            if (o.Stream() != m_.Stream()) (void)elx_stream_wait_event(o.Stream(), m_.Event());
    }
    LocalFence(const LocalFence&) = delete;
    LocalFence& operator=(const LocalFence&) = delete;

private:
    bool gpu_;
    SyncInfo<Device::GPU> m_;
    std::vector<SyncInfo<Device::GPU>> o_;
    int uncaught_ = std::uncaught_exceptions();
};
}  // namespace detail

template <typename T, Device D = Device::CPU>
class Matrix : public AbstractMatrix<T> {
public:
    Matrix() {
        if (D == Device::GPU) {
            const SyncInfo<Device::GPU>& si = gpu::DefaultSyncInfo();
            this->stream_ = si.Stream();
            this->event_ = si.Event();
        }
    }
    Matrix(Int height, Int width, Int ldim = 0) : Matrix() { Resize(height, width, ldim); }
    Matrix(const Matrix& A) : Matrix() { *this = A; }
    // the moved-from matrix keeps a usable SyncInfo (the default stream and
    // event, as Matrix() gives), so reusing it as an output fences correctly
    Matrix(Matrix&& A) noexcept {
        if (D == Device::GPU) {
            void* s = nullptr;
            void* e = nullptr;
            if (elx_default_stream(&s) == ELX_OK && elx_default_event(&e) == ELX_OK) {
                this->stream_ = s;
                this->event_ = e;
            }
        }
        Swap(A);
    }
    ~Matrix() { Release(); }
    Matrix& operator=(const Matrix& A) {  // deep copy (El::Copy of Matrix)
        if (this == &A) return *this;
        Resize(A.Height(), A.Width());
        detail::LocalFence<T> fence(*this, {&A});
        detail::Check(elx_matrix_copy(detail::TypeCode<T>::value, static_cast<int>(D), A.Height(), A.Width(),
                                      A.LockedBuffer(), A.LDim(), this->buf_, this->ld_, this->stream_));
        return *this;
    }
    Matrix& operator=(Matrix&& A) noexcept { Swap(A); return *this; }
    Device GetDevice() const noexcept override { return D; }

    void Resize(Int height, Int width) override { Resize(height, width, height > 1 ? height : 1); }
    void Resize(Int height, Int width, Int ldim) {
        if (height < 0 || width < 0) throw LogicError("Height and width must be non-negative");
        if (ldim <= 0) ldim = height > 1 ? height : 1;
        if (ldim < height) throw LogicError("Leading dimension must be no less than height");
        if (!this->owned_) {
            if (height != this->h_ || width != this->w_) throw LogicError("Cannot resize this matrix");
            return;
        }
        const std::size_t need = static_cast<std::size_t>(ldim) * static_cast<std::size_t>(width);
        if (need > cap_) {  // grow-only, like Memory::Require (Memory/impl.hpp:254-286)
            Free();
            Allocate(need);
        }
        this->h_ = height;
        this->w_ = width;
        this->ld_ = ldim;
    }
    void Empty() { Release(); this->h_ = this->w_ = 0; this->ld_ = 1; }
    // view caller storage (Matrix::Attach / LockedAttach)
    void Attach(Int height, Int width, T* buffer, Int ldim) { View(height, width, buffer, ldim, false); }
    void LockedAttach(Int height, Int width, const T* buffer, Int ldim) {
        View(height, width, const_cast<T*>(buffer), ldim, true);
    }
    // entry access; on the GPU a synchronizing single-element transfer
    T Get(Int i, Int j) const {
        CheckIndex(i, j);
        T v;
        if (D == Device::GPU)
            detail::Check(elx_memcpy_d2h(&v, this->buf_ + i + j * this->ld_, sizeof(T), this->stream_));
        else
            v = this->buf_[i + j * this->ld_];
        return v;
    }
    void Set(Int i, Int j, T v) {
        CheckIndex(i, j);
        T* p = this->Buffer() + i + j * this->ld_;
        if (D == Device::GPU) detail::Check(elx_memcpy_h2d(p, &v, sizeof(T), this->stream_));
        else *p = v;
    }
    // subsequent device work queues on `stream` (null: the default stream),
    // ordered after the work already queued on the old one
    void SetStream(void* stream) {
        if (D != Device::GPU) return;
        SetSyncInfo(SyncInfo<Device::GPU>(static_cast<hipStream_t>(stream ? stream : gpu::DefaultSyncInfo().Stream()),
                                          nullptr));
    }
    // Matrix<T,Device::GPU>::GetSyncInfo / SetSyncInfo (Matrix/decl.hpp:478-479,
    // impl_gpu.hpp:503-513): Set merges the non-null parts.  A stream change on a
    // matrix that owns pool memory first fences the new stream after the old
    // one, so the buffer's later stream-ordered free (on the new stream) comes
    // after every use; on the local-block view of a DistMatrix (Matrix()) the
    // DistMatrix itself moves to the new stream.
    SyncInfo<D> GetSyncInfo() const noexcept { return SyncInfoOf(this->stream_, this->event_, Tag<D>{}); }
    void SetSyncInfo(SyncInfo<D> const& si) { SetSyncInfoImpl(si); }

    // DistMatrix::Matrix() binds its local view to the owning DistMatrix
    void BindOwner_(elx_dm_t owner) { owner_ = owner; }
    void ViewStream_(void* stream) { if (D == Device::GPU) this->stream_ = stream; }

private:
    template <Device> struct Tag {};
    static SyncInfo<Device::CPU> SyncInfoOf(void*, void*, Tag<Device::CPU>) noexcept { return {}; }
    static SyncInfo<Device::GPU> SyncInfoOf(void* s, void* e, Tag<Device::GPU>) noexcept {
        return SyncInfo<Device::GPU>(static_cast<hipStream_t>(s), static_cast<hipEvent_t>(e));
    }
    void SetSyncInfoImpl(SyncInfo<Device::CPU> const&) {}
    void SetSyncInfoImpl(SyncInfo<Device::GPU> const& si) {
        SyncInfo<Device::GPU> cur = this->GPUSyncInfo();
        const hipStream_t old = cur.Stream();
        cur.Merge(si);
        if (cur.Stream() != old) {
            if (owner_) {
                detail::Check(elx_dm_set_stream(owner_, cur.Stream()));
            } else if (this->owned_ && this->buf_ && old) {
                AddSynchronizationPoint(SyncInfo<Device::GPU>(old, cur.Event()), cur);
            }
        }
        this->stream_ = cur.Stream();
        this->event_ = cur.Event();
    }
    void CheckIndex(Int i, Int j) const {
        if (i < 0 || j < 0 || i >= this->h_ || j >= this->w_) throw LogicError("Entry out of bounds");
    }
    void View(Int height, Int width, T* buffer, Int ldim, bool locked) {
        if (ldim < (height > 1 ? height : 1)) throw LogicError("Leading dimension must be no less than height");
        Release();
        this->buf_ = buffer;
        this->h_ = height;
        this->w_ = width;
        this->ld_ = ldim;
        this->owned_ = false;
        this->locked_ = locked;
    }
    void Allocate(std::size_t elems) {
        void* p = nullptr;
        if (elems) {
            if (D == Device::GPU) {
                detail::Check(elx_pool_alloc(&p, elems * sizeof(T), this->stream_));
            } else {
                p = ::operator new(elems * sizeof(T));
            }
        }
        this->buf_ = static_cast<T*>(p);
        cap_ = elems;
    }
    void Free() {
        if (this->owned_ && this->buf_) {
            if (D == Device::GPU) (void)elx_pool_free(this->buf_, this->stream_);
            else ::operator delete(this->buf_);
        }
        this->buf_ = nullptr;
        cap_ = 0;
    }
    void Release() { Free(); this->owned_ = true; this->locked_ = false; }
    void Swap(Matrix& o) noexcept {
        std::swap(this->buf_, o.buf_); std::swap(this->h_, o.h_); std::swap(this->w_, o.w_);
        std::swap(this->ld_, o.ld_); std::swap(this->owned_, o.owned_); std::swap(this->locked_, o.locked_);
        std::swap(this->stream_, o.stream_); std::swap(this->event_, o.event_); std::swap(cap_, o.cap_);
        std::swap(owner_, o.owner_);
    }
    std::size_t cap_ = 0;
    elx_dm_t owner_ = nullptr;
};

// SyncInfoFromMatrix / SetSyncInfo (Matrix/decl.hpp:287-296,521-533)
template <typename T>
SyncInfo<Device::CPU> SyncInfoFromMatrix(Matrix<T, Device::CPU> const&) {
    return SyncInfo<Device::CPU>{};
}
template <typename T>
SyncInfo<Device::GPU> SyncInfoFromMatrix(Matrix<T, Device::GPU> const& mat) {
    return mat.GetSyncInfo();
}
template <typename T, Device D>
void SetSyncInfo(Matrix<T, D>&, SyncInfo<D> const&) {}
template <typename T>
void SetSyncInfo(Matrix<T, Device::GPU>& mat, SyncInfo<Device::GPU> const& si) {
    mat.SetSyncInfo(si);
}

// ---- DistMatrix ----------------------------------------------------------------
template <typename T>
class AbstractDistMatrix {
public:
    virtual ~AbstractDistMatrix() = default;
    Int Height() const { return Info(0); }
    Int Width() const { return Info(1); }
    Int LocalHeight() const { return Info(2); }
    Int LocalWidth() const { return Info(3); }
    Int LDim() const { return Info(4); }
    int ColAlign() const { return (int)Info(5); }
    int RowAlign() const { return (int)Info(6); }
    int ColShift() const { return (int)Info(7); }
    int RowShift() const { return (int)Info(8); }
    int ColStride() const { return (int)Info(9); }
    int RowStride() const { return (int)Info(10); }
    bool Participating() const { return Info(11) != 0; }
    bool Viewing() const { return Info(12) != 0; }
    Dist ColDist() const { return cd_; }
    Dist RowDist() const { return rd_; }
    Device GetLocalDevice() const { return dev_; }
    const El::Grid& Grid() const { return *grid_; }
    Int GlobalRow(Int iLoc) const { return ColShift() + iLoc * ColStride(); }
    Int GlobalCol(Int jLoc) const { return RowShift() + jLoc * RowStride(); }

    void Resize(Int height, Int width) { detail::Check(elx_dm_resize(h(), height, width)); }
    void Align(int colAlign, int rowAlign, bool constrain = true) {
        detail::Check(elx_dm_align(h(), colAlign, rowAlign, constrain));
    }
    // (any element type: alignment is distribution data, DistData in the reference)
    template <typename S>
    void AlignWith(const AbstractDistMatrix<S>& other, bool constrain = true) {
        detail::Check(elx_dm_align_with(h(), other.h(), constrain));
    }
    // ElementalMatrix::Attach: view caller storage as this rank's local block
    void Attach(Int height, Int width, const El::Grid& /*grid: must be this matrix's*/, int colAlign, int rowAlign,
                T* buffer, Int ldim, int root = 0) {
        detail::Check(elx_dm_attach(h(), height, width, colAlign, rowAlign, buffer, ldim, root));
    }
    T* Buffer() { void* p = nullptr; detail::Check(elx_dm_buffer(h(), &p)); return static_cast<T*>(p); }
    const T* LockedBuffer() const { void* p = nullptr; detail::Check(elx_dm_buffer(h(), &p)); return static_cast<const T*>(p); }
    // host <-> local block (column-major, leading dimension ld)
    void SetLocalBlock(const T* host, Int ld) { detail::Check(elx_dm_set_local(h(), host, ld)); }
    void GetLocalBlock(T* host, Int ld) const { detail::Check(elx_dm_get_local(h(), host, ld)); }
    void Synchronize() const { detail::Check(elx_dm_synchronize(h())); }
    // entry access (ElementMatrix/setup.hpp:463-610): Get is collective over the
    // grid; Set / Update write the copies held by this rank
    T Get(Int i, Int j) const {
        double v = 0;
        detail::Check(elx_dm_get(h(), i, j, &v));
        return detail::FromDouble<T>(v);
    }
    void Set(Int i, Int j, T value) { detail::Check(elx_dm_set(h(), i, j, detail::ToDouble(value))); }
    void Update(Int i, Int j, T value) { detail::Check(elx_dm_update(h(), i, j, detail::ToDouble(value))); }
    // SetSyncInfo(mat, si) / SyncInfoFromMatrix(mat): the matrix's HIP stream
    void SetStream(void* stream) { detail::Check(elx_dm_set_stream(h(), stream)); }
    void* Stream() const { void* s = nullptr; detail::Check(elx_dm_stream(h(), &s)); return s; }
    elx_dm_t h() const { return dm_.get(); }

protected:
    AbstractDistMatrix(const El::Grid& g, Dist cd, Dist rd, Device dev, int root)
        : grid_(&g), cd_(cd), rd_(rd), dev_(dev) {
        elx_dm_t m = nullptr;
        detail::Check(elx_dm_create(&m, g.Handle(), detail::TypeCode<T>::value, cd, rd,
                                    static_cast<int>(dev), root));
        dm_.reset(m, [](elx_dm_s* p) { if (p) elx_dm_destroy(p); });
    }
    AbstractDistMatrix(const El::Grid& g, Dist cd, Dist rd, Device dev, elx_dm_t view)
        : grid_(&g), cd_(cd), rd_(rd), dev_(dev), dm_(view, [](elx_dm_s* p) { if (p) elx_dm_destroy(p); }) {}
    Int Info(int i) const {
        Int v[13];
        detail::Check(elx_dm_info(h(), v));
        return v[i];
    }
    const El::Grid* grid_;
    Dist cd_, rd_;
    Device dev_;
    std::shared_ptr<elx_dm_s> dm_;
};

template <typename T, Dist U = MC, Dist V = MR, DistWrap W = ELEMENT, Device D = Device::CPU>
class DistMatrix : public AbstractDistMatrix<T> {
    static_assert(W == ELEMENT, "BLOCK distributions are outside the El::Gemm path");
public:
    explicit DistMatrix(const El::Grid& g, int root = 0) : AbstractDistMatrix<T>(g, U, V, D, root) {}
    DistMatrix(Int height, Int width, const El::Grid& g, int root = 0) : DistMatrix(g, root) {
        this->Resize(height, width);
    }
    // cross-distribution / cross-device copy construction (DistMatrix(const DistMatrix<T,U2,V2,...>&))
    template <Dist U2, Dist V2, Device D2>
    explicit DistMatrix(const DistMatrix<T, U2, V2, ELEMENT, D2>& A) : DistMatrix(A.Grid()) { *this = A; }
    DistMatrix(const DistMatrix& A) : DistMatrix(A.Grid()) { *this = A; }
    DistMatrix& operator=(const DistMatrix& A) {
        if (this != &A) detail::Check(elx_dm_copy(this->h(), A.h()));
        return *this;
    }
    // operator= : the redistribution table (bit-exact)
    DistMatrix& operator=(const AbstractDistMatrix<T>& A) {
        detail::Check(elx_dm_copy(this->h(), A.h()));
        return *this;
    }
    // the local block as an El::Matrix<T,D> view (ElementalMatrix::Matrix() /
    // LockedMatrix(), include/El/core/DistMatrix/Element.hpp): buffer, local
    // sizes, ldim and the matrix's stream, refreshed on every call
    El::Matrix<T, D>& Matrix() { RefreshLocal(); return local_; }
    const El::Matrix<T, D>& LockedMatrix() const { RefreshLocal(); return local_; }
    // A(IR(i0,i1), IR(j0,j1)) views
    DistMatrix operator()(Range rows, Range cols) const { return View(rows.beg, rows.end, cols.beg, cols.end); }
    DistMatrix operator()(AllRange, Range cols) const { return View(0, this->Height(), cols.beg, cols.end); }
    DistMatrix operator()(Range rows, AllRange) const { return View(rows.beg, rows.end, 0, this->Width()); }

private:
    // the view keeps its event; its stream is the DistMatrix's, and
    // SetSyncInfo on it moves the DistMatrix (SyncInfoFromMatrix(A.LockedMatrix())
    // / SetSyncInfo(A.Matrix(), si), the reference callers' idiom)
    void RefreshLocal() const {
        const Int ld = this->LDim() > 1 ? this->LDim() : 1;
        local_.Attach(this->LocalHeight(), this->LocalWidth(), const_cast<T*>(this->LockedBuffer()), ld);
        local_.ViewStream_(this->Stream());
        local_.BindOwner_(this->h());
    }
    mutable El::Matrix<T, D> local_;
    DistMatrix(const El::Grid& g, elx_dm_t view) : AbstractDistMatrix<T>(g, U, V, D, view) {}
    DistMatrix View(Int i0, Int i1, Int j0, Int j1) const {
        elx_dm_t v = nullptr;
        detail::Check(elx_dm_view(&v, this->h(), i0, i1, j0, j1));
        return DistMatrix(this->Grid(), v);
    }
};

// ---- level 3 (include/El/blas_like/level3.hpp:37-90) ----------------------------
// Gemm on local matrices (level3.hpp:37-65, Gemm.cpp:141-250): the MFMA kernels on
// the GPU (on C's stream), the library's host loops on the CPU
template <typename T>
void Gemm(Orientation orientA, Orientation orientB, T alpha, const AbstractMatrix<T>& A, const AbstractMatrix<T>& B,
          T beta, AbstractMatrix<T>& C) {
    if (A.GetDevice() != C.GetDevice() || B.GetDevice() != C.GetDevice())
        throw LogicError("Gemm: A, B and C must be on the same device");
    const Int m = orientA == NORMAL ? A.Height() : A.Width(), k = orientA == NORMAL ? A.Width() : A.Height();
    const Int kb = orientB == NORMAL ? B.Height() : B.Width(), n = orientB == NORMAL ? B.Width() : B.Height();
    if (m != C.Height() || n != C.Width() || k != kb) throw LogicError("Nonconformal Gemm");
    detail::LocalFence<T> fence(C, {&A, &B});
    detail::Check(elx_matrix_gemm(detail::TypeCode<T>::value, static_cast<int>(C.GetDevice()), orientA, orientB, m, n,
                                  k, detail::ToDouble(alpha), A.LockedBuffer(), A.LDim(), B.LockedBuffer(), B.LDim(),
                                  detail::ToDouble(beta), C.Buffer(), C.LDim(), C.Stream()));
}
// beta-less form: C resized to op(A) op(B) and overwritten
template <typename T>
void Gemm(Orientation orientA, Orientation orientB, T alpha, const AbstractMatrix<T>& A, const AbstractMatrix<T>& B,
          AbstractMatrix<T>& C) {
    C.Resize(orientA == NORMAL ? A.Height() : A.Width(), orientB == NORMAL ? B.Width() : B.Height());
    Gemm(orientA, orientB, alpha, A, B, detail::FromDouble<T>(0.0), C);
}
template <typename T, Device D>
void Gemm(Orientation orientA, Orientation orientB, T alpha, const Matrix<T, D>& A, const Matrix<T, D>& B, T beta,
          Matrix<T, D>& C) {
    Gemm(orientA, orientB, alpha, static_cast<const AbstractMatrix<T>&>(A), static_cast<const AbstractMatrix<T>&>(B),
         beta, static_cast<AbstractMatrix<T>&>(C));
}
template <typename T, Device D>
void Gemm(Orientation orientA, Orientation orientB, T alpha, const Matrix<T, D>& A, const Matrix<T, D>& B,
          Matrix<T, D>& C) {
    Gemm(orientA, orientB, alpha, static_cast<const AbstractMatrix<T>&>(A), static_cast<const AbstractMatrix<T>&>(B),
         static_cast<AbstractMatrix<T>&>(C));
}
template <typename T>
void Gemm(Orientation orientA, Orientation orientB, T alpha, const AbstractDistMatrix<T>& A,
          const AbstractDistMatrix<T>& B, T beta, AbstractDistMatrix<T>& C, GemmAlgorithm alg = GEMM_DEFAULT) {
    detail::Check(elx_gemm(orientA, orientB, detail::ToDouble(alpha), A.h(), B.h(), detail::ToDouble(beta), C.h(), alg));
}
// beta-less form: C is resized to op(A) op(B) and overwritten (Gemm.cpp:304-316)
template <typename T>
void Gemm(Orientation orientA, Orientation orientB, T alpha, const AbstractDistMatrix<T>& A,
          const AbstractDistMatrix<T>& B, AbstractDistMatrix<T>& C, GemmAlgorithm alg = GEMM_DEFAULT) {
    const Int m = orientA == NORMAL ? A.Height() : A.Width();
    const Int n = orientB == NORMAL ? B.Width() : B.Height();
    C.Resize(m, n);
    detail::Check(elx_gemm(orientA, orientB, detail::ToDouble(alpha), A.h(), B.h(), 0.0, C.h(), alg));
}
template <typename T>
void LocalGemm(Orientation orientA, Orientation orientB, T alpha, const AbstractDistMatrix<T>& A,
               const AbstractDistMatrix<T>& B, T beta, AbstractDistMatrix<T>& C) {
    detail::Check(elx_local_gemm(orientA, orientB, detail::ToDouble(alpha), A.h(), B.h(), detail::ToDouble(beta), C.h()));
}
// Syrk / Herk (src/blas_like/level3/Syrk.cpp:196-225): C's uplo triangle only
template <typename T>
void Syrk(UpperOrLower uplo, Orientation orientation, T alpha, const AbstractDistMatrix<T>& A, T beta,
          AbstractDistMatrix<T>& C, bool conjugate = false) {
    detail::Check(elx_syrk(uplo, orientation, detail::ToDouble(alpha), A.h(), detail::ToDouble(beta), C.h(), conjugate));
}
// beta-less form: C resized to n x n and zeroed first (Syrk.cpp:213-225)
template <typename T>
void Syrk(UpperOrLower uplo, Orientation orientation, T alpha, const AbstractDistMatrix<T>& A,
          AbstractDistMatrix<T>& C, bool conjugate = false) {
    const Int n = orientation == NORMAL ? A.Height() : A.Width();
    C.Resize(n, n);
    detail::Check(elx_dm_zero(C.h()));
    detail::Check(elx_syrk(uplo, orientation, detail::ToDouble(alpha), A.h(), 0.0, C.h(), conjugate));
}
template <typename T>
void Herk(UpperOrLower uplo, Orientation orientation, T alpha, const AbstractDistMatrix<T>& A, T beta,
          AbstractDistMatrix<T>& C) {
    Syrk(uplo, orientation, alpha, A, beta, C, true);
}
template <typename T>
void Trrk(UpperOrLower uplo, Orientation orientA, Orientation orientB, T alpha, const AbstractDistMatrix<T>& A,
          const AbstractDistMatrix<T>& B, T beta, AbstractDistMatrix<T>& C) {
    detail::Check(elx_trrk(uplo, orientA, orientB, detail::ToDouble(alpha), A.h(), B.h(), detail::ToDouble(beta), C.h()));
}
template <typename T>
void Syr2k(UpperOrLower uplo, Orientation orientation, T alpha, const AbstractDistMatrix<T>& A,
           const AbstractDistMatrix<T>& B, T beta, AbstractDistMatrix<T>& C, bool conjugate = false) {
    detail::Check(elx_syr2k(uplo, orientation, detail::ToDouble(alpha), A.h(), B.h(), detail::ToDouble(beta), C.h(),
                            conjugate));
}
template <typename T>
void Her2k(UpperOrLower uplo, Orientation orientation, T alpha, const AbstractDistMatrix<T>& A,
           const AbstractDistMatrix<T>& B, T beta, AbstractDistMatrix<T>& C) {
    Syr2k(uplo, orientation, alpha, A, B, beta, C, true);
}
// checkIfSingular: SingularMatrixException on an exact zero NON_UNIT diagonal (Trsm.cpp:60-68)
template <typename T>
void Trsm(LeftOrRight side, UpperOrLower uplo, Orientation orientation, UnitOrNonUnit diag, T alpha,
          const AbstractDistMatrix<T>& A, AbstractDistMatrix<T>& B, bool checkIfSingular = false) {
    detail::Check(elx_trsm(side, uplo, orientation, diag, detail::ToDouble(alpha), A.h(), B.h(),
                           checkIfSingular ? 1 : 0));
}
template <typename T>
void Symm(LeftOrRight side, UpperOrLower uplo, T alpha, const AbstractDistMatrix<T>& A, const AbstractDistMatrix<T>& B,
          T beta, AbstractDistMatrix<T>& C, bool conjugate = false) {
    detail::Check(elx_symm(side, uplo, detail::ToDouble(alpha), A.h(), B.h(), detail::ToDouble(beta), C.h(), conjugate));
}
template <typename T>
void Hemm(LeftOrRight side, UpperOrLower uplo, T alpha, const AbstractDistMatrix<T>& A, const AbstractDistMatrix<T>& B,
          T beta, AbstractDistMatrix<T>& C) {
    Symm(side, uplo, alpha, A, B, beta, C, true);
}
template <typename T>
void ScaleTrapezoid(T alpha, UpperOrLower uplo, AbstractDistMatrix<T>& A, Int offset = 0) {
    detail::Check(elx_dm_scale_trapezoid(detail::ToDouble(alpha), uplo, A.h(), offset));
}

// ---- level 1 front doors ------------------------------------------------------------
template <typename T> void Copy(const AbstractDistMatrix<T>& A, AbstractDistMatrix<T>& B) { detail::Check(elx_dm_copy(B.h(), A.h())); }
// S != T: redistribute in S, convert locally (CopyDistMatrix.hpp:28-57)
template <typename S, typename T> void Copy(const AbstractDistMatrix<S>& A, AbstractDistMatrix<T>& B) { detail::Check(elx_dm_copy(B.h(), A.h())); }
template <typename T> void Transpose(const AbstractDistMatrix<T>& A, AbstractDistMatrix<T>& B, bool /*conjugate*/ = false) {
    detail::Check(elx_dm_transpose(A.h(), B.h()));
}
template <typename T, typename S> void Axpy(S alpha, const AbstractDistMatrix<T>& X, AbstractDistMatrix<T>& Y) {
    detail::Check(elx_dm_axpy(static_cast<double>(alpha), X.h(), Y.h()));
}
template <typename T, typename S> void Scale(S alpha, AbstractDistMatrix<T>& A) {
    detail::Check(elx_dm_scale(static_cast<double>(alpha), A.h()));
}
template <typename T> void Zero(AbstractDistMatrix<T>& A) { detail::Check(elx_dm_zero(A.h())); }
// El::Fill (include/El/blas_like/level1/Fill.hpp:20-70)
template <typename T> void Fill(AbstractDistMatrix<T>& A, T alpha) {
    detail::Check(elx_dm_fill(A.h(), detail::ToDouble(alpha)));
}
// level-1 on local matrices (Fill / Zero / Scale / Axpy / Copy of AbstractMatrix)
template <typename T> void Fill(AbstractMatrix<T>& A, T alpha) {
    detail::Check(elx_matrix_fill(detail::TypeCode<T>::value, static_cast<int>(A.GetDevice()), A.Height(), A.Width(),
                                  detail::ToDouble(alpha), A.Buffer(), A.LDim(), A.Stream()));
}
template <typename T> void Zero(AbstractMatrix<T>& A) { Fill(A, detail::FromDouble<T>(0.0)); }
template <typename T, typename S> void Scale(S alpha, AbstractMatrix<T>& A) {
    detail::Check(elx_matrix_scale(detail::TypeCode<T>::value, static_cast<int>(A.GetDevice()), A.Height(), A.Width(),
                                   static_cast<double>(alpha), A.Buffer(), A.LDim(), A.Stream()));
}
template <typename T, typename S> void Axpy(S alpha, const AbstractMatrix<T>& X, AbstractMatrix<T>& Y) {
    if (X.GetDevice() != Y.GetDevice()) throw LogicError("Axpy: X and Y must be on the same device");
    if (X.Height() != Y.Height() || X.Width() != Y.Width()) throw LogicError("Nonconformal Axpy");
    detail::LocalFence<T> fence(Y, {&X});
    detail::Check(elx_matrix_axpy(detail::TypeCode<T>::value, static_cast<int>(Y.GetDevice()), Y.Height(), Y.Width(),
                                  static_cast<double>(alpha), X.LockedBuffer(), X.LDim(), Y.Buffer(), Y.LDim(),
                                  Y.Stream()));
}
template <typename T> void Copy(const AbstractMatrix<T>& A, AbstractMatrix<T>& B) {
    if (A.GetDevice() != B.GetDevice()) throw LogicError("Copy: cross-device Matrix copies go through DistMatrix");
    B.Resize(A.Height(), A.Width());
    detail::LocalFence<T> fence(B, {&A});
    detail::Check(elx_matrix_copy(detail::TypeCode<T>::value, static_cast<int>(B.GetDevice()), A.Height(), A.Width(),
                                  A.LockedBuffer(), A.LDim(), B.Buffer(), B.LDim(), B.Stream()));
}
template <typename T> void Hadamard(const AbstractDistMatrix<T>& A, const AbstractDistMatrix<T>& B, AbstractDistMatrix<T>& C) {
    detail::Check(elx_dm_hadamard(A.h(), B.h(), C.h()));
}
enum class EntrywiseFn { IDENTITY = ELX_MAP_IDENTITY, NEGATE = ELX_MAP_NEGATE, ABS = ELX_MAP_ABS, SQUARE = ELX_MAP_SQUARE,
                         SQRT = ELX_MAP_SQRT, EXP = ELX_MAP_EXP, LOG = ELX_MAP_LOG, RELU = ELX_MAP_RELU,
                         SIGMOID = ELX_MAP_SIGMOID, RECIPROCAL = ELX_MAP_RECIP, TANH = ELX_MAP_TANH };
enum class CombineFn { ADD = ELX_COMBINE_ADD, SUB = ELX_COMBINE_SUB, MUL = ELX_COMBINE_MUL, DIV = ELX_COMBINE_DIV,
                       MAX = ELX_COMBINE_MAX, MIN = ELX_COMBINE_MIN, RELU_GRAD = ELX_COMBINE_RELU_GRAD };
// B := f(A, B) (EntrywiseMap.hpp:187-202; the device functor is one of CombineFn)
template <typename T> void Combine(const AbstractDistMatrix<T>& A, AbstractDistMatrix<T>& B, CombineFn f) {
    detail::Check(elx_dm_combine(static_cast<int>(f), A.h(), B.h()));
}
template <typename T> void EntrywiseMap(const AbstractDistMatrix<T>& A, AbstractDistMatrix<T>& B, EntrywiseFn f) {
    detail::Check(elx_dm_entrywise_map(static_cast<int>(f), A.h(), B.h()));
}
template <typename T, typename S> void AxpyContract(S alpha, const AbstractDistMatrix<T>& A, AbstractDistMatrix<T>& B) {
    detail::Check(elx_dm_axpy_contract(static_cast<double>(alpha), A.h(), B.h()));
}
// El::FrobeniusNorm on DistMatrices (collective; Base<T> is T for the real types)
template <typename T> double FrobeniusNorm(const AbstractDistMatrix<T>& A) {
    double v = 0.0;
    detail::Check(elx_dm_frobenius_norm(A.h(), &v));
    return v;
}
// grid-independent synthetic fill (stands in for Uniform(A, m, n, center, radius) in benchmarks)
// El::InitializeRandom (random.cpp:24-35); Initialize() seeds deterministically
inline void InitializeRandom(bool deterministic = true, int worldRank = 0) {
    detail::Check(elx_initialize_random(deterministic ? 1 : 0, worldRank));
}
// El::Uniform / MakeUniform (Uniform.cpp:18-66): the reference's draws bit for bit
template <typename T> void MakeUniform(AbstractDistMatrix<T>& A, T center = T(0), double radius = 1.0) {
    detail::Check(elx_dm_make_uniform(A.h(), detail::ToDouble(center), radius));
}
template <typename T> void Uniform(AbstractDistMatrix<T>& A, Int m, Int n, T center = T(0), double radius = 1.0) {
    detail::Check(elx_dm_uniform(A.h(), m, n, detail::ToDouble(center), radius));
}
template <typename T> void HashFill(AbstractDistMatrix<T>& A, std::uint64_t seed, double center, double radius) {
    detail::Check(elx_dm_fill_hash(A.h(), seed, center, radius));
}

// El::Write / El::Read (src/io/Write.cpp:70-86, src/io/Read.cpp:71-120); the file's
// Int fields are sizeof(El::Int) of the producing build (4 by default)
template <typename T>
void Write(const AbstractDistMatrix<T>& A, const std::string& basename = "matrix", FileFormat format = BINARY,
           int intBytes = 4) {
    detail::Check(elx_dm_write(A.h(), basename.c_str(), static_cast<int>(format), intBytes));
}
template <typename T>
void Read(AbstractDistMatrix<T>& A, const std::string& filename, FileFormat format = AUTO, int intBytes = 4) {
    detail::Check(elx_dm_read(A.h(), filename.c_str(), static_cast<int>(format), intBytes));
}

// ---- environment ------------------------------------------------------------------
// the algorithmic blocksize stack (include/El/core/environment/decl.hpp:88-94,
// src/blas_like/blocksizes.cpp:38-72); an empty stack is a LogicError
inline Int Blocksize() {
    const Int nb = elx_blocksize();
    if (nb < 0) throw LogicError(elx_last_error());
    return nb;
}
inline void SetBlocksize(Int nb) { detail::Check(elx_set_blocksize(nb)); }
inline void PushBlocksizeStack(Int nb) { detail::Check(elx_push_blocksize(nb)); }
inline void PopBlocksizeStack() { detail::Check(elx_pop_blocksize()); }
inline void EmptyBlocksizeStack() { detail::Check(elx_empty_blocksize_stack()); }
// El::Initialize (src/core/environment.cpp:215-330): the world communicator
// from the launcher's environment (RANK / WORLD_SIZE / LOCAL_RANK /
// MASTER_ADDR: RCCL, one process per GPU; size 1 without them), blocksize
// stack {128}, deterministic RNG.  Finalize drops the world and the stack.
inline void Initialize() { detail::Check(elx_initialize()); }
inline void Initialize(int&, char**&) { Initialize(); }
inline void Finalize() { detail::Check(elx_finalize()); }
inline bool Initialized() { return true; }

}  // namespace El

// functor-generic EntrywiseMap / Combine on GPU matrices: device templates,
// available when the caller compiles with hipcc (EntrywiseMap.hpp:141-203)
#if defined(__HIPCC__)
#include "El/EntrywiseMap.hip.hpp"
#endif
