#include "comm.hpp"
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

namespace elx {

CommStats& GlobalCommStats() {
    static CommStats s;
    return s;
}

CommProfiler& CommProf() {
    static CommProfiler p;
    return p;
}

void CommProfiler::Clear() {
    for (auto& r : recs) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    recs.clear();
}

CommProfiler::Rec CommProfiler::Begin(hipStream_t s) {
    Rec r;
    if (!on || !s) return r;
    ELX_CHECK_HIP(hipEventCreate(&r.a));
    ELX_CHECK_HIP(hipEventCreate(&r.b));
    ELX_CHECK_HIP(hipEventRecord(r.a, s));
    return r;
}

void CommProfiler::End(Rec r, hipStream_t s, int64_t bytes) {
    if (!r.a) return;
    ELX_CHECK_HIP(hipEventRecord(r.b, s));
    r.bytes = bytes;
    recs.push_back(r);
}

void CommProfiler::Stats(double& ms, int64_t& bytes, int64_t& calls) {
    ms = 0;
    bytes = calls = 0;
    for (auto& r : recs) {
        ELX_CHECK_HIP(hipEventSynchronize(r.b));
        float t = 0;
        ELX_CHECK_HIP(hipEventElapsedTime(&t, r.a, r.b));
        ms += t;
        bytes += r.bytes;
        ++calls;
    }
}

namespace {

double Now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Watchdog {
    std::mutex mu;
    std::string stage = "init";
    double deadline = 0;  // steady-clock seconds; 0 = no deadline
    double budget = 0;
    std::vector<ncclComm_t> comms;
    bool started = false;
    // written to stdout before exiting (e.g. a result line already measured);
    // to file descriptor ELX_WATCHDOG_FD instead when that is set (a caller that
    // moved descriptor 1 to stderr keeps its result line on a duplicate)
    std::string epitaph;
    int epitaph_code = kWatchdogExit;

    [[noreturn]] void Fail(const std::string& why) {
        const int code = epitaph_code;
        std::fprintf(stderr, "[elx watchdog] FATAL in stage '%s': %s; aborting %zu RCCL communicator(s), exit %d\n",
                     stage.c_str(), why.c_str(), comms.size(), code);
        std::fflush(stderr);
        for (ncclComm_t c : comms) (void)ncclCommAbort(c);
        const char* fdv = std::getenv("ELX_WATCHDOG_FD");
        if (!epitaph.empty()) {
            if (fdv && *fdv) ::dprintf(std::atoi(fdv), "%s\n", epitaph.c_str());
            else std::fprintf(stdout, "%s\n", epitaph.c_str());
        }
        std::fflush(stdout);
        _exit(code);
    }
    void Loop() {
        for (;;) {
            std::this_thread::sleep_for(std::chrono::milliseconds(50));
            std::lock_guard<std::mutex> lk(mu);
            for (ncclComm_t c : comms) {
                ncclResult_t e = ncclSuccess;
                if (ncclCommGetAsyncError(c, &e) == ncclSuccess && e != ncclSuccess && e != ncclInProgress)
                    Fail(Cat("RCCL asynchronous error: ", ncclGetErrorString(e)));
            }
            if (deadline > 0 && Now() > deadline) Fail(Cat("deadline of ", budget, " s exceeded"));
        }
    }
};
Watchdog& WD() {
    static Watchdog* w = new Watchdog();  // never destroyed: the thread may outlive static teardown
    return *w;
}

// Blocking communicators by default; ELX_RCCL_NONBLOCKING=1 creates them with
// ncclConfig_t.blocking = 0 (every init, split and group end that returns
// ncclInProgress is then polled by CheckNccl).  Either way a peer that never
// arrives is caught by the watchdog's stage deadline (ncclCommAbort from the
// watchdog thread, then exit), not by waiting forever.  Not the default: on
// RCCL 2.26.6 (torch's librccl) a nonblocking world's ncclCommSplit handed back
// a child that ncclCommUserRank rejected (invalid argument) at world size 1
// (profiles/r03b_gputests_summary.log).
bool NonBlocking() {
    static const bool nb = [] {
        const char* e = std::getenv("ELX_RCCL_NONBLOCKING");
        return e && std::atoi(e) != 0;
    }();
    return nb;
}
ncclConfig_t CommConfig() {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = NonBlocking() ? 0 : 1;
    return cfg;
}

ncclDataType_t NcclType(DType t) {
    switch (t) {
    case DType::F32: return ncclFloat32;
    case DType::F64: return ncclFloat64;
    case DType::F16: return ncclFloat16;
    case DType::BF16: return ncclBfloat16;
    case DType::I32: return ncclInt32;
    case DType::I64: return ncclInt64;
    case DType::U8: return ncclUint8;
    }
    throw LogicError("bad dtype");
}

void CheckNccl(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw CommError(Cat("RCCL ", what, " failed: ", ncclGetErrorString(r)));
}
// result of a call on a (possibly nonblocking) communicator: wait out ncclInProgress
void CheckNccl(ncclResult_t r, const char* what, ncclComm_t c) {
    while (r == ncclInProgress) {
        std::this_thread::yield();
        if (ncclCommGetAsyncError(c, &r) != ncclSuccess) break;
    }
    CheckNccl(r, what);
}

void CopyBytes(Device dev, void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0 || dst == src) return;
    if (dev == Device::GPU) ELX_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    else std::memcpy(dst, src, bytes);
}

// Pinned staging buffer for host-backend collectives on device data.
struct Staging {
    void* p = nullptr;
    size_t cap = 0;
    void* Get(size_t bytes) {
        if (bytes > cap) {
            if (p) (void)hipHostFree(p);
            ELX_CHECK_HIP(hipHostMalloc(&p, bytes, hipHostMallocDefault));
            cap = bytes;
        }
        return p;
    }
};

}  // namespace

std::shared_ptr<Comm> Comm::Self() {
    auto c = std::shared_ptr<Comm>(new Comm());
    c->kind_ = Kind::SELF;
    return c;
}

std::shared_ptr<Comm> Comm::InitRCCL(int rank, int size, const unsigned char id[128]) {
    Runtime::Get().EnsureGPU();
    ncclUniqueId uid;
    static_assert(sizeof(uid.internal) == 128, "ncclUniqueId size");
    std::memcpy(uid.internal, id, 128);
    auto c = std::shared_ptr<Comm>(new Comm());
    c->kind_ = Kind::RCCL;
    c->rank_ = rank;
    c->size_ = size;
    ncclConfig_t cfg = CommConfig();
    ncclComm_t nc = nullptr;
    const ncclResult_t r = ncclCommInitRankConfig(&nc, size, uid, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) CheckNccl(r, "ncclCommInitRankConfig");
    c->nccl_ = nc;
    WatchdogRegister(nc);
    CheckNccl(r, "ncclCommInitRankConfig", nc);
    return c;
}

std::shared_ptr<Comm> Comm::WrapRCCL(ncclComm_t nc) {
    ELX_REQUIRE(nc != nullptr, "null RCCL communicator");
    Runtime::Get().EnsureGPU();
    auto c = std::shared_ptr<Comm>(new Comm());
    c->kind_ = Kind::RCCL;
    c->nccl_ = nc;
    c->owned_ = false;
    CheckNccl(ncclCommUserRank(nc, &c->rank_), "ncclCommUserRank");
    CheckNccl(ncclCommCount(nc, &c->size_), "ncclCommCount");
    return c;
}

std::shared_ptr<Comm> Comm::InitHost(int rank, int size, elx_host_coll_fn coll, elx_host_split_fn split, void* ctx) {
    ELX_REQUIRE(coll != nullptr, "host comm needs a collective callback");
    ELX_REQUIRE(rank >= 0 && rank < size, "bad rank ", rank, " of ", size);
    auto c = std::shared_ptr<Comm>(new Comm());
    c->kind_ = Kind::HOST;
    c->rank_ = rank;
    c->size_ = size;
    c->coll_ = coll;
    c->split_ = split;
    c->ctx_ = ctx;
    c->group_ = 0;
    return c;
}

Comm::~Comm() {
    if (nccl_ && owned_) {
        WatchdogUnregister(nccl_);
        ncclResult_t r = ncclCommFinalize(nccl_);
        while (r == ncclInProgress && ncclCommGetAsyncError(nccl_, &r) == ncclSuccess) std::this_thread::yield();
        (void)ncclCommDestroy(nccl_);
    }
}

std::shared_ptr<Comm> Comm::Split(int color, int key) {
    if (kind_ == Kind::SELF) return Self();
    auto c = std::shared_ptr<Comm>(new Comm());
    c->kind_ = kind_;
    if (kind_ == Kind::RCCL) {
        ncclConfig_t cfg = CommConfig();
        const ncclResult_t r = ncclCommSplit(nccl_, color, key, &c->nccl_, &cfg);
        if (r != ncclSuccess && r != ncclInProgress) CheckNccl(r, "ncclCommSplit");
        CheckNccl(r, "ncclCommSplit", nccl_);
        if (c->nccl_) {
            WatchdogRegister(c->nccl_);
            ncclResult_t st = ncclInProgress;
            CheckNccl(st, "ncclCommSplit (child)", c->nccl_);
        }
        CheckNccl(ncclCommUserRank(c->nccl_, &c->rank_), "ncclCommUserRank");
        CheckNccl(ncclCommCount(c->nccl_, &c->size_), "ncclCommCount");
        return c;
    }
    ELX_REQUIRE(split_ != nullptr, "host comm has no split callback");
    ELX_REQUIRE(group_ == 0, "host comm: only the world communicator can be split");
    int g = 0, r = 0, sz = 1;
    if (split_(ctx_, group_, color, key, &g, &r, &sz) != 0) throw CommError("host split callback failed");
    c->coll_ = coll_;
    c->split_ = split_;
    c->ctx_ = ctx_;
    c->group_ = g;
    c->rank_ = r;
    c->size_ = sz;
    return c;
}

void Comm::HostCall(int op, DType t, const void* send, void* recv, Int count, int peer, int peer2) {
    auto t0 = std::chrono::steady_clock::now();
    const int rc = coll_(ctx_, op, group_, static_cast<int>(t), send, recv, count, peer, peer2);
    GlobalCommStats().seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc != 0) throw CommError(Cat("host collective op ", op, " failed with ", rc));
}

void Comm::AllGather(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s) {
    const size_t es = DTypeSize(t), bytes = static_cast<size_t>(count) * es;
    auto& st = GlobalCommStats();
    st.calls++;
    st.bytes += static_cast<int64_t>(bytes) * (size_ - 1);
    if (size_ == 1) { CopyBytes(dev, recv, send, bytes, s); return; }
    if (count == 0) return;
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        CheckNccl(ncclAllGather(send, recv, count, NcclType(t), nccl_, s), "ncclAllGather", nccl_);
        return;
    }
    if (dev == Device::CPU) { HostCall(ELX_COLL_ALLGATHER, t, send, recv, count, 0, 0); return; }
    static Staging stg;
    char* h = static_cast<char*>(stg.Get(bytes * (size_ + 1)));
    ELX_CHECK_HIP(hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
    HostCall(ELX_COLL_ALLGATHER, t, h, h + bytes, count, 0, 0);
    ELX_CHECK_HIP(hipMemcpyAsync(recv, h + bytes, bytes * size_, hipMemcpyHostToDevice, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
}

namespace {
ncclRedOp_t NcclOp(ReduceOp op) {
    switch (op) {
    case ReduceOp::SUM: return ncclSum;
    case ReduceOp::PROD: return ncclProd;
    case ReduceOp::MAX: return ncclMax;
    case ReduceOp::MIN: return ncclMin;
    }
    throw LogicError("unknown reduction op");
}
}  // namespace

void Comm::ReduceScatter(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s, ReduceOp op) {
    const size_t es = DTypeSize(t), bytes = static_cast<size_t>(count) * es;
    auto& st = GlobalCommStats();
    st.calls++;
    st.bytes += static_cast<int64_t>(bytes) * (size_ - 1);
    if (size_ == 1) { CopyBytes(dev, recv, send, bytes, s); return; }
    if (count == 0) return;
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        CheckNccl(ncclReduceScatter(send, recv, count, NcclType(t), NcclOp(op), nccl_, s), "ncclReduceScatter", nccl_);
        return;
    }
    if (op != ReduceOp::SUM || !(t == DType::F32 || t == DType::F64)) {
        HostFold(true, t, op, send, recv, count, dev, s);
        return;
    }
    if (dev == Device::CPU) { HostCall(ELX_COLL_REDUCE_SCATTER, t, send, recv, count, 0, 0); return; }
    static Staging stg;
    char* h = static_cast<char*>(stg.Get(bytes * (size_ + 1)));
    ELX_CHECK_HIP(hipMemcpyAsync(h, send, bytes * size_, hipMemcpyDeviceToHost, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
    HostCall(ELX_COLL_REDUCE_SCATTER, t, h, h + bytes * size_, count, 0, 0);
    ELX_CHECK_HIP(hipMemcpyAsync(recv, h + bytes * size_, bytes, hipMemcpyHostToDevice, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
}

void Comm::AllReduce(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s, ReduceOp op) {
    const size_t bytes = static_cast<size_t>(count) * DTypeSize(t);
    if (size_ == 1) { CopyBytes(dev, recv, send, bytes, s); return; }
    if (count == 0) return;
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        CheckNccl(ncclAllReduce(send, recv, count, NcclType(t), NcclOp(op), nccl_, s), "ncclAllReduce", nccl_);
        return;
    }
    if (op != ReduceOp::SUM || !(t == DType::F32 || t == DType::F64)) {
        HostFold(false, t, op, send, recv, count, dev, s);
        return;
    }
    if (dev == Device::CPU) { HostCall(ELX_COLL_ALLREDUCE, t, send, recv, count, 0, 0); return; }
    static Staging stg;
    char* h = static_cast<char*>(stg.Get(bytes * 2));
    ELX_CHECK_HIP(hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
    HostCall(ELX_COLL_ALLREDUCE, t, h, h + bytes, count, 0, 0);
    ELX_CHECK_HIP(hipMemcpyAsync(recv, h + bytes, bytes, hipMemcpyHostToDevice, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
}

// Every rank gathers the contributions it reduces (ALLTOALL of its slice for
// a reduce-scatter, ALLGATHER for an all-reduce) and folds them in rank order.
// 16-bit: each step in float, rounded back to 16 bits, as GPUHalfSumFunc's
// out[i] = float(in[i]) + float(out[i]) (environment.cpp:135-142).
namespace {
template <typename V>
V FoldOp(ReduceOp op, V acc, V x) {
    switch (op) {
    case ReduceOp::SUM: return x + acc;
    case ReduceOp::PROD: return x * acc;
    case ReduceOp::MAX: return acc < x ? x : acc;
    case ReduceOp::MIN: return x < acc ? x : acc;
    }
    return acc;
}
template <typename E>
void FoldRanks(ReduceOp op, const char* gathered, char* out, Int count, int size) {
    const E* g = reinterpret_cast<const E*>(gathered);
    E* o = reinterpret_cast<E*>(out);
    for (Int i = 0; i < count; ++i) o[i] = g[i];
    for (int r = 1; r < size; ++r)
        for (Int i = 0; i < count; ++i) o[i] = FoldOp(op, o[i], g[r * count + i]);
}
}  // namespace

void Comm::HostFold(bool scatter, DType t, ReduceOp op, const void* send, void* recv, Int count, Device dev,
                    hipStream_t s) {
    const size_t es = DTypeSize(t);
    const Int sendCount = scatter ? count * size_ : count;
    std::vector<char> hs(static_cast<size_t>(sendCount) * es), hr(static_cast<size_t>(count) * size_ * es),
        out(static_cast<size_t>(count) * es);
    if (dev == Device::GPU) {
        ELX_CHECK_HIP(hipMemcpyAsync(hs.data(), send, sendCount * es, hipMemcpyDeviceToHost, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
    } else {
        std::memcpy(hs.data(), send, sendCount * es);
    }
    HostCall(scatter ? ELX_COLL_ALLTOALL : ELX_COLL_ALLGATHER, t, hs.data(), hr.data(), count, 0, 0);
    if (t == DType::F64) {
        FoldRanks<double>(op, hr.data(), out.data(), count, size_);
    } else if (t == DType::F32) {
        FoldRanks<float>(op, hr.data(), out.data(), count, size_);
    } else if (t == DType::I32) {
        FoldRanks<int32_t>(op, hr.data(), out.data(), count, size_);
    } else if (t == DType::I64) {
        FoldRanks<int64_t>(op, hr.data(), out.data(), count, size_);
    } else if (t == DType::U8) {
        FoldRanks<uint8_t>(op, hr.data(), out.data(), count, size_);
    } else {
        const bool bf = t == DType::BF16;
        auto ld = [&](uint16_t v) { return bf ? BF16ToFloat(v) : HalfToFloat(v); };
        auto stv = [&](float v) { return bf ? FloatToBF16(v) : FloatToHalf(v); };
        const uint16_t* g = reinterpret_cast<const uint16_t*>(hr.data());
        uint16_t* o = reinterpret_cast<uint16_t*>(out.data());
        for (Int i = 0; i < count; ++i) o[i] = g[i];
        for (int r = 1; r < size_; ++r)
            for (Int i = 0; i < count; ++i) o[i] = stv(FoldOp(op, ld(o[i]), ld(g[r * count + i])));
    }
    if (dev == Device::GPU) {
        ELX_CHECK_HIP(hipMemcpyAsync(recv, out.data(), count * es, hipMemcpyHostToDevice, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
    } else {
        std::memcpy(recv, out.data(), count * es);
    }
}

void Comm::Bcast(DType t, void* buf, Int count, int root, Device dev, hipStream_t s) {
    const size_t bytes = static_cast<size_t>(count) * DTypeSize(t);
    if (size_ == 1 || count == 0) return;
    GlobalCommStats().calls++;
    if (rank_ != root) GlobalCommStats().bytes += static_cast<int64_t>(bytes);
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        CheckNccl(ncclBroadcast(buf, buf, count, NcclType(t), root, nccl_, s), "ncclBroadcast", nccl_);
        return;
    }
    if (dev == Device::CPU) { HostCall(ELX_COLL_BCAST, t, buf, buf, count, root, 0); return; }
    static Staging stg;
    char* h = static_cast<char*>(stg.Get(bytes));
    ELX_CHECK_HIP(hipMemcpyAsync(h, buf, bytes, hipMemcpyDeviceToHost, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
    HostCall(ELX_COLL_BCAST, t, h, h, count, root, 0);
    ELX_CHECK_HIP(hipMemcpyAsync(buf, h, bytes, hipMemcpyHostToDevice, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
}

void Comm::AllToAllV(DType t, const void* send, const std::vector<Int>& sc, const std::vector<Int>& sd, void* recv,
                     const std::vector<Int>& rc, const std::vector<Int>& rd, Device dev, hipStream_t s) {
    const size_t es = DTypeSize(t);
    const char* sb = static_cast<const char*>(send);
    char* rb = static_cast<char*>(recv);
    auto& st = GlobalCommStats();
    st.calls++;
    for (int q = 0; q < size_; ++q)
        if (q != rank_) st.bytes += static_cast<int64_t>(rc[q] * es);
    // the self portion never leaves the device
    CopyBytes(dev, rb + rd[rank_] * es, sb + sd[rank_] * es, static_cast<size_t>(rc[rank_]) * es, s);
    if (size_ == 1) return;
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        const ncclDataType_t nt = NcclType(t);
        int64_t in_bytes = 0;
        for (int q = 0; q < size_; ++q)
            if (q != rank_) in_bytes += static_cast<int64_t>(rc[q] * es);
        auto rec = CommProf().Begin(s);
        CheckNccl(ncclGroupStart(), "ncclGroupStart");
        for (int q = 0; q < size_; ++q) {
            if (q == rank_) continue;
            if (sc[q] > 0) CheckNccl(ncclSend(sb + sd[q] * es, sc[q], nt, q, nccl_, s), "ncclSend", nccl_);
            if (rc[q] > 0) CheckNccl(ncclRecv(rb + rd[q] * es, rc[q], nt, q, nccl_, s), "ncclRecv", nccl_);
        }
        CheckNccl(ncclGroupEnd(), "ncclGroupEnd", nccl_);
        CommProf().End(rec, s, in_bytes);
        return;
    }
    // host backend: uniform-count all-to-all padded to the largest pair
    std::vector<int64_t> mine(sc.begin(), sc.end()), all(static_cast<size_t>(size_) * size_);
    {
        // gather every rank's send-count vector as doubles (exact for counts < 2^53)
        std::vector<double> md(mine.begin(), mine.end()), ad(all.size());
        HostCall(ELX_COLL_ALLGATHER, DType::F64, md.data(), ad.data(), size_, 0, 0);
        for (size_t i = 0; i < ad.size(); ++i) all[i] = static_cast<int64_t>(ad[i]);
    }
    const Int maxc = *std::max_element(all.begin(), all.end());
    if (maxc == 0) return;
    const size_t pb = static_cast<size_t>(maxc) * es;
    std::vector<char> hs(pb * size_), hr(pb * size_);
    if (dev == Device::GPU) ELX_CHECK_HIP(hipStreamSynchronize(s));
    for (int q = 0; q < size_; ++q) {
        if (q == rank_ || sc[q] == 0) continue;
        if (dev == Device::GPU)
            ELX_CHECK_HIP(hipMemcpy(hs.data() + q * pb, sb + sd[q] * es, sc[q] * es, hipMemcpyDeviceToHost));
        else
            std::memcpy(hs.data() + q * pb, sb + sd[q] * es, sc[q] * es);
    }
    HostCall(ELX_COLL_ALLTOALL, t, hs.data(), hr.data(), maxc, 0, 0);
    for (int q = 0; q < size_; ++q) {
        if (q == rank_ || rc[q] == 0) continue;
        if (dev == Device::GPU)
            ELX_CHECK_HIP(hipMemcpy(rb + rd[q] * es, hr.data() + q * pb, rc[q] * es, hipMemcpyHostToDevice));
        else
            std::memcpy(rb + rd[q] * es, hr.data() + q * pb, rc[q] * es);
    }
}

// ELX_GROUPED_EXCHANGE=0 runs the sets of a group as separate exchanges
bool GroupedExchange() {
    static const bool on = [] {
        const char* e = std::getenv("ELX_GROUPED_EXCHANGE");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

void Comm::AllToAllVGroup(const std::vector<VSet>& sets, Device dev, hipStream_t s) {
    if (sets.size() == 1 || size_ == 1 || !GroupedExchange()) {
        for (const VSet& v : sets) AllToAllV(v.t, v.send, *v.sc, *v.sd, v.recv, *v.rc, *v.rd, dev, s);
        return;
    }
    if (kind_ == Kind::HOST) {
        HostGroup(sets, dev, s);
        return;
    }
    ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
    auto& st = GlobalCommStats();
    int64_t in_bytes = 0;
    for (const VSet& v : sets) {
        const size_t es = DTypeSize(v.t);
        st.calls++;
        for (int q = 0; q < size_; ++q)
            if (q != rank_) in_bytes += static_cast<int64_t>((*v.rc)[q] * es);
        // the self portion never leaves the device
        CopyBytes(dev, static_cast<char*>(v.recv) + (*v.rd)[rank_] * es,
                  static_cast<const char*>(v.send) + (*v.sd)[rank_] * es, static_cast<size_t>((*v.rc)[rank_]) * es, s);
    }
    st.bytes += in_bytes;
    auto rec = CommProf().Begin(s);
    CheckNccl(ncclGroupStart(), "ncclGroupStart");
    for (const VSet& v : sets) {
        const size_t es = DTypeSize(v.t);
        const ncclDataType_t nt = NcclType(v.t);
        const char* sb = static_cast<const char*>(v.send);
        char* rb = static_cast<char*>(v.recv);
        for (int q = 0; q < size_; ++q) {
            if (q == rank_) continue;
            if ((*v.sc)[q] > 0) CheckNccl(ncclSend(sb + (*v.sd)[q] * es, (*v.sc)[q], nt, q, nccl_, s), "ncclSend", nccl_);
            if ((*v.rc)[q] > 0) CheckNccl(ncclRecv(rb + (*v.rd)[q] * es, (*v.rc)[q], nt, q, nccl_, s), "ncclRecv", nccl_);
        }
    }
    CheckNccl(ncclGroupEnd(), "ncclGroupEnd", nccl_);
    CommProf().End(rec, s, in_bytes);
}

// The host backend's grouped exchange: ONE all-to-all carrying every set, each
// peer's message the sets' portions for it concatenated in set order — the
// order in which the RCCL branch posts its sends and receives per peer (and in
// which RCCL matches them), with the same per-set counts and displacements.
// 2-byte carrier units (every element size is a multiple); self portions never
// leave the device.
void Comm::HostGroup(const std::vector<VSet>& sets, Device dev, hipStream_t s) {
    constexpr size_t U = 2;
    std::vector<Int> sc(size_, 0), rc(size_, 0), sd(size_, 0), rd(size_, 0);
    for (const VSet& v : sets) {
        const size_t es = DTypeSize(v.t);
        for (int q = 0; q < size_; ++q) {
            if (q == rank_) continue;
            sc[q] += static_cast<Int>((*v.sc)[q] * es / U);
            rc[q] += static_cast<Int>((*v.rc)[q] * es / U);
        }
        CopyBytes(dev, static_cast<char*>(v.recv) + (*v.rd)[rank_] * es,
                  static_cast<const char*>(v.send) + (*v.sd)[rank_] * es, static_cast<size_t>((*v.rc)[rank_]) * es, s);
    }
    for (int q = 1; q < size_; ++q) {
        sd[q] = sd[q - 1] + sc[q - 1];
        rd[q] = rd[q - 1] + rc[q - 1];
    }
    std::vector<char> hs(static_cast<size_t>(sd[size_ - 1] + sc[size_ - 1]) * U + U);
    std::vector<char> hr(static_cast<size_t>(rd[size_ - 1] + rc[size_ - 1]) * U + U);
    auto move = [&](void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
        if (bytes == 0) return;
        if (dev == Device::GPU) ELX_CHECK_HIP(hipMemcpy(dst, src, bytes, kind));
        else std::memcpy(dst, src, bytes);
    };
    if (dev == Device::GPU) ELX_CHECK_HIP(hipStreamSynchronize(s));
    for (int q = 0; q < size_; ++q) {
        if (q == rank_) continue;
        size_t off = static_cast<size_t>(sd[q]) * U;
        for (const VSet& v : sets) {
            const size_t es = DTypeSize(v.t), bytes = static_cast<size_t>((*v.sc)[q]) * es;
            move(hs.data() + off, static_cast<const char*>(v.send) + (*v.sd)[q] * es, bytes, hipMemcpyDeviceToHost);
            off += bytes;
        }
    }
    std::vector<Int> sc0 = sc, rc0 = rc;  // self entries stay 0: handled above
    AllToAllV(DType::F16, hs.data(), sc0, sd, hr.data(), rc0, rd, Device::CPU, nullptr);
    for (int q = 0; q < size_; ++q) {
        if (q == rank_) continue;
        size_t off = static_cast<size_t>(rd[q]) * U;
        for (const VSet& v : sets) {
            const size_t es = DTypeSize(v.t), bytes = static_cast<size_t>((*v.rc)[q]) * es;
            move(static_cast<char*>(v.recv) + (*v.rd)[q] * es, hr.data() + off, bytes, hipMemcpyHostToDevice);
            off += bytes;
        }
    }
}

void Comm::SendRecv(DType t, const void* send, int dest, void* recv, int src, Int count, Device dev, hipStream_t s) {
    SendRecv(t, send, count, dest, recv, count, src, dev, s);
}

void Comm::SendRecv(DType t, const void* send, Int scount, int dest, void* recv, Int rcount, int src, Device dev,
                    hipStream_t s) {
    const size_t es = DTypeSize(t);
    ELX_REQUIRE(dest >= 0 && dest < size_ && src >= 0 && src < size_, "SendRecv: bad peer ", dest, "/", src, " of ",
                size_);
    ELX_REQUIRE(scount >= 0 && rcount >= 0, "SendRecv: negative count");
    auto& st = GlobalCommStats();
    st.calls++;
    if (src != rank_) st.bytes += static_cast<int64_t>(rcount * es);
    if (dest == rank_ && src == rank_) {
        ELX_REQUIRE(scount == rcount, "SendRecv to self: send count ", scount, " != receive count ", rcount);
        CopyBytes(dev, recv, send, static_cast<size_t>(rcount) * es, s);
        return;
    }
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        if (scount == 0 && rcount == 0) return;
        const ncclDataType_t nt = NcclType(t);
        CheckNccl(ncclGroupStart(), "ncclGroupStart");
        if (scount > 0) CheckNccl(ncclSend(send, scount, nt, dest, nccl_, s), "ncclSend", nccl_);
        if (rcount > 0) CheckNccl(ncclRecv(recv, rcount, nt, src, nccl_, s), "ncclRecv", nccl_);
        CheckNccl(ncclGroupEnd(), "ncclGroupEnd", nccl_);
        return;
    }
    ELX_REQUIRE(scount == rcount, "SendRecv on the host backend needs equal send and receive counts (",
                scount, " vs ", rcount, ")");
    const Int count = scount;
    const size_t bytes = static_cast<size_t>(count) * es;
    if (count == 0) return;
    if (dev == Device::CPU) { HostCall(ELX_COLL_SENDRECV, t, send, recv, count, dest, src); return; }
    static Staging stg;
    char* h = static_cast<char*>(stg.Get(bytes * 2));
    ELX_CHECK_HIP(hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
    HostCall(ELX_COLL_SENDRECV, t, h, h + bytes, count, dest, src);
    ELX_CHECK_HIP(hipMemcpyAsync(recv, h + bytes, bytes, hipMemcpyHostToDevice, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
}

void Comm::Barrier() {
    if (size_ == 1) return;
    if (kind_ == Kind::RCCL) {
        hipStream_t s = Runtime::Get().CommStream();
        static Buffer flag;
        if (!flag.data()) flag.Reset(Device::GPU, 64, nullptr);
        CheckNccl(ncclAllReduce(flag.data(), flag.data(), 1, ncclFloat32, ncclSum, nccl_, s), "barrier", nccl_);
        ELX_CHECK_HIP(hipStreamSynchronize(s));
        return;
    }
    HostCall(ELX_COLL_BARRIER, DType::F32, nullptr, nullptr, 0, 0, 0);
}

void WatchdogStage(const char* name, double seconds) {
    Watchdog& w = WD();
    std::lock_guard<std::mutex> lk(w.mu);
    w.stage = name ? name : "";
    w.budget = seconds;
    w.deadline = seconds > 0 ? Now() + seconds : 0;
    std::fprintf(stderr, "[elx] stage %s%s\n", w.stage.c_str(),
                 seconds > 0 ? Cat(" (deadline ", seconds, " s)").c_str() : "");
    std::fflush(stderr);
    if (!w.started) {
        w.started = true;
        std::thread([&w] { w.Loop(); }).detach();
    }
}

void WatchdogEpitaph(const char* text, int exit_code) {
    Watchdog& w = WD();
    std::lock_guard<std::mutex> lk(w.mu);
    w.epitaph = text ? text : "";
    w.epitaph_code = exit_code;
}

void WatchdogRegister(ncclComm_t c) {
    if (!c) return;
    Watchdog& w = WD();
    std::lock_guard<std::mutex> lk(w.mu);
    w.comms.push_back(c);
}

void WatchdogUnregister(ncclComm_t c) {
    Watchdog& w = WD();
    std::lock_guard<std::mutex> lk(w.mu);
    w.comms.erase(std::remove(w.comms.begin(), w.comms.end(), c), w.comms.end());
}

namespace {
void SendAll(int fd, const char* p, size_t n) {
    while (n) {
        const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k <= 0) throw CommError(Cat("rendezvous send failed: ", std::strerror(errno)));
        p += k;
        n -= static_cast<size_t>(k);
    }
}
void RecvAll(int fd, char* p, size_t n, double deadline) {
    while (n) {
        pollfd pf{fd, POLLIN, 0};
        const int left = static_cast<int>(std::max(0.0, deadline - Now()) * 1000);
        if (::poll(&pf, 1, left) <= 0) throw CommError("rendezvous: timed out waiting for rank 0's data");
        const ssize_t k = ::recv(fd, p, n, 0);
        if (k <= 0) throw CommError("rendezvous: rank 0 closed the connection early");
        p += k;
        n -= static_cast<size_t>(k);
    }
}
struct Fd {
    int fd = -1;
    ~Fd() { if (fd >= 0) ::close(fd); }
};
}  // namespace

// Handshake: each client sends kRdvMagic, its rank, the world size and the
// job's token; rank 0 serves each valid rank in 1..size-1 once and drops
// anything else (a stray or foreign connection never uses up a peer's slot,
// and the id is sent only to peers that name this rendezvous and this job).
// The token is a 64-bit FNV-1a hash of ELX_RENDEZVOUS_SECRET, which every rank
// of a job shares (unset: 0).  Rank 0 listens on MASTER_ADDR itself when that
// is 127.0.0.1 or a non-loopback address of this host; on every interface only
// when MASTER_ADDR resolves to another loopback alias (Debian maps the host's
// own name to 127.0.1.1 while peers on other nodes dial the real address) or
// the address is not local (EADDRNOTAVAIL).  The peers dial MASTER_ADDR.
namespace {
constexpr char kRdvMagic[8] = {'E', 'L', 'X', 'R', 'D', 'V', '0', '2'};
struct RdvHello {
    char magic[8];
    int32_t rank, size;
    uint64_t token;
};
uint64_t RdvToken() {
    const char* s = std::getenv("ELX_RENDEZVOUS_SECRET");
    if (!s || !*s) return 0;
    uint64_t h = 14695981039346656037ull;
    for (; *s; ++s) h = (h ^ static_cast<unsigned char>(*s)) * 1099511628211ull;
    return h;
}
bool ResolveV4(const char* addr, int port, sockaddr_in& out) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    const std::string ps = std::to_string(port);
    if (::getaddrinfo(addr && *addr ? addr : "127.0.0.1", ps.c_str(), &hints, &res) != 0 || !res) return false;
    std::memcpy(&out, res->ai_addr, sizeof(sockaddr_in));
    ::freeaddrinfo(res);
    return true;
}
// bind rank 0's listener (policy above)
void BindListener(int fd, const sockaddr_in& sa, int port) {
    const uint32_t ip = ntohl(sa.sin_addr.s_addr);
    const bool loopback = (ip >> 24) == 127;
    sockaddr_in at = sa;
    if (loopback && ip != 0x7F000001u) at.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(fd, reinterpret_cast<const sockaddr*>(&at), sizeof(at)) == 0) return;
    if (errno == EADDRNOTAVAIL && at.sin_addr.s_addr != htonl(INADDR_ANY)) {
        at.sin_addr.s_addr = htonl(INADDR_ANY);
        if (::bind(fd, reinterpret_cast<const sockaddr*>(&at), sizeof(at)) == 0) return;
    }
    throw CommError(Cat("rendezvous: bind to port ", port, " failed: ", std::strerror(errno)));
}
}  // namespace

void RendezvousBcast(void* data, size_t bytes, int rank, int size, const char* addr, int port, double timeout_s) {
    ELX_REQUIRE(size >= 1 && rank >= 0 && rank < size, "rendezvous: bad rank ", rank, " of ", size);
    ELX_REQUIRE(port > 0 && port < 65536, "rendezvous: bad port ", port);
    if (size == 1) return;
    const double deadline = Now() + timeout_s;
    const uint64_t token = RdvToken();
    sockaddr_in sa{};
    if (!ResolveV4(addr, port, sa)) throw CommError(Cat("rendezvous: cannot resolve ", addr ? addr : "(null)"));
    if (rank == 0) {
        Fd ls;
        ls.fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (ls.fd < 0) throw CommError("rendezvous: socket() failed");
        const int one = 1;
        ::setsockopt(ls.fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        BindListener(ls.fd, sa, port);
        if (::listen(ls.fd, std::max(size, 128)) != 0) throw CommError("rendezvous: listen() failed");
        std::vector<bool> served(size, false);
        int left = size - 1;
        while (left > 0) {
            pollfd pf{ls.fd, POLLIN, 0};
            const int ms = static_cast<int>(std::max(0.0, deadline - Now()) * 1000);
            if (::poll(&pf, 1, ms) <= 0)
                throw CommError(Cat("rendezvous: only ", size - 1 - left, " of ", size - 1, " peers connected in time"));
            Fd peer;
            peer.fd = ::accept(ls.fd, nullptr, nullptr);
            if (peer.fd < 0) continue;
            RdvHello h{};
            try {
                RecvAll(peer.fd, reinterpret_cast<char*>(&h), sizeof(h), std::min(deadline, Now() + 5.0));
            } catch (const CommError&) {
                continue;  // silent or short: not a peer
            }
            if (std::memcmp(h.magic, kRdvMagic, sizeof(kRdvMagic)) != 0 || h.size != size || h.rank < 1 ||
                h.rank >= size || h.token != token || served[h.rank])
                continue;
            SendAll(peer.fd, static_cast<const char*>(data), bytes);
            served[h.rank] = true;
            --left;
        }
        return;
    }
    RdvHello hello{};
    std::memcpy(hello.magic, kRdvMagic, sizeof(kRdvMagic));
    hello.rank = rank;
    hello.size = size;
    hello.token = token;
    for (;;) {  // rank 0 may not be listening yet
        Fd s;
        s.fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (s.fd < 0) throw CommError("rendezvous: socket() failed");
        if (::connect(s.fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) {
            SendAll(s.fd, reinterpret_cast<const char*>(&hello), sizeof(hello));
            RecvAll(s.fd, static_cast<char*>(data), bytes, deadline);
            return;
        }
        if (Now() > deadline) throw CommError(Cat("rendezvous: could not reach rank 0 at ", addr ? addr : "127.0.0.1", ":", port));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}

std::shared_ptr<Comm>& WorldComm() {
    static std::shared_ptr<Comm> w = Comm::Self();
    return w;
}

void InitWorldFromEnv() {
    auto geti = [](const char* k, int dflt) {
        const char* e = std::getenv(k);
        return e && *e ? std::atoi(e) : dflt;
    };
    // launched (RANK and WORLD_SIZE set, as torch.distributed.run does): an RCCL
    // world, one process per GPU, even of size 1; otherwise (or ELX_WORLD=self)
    // the size-1 world
    const char* mode = std::getenv("ELX_WORLD");
    const bool launched = std::getenv("RANK") && std::getenv("WORLD_SIZE");
    if (!launched || (mode && std::string(mode) == "self")) {
        WorldComm() = Comm::Self();
        return;
    }
    const int size = geti("WORLD_SIZE", 1), rank = geti("RANK", 0);
    ELX_REQUIRE(size >= 1 && rank >= 0 && rank < size, "El::Initialize: RANK ", rank, " / WORLD_SIZE ", size);
    Runtime::Get().SetDevice(geti("LOCAL_RANK", 0));
    Runtime::Get().EnsureGPU();
    const char* addr = std::getenv("MASTER_ADDR");
    const int port = geti("ELX_RENDEZVOUS_PORT", geti("MASTER_PORT", 29499) + 1);
    unsigned char id[128] = {};
    if (rank == 0) {
        ncclUniqueId uid;
        CheckNccl(ncclGetUniqueId(&uid), "ncclGetUniqueId");
        std::memcpy(id, uid.internal, 128);
    }
    RendezvousBcast(id, sizeof(id), rank, size, addr ? addr : "127.0.0.1", port,
                    geti("ELX_RENDEZVOUS_TIMEOUT", 300));
    WorldComm() = Comm::InitRCCL(rank, size, id);
}

}  // namespace elx
