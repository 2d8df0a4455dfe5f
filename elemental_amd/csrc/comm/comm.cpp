#include "comm.hpp"
#include <chrono>
#include <cstring>
#include <algorithm>

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

ncclDataType_t NcclType(DType t) {
    switch (t) {
    case DType::F32: return ncclFloat32;
    case DType::F64: return ncclFloat64;
    case DType::F16: return ncclFloat16;
    case DType::BF16: return ncclBfloat16;
    }
    throw LogicError("bad dtype");
}

void CheckNccl(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw CommError(Cat("RCCL ", what, " failed: ", ncclGetErrorString(r)));
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
    CheckNccl(ncclCommInitRank(&c->nccl_, size, uid, rank), "ncclCommInitRank");
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
    if (nccl_ && owned_) (void)ncclCommDestroy(nccl_);
}

std::shared_ptr<Comm> Comm::Split(int color, int key) {
    if (kind_ == Kind::SELF) return Self();
    auto c = std::shared_ptr<Comm>(new Comm());
    c->kind_ = kind_;
    if (kind_ == Kind::RCCL) {
        CheckNccl(ncclCommSplit(nccl_, color, key, &c->nccl_, nullptr), "ncclCommSplit");
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
        CheckNccl(ncclAllGather(send, recv, count, NcclType(t), nccl_, s), "ncclAllGather");
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

void Comm::ReduceScatter(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s) {
    const size_t es = DTypeSize(t), bytes = static_cast<size_t>(count) * es;
    auto& st = GlobalCommStats();
    st.calls++;
    st.bytes += static_cast<int64_t>(bytes) * (size_ - 1);
    if (size_ == 1) { CopyBytes(dev, recv, send, bytes, s); return; }
    if (count == 0) return;
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        CheckNccl(ncclReduceScatter(send, recv, count, NcclType(t), ncclSum, nccl_, s), "ncclReduceScatter");
        return;
    }
    if (t == DType::F16 || t == DType::BF16) { HostSum16(true, t, send, recv, count, dev, s); return; }
    if (dev == Device::CPU) { HostCall(ELX_COLL_REDUCE_SCATTER, t, send, recv, count, 0, 0); return; }
    static Staging stg;
    char* h = static_cast<char*>(stg.Get(bytes * (size_ + 1)));
    ELX_CHECK_HIP(hipMemcpyAsync(h, send, bytes * size_, hipMemcpyDeviceToHost, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
    HostCall(ELX_COLL_REDUCE_SCATTER, t, h, h + bytes * size_, count, 0, 0);
    ELX_CHECK_HIP(hipMemcpyAsync(recv, h + bytes * size_, bytes, hipMemcpyHostToDevice, s));
    ELX_CHECK_HIP(hipStreamSynchronize(s));
}

void Comm::AllReduce(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s) {
    const size_t bytes = static_cast<size_t>(count) * DTypeSize(t);
    if (size_ == 1) { CopyBytes(dev, recv, send, bytes, s); return; }
    if (count == 0) return;
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        CheckNccl(ncclAllReduce(send, recv, count, NcclType(t), ncclSum, nccl_, s), "ncclAllReduce");
        return;
    }
    if (t == DType::F16 || t == DType::BF16) { HostSum16(false, t, send, recv, count, dev, s); return; }
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
// a reduce-scatter, ALLGATHER for an all-reduce) and folds them in rank order,
// each addition done in float and rounded back to 16 bits, as
// GPUHalfSumFunc's out[i] = float(in[i]) + float(out[i]) (environment.cpp:135-142).
void Comm::HostSum16(bool scatter, DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s) {
    const size_t es = DTypeSize(t);
    const Int sendCount = scatter ? count * size_ : count;
    std::vector<uint16_t> hs(static_cast<size_t>(sendCount)), hr(static_cast<size_t>(count) * size_);
    if (dev == Device::GPU) {
        ELX_CHECK_HIP(hipMemcpyAsync(hs.data(), send, sendCount * es, hipMemcpyDeviceToHost, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
    } else {
        std::memcpy(hs.data(), send, sendCount * es);
    }
    HostCall(scatter ? ELX_COLL_ALLTOALL : ELX_COLL_ALLGATHER, t, hs.data(), hr.data(), count, 0, 0);
    const bool bf = t == DType::BF16;
    auto ld = [&](uint16_t v) { return bf ? BF16ToFloat(v) : HalfToFloat(v); };
    auto st = [&](float v) { return bf ? FloatToBF16(v) : FloatToHalf(v); };
    std::vector<uint16_t> out(hr.begin(), hr.begin() + count);
    for (int r = 1; r < size_; ++r)
        for (Int i = 0; i < count; ++i) out[i] = st(ld(hr[r * count + i]) + ld(out[i]));
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
        CheckNccl(ncclBroadcast(buf, buf, count, NcclType(t), root, nccl_, s), "ncclBroadcast");
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
            if (sc[q] > 0) CheckNccl(ncclSend(sb + sd[q] * es, sc[q], nt, q, nccl_, s), "ncclSend");
            if (rc[q] > 0) CheckNccl(ncclRecv(rb + rd[q] * es, rc[q], nt, q, nccl_, s), "ncclRecv");
        }
        CheckNccl(ncclGroupEnd(), "ncclGroupEnd");
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

void Comm::AllToAllVGroup(const std::vector<VSet>& sets, Device dev, hipStream_t s) {
    if (sets.size() == 1 || kind_ != Kind::RCCL || size_ == 1) {
        for (const VSet& v : sets) AllToAllV(v.t, v.send, *v.sc, *v.sd, v.recv, *v.rc, *v.rd, dev, s);
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
            if ((*v.sc)[q] > 0) CheckNccl(ncclSend(sb + (*v.sd)[q] * es, (*v.sc)[q], nt, q, nccl_, s), "ncclSend");
            if ((*v.rc)[q] > 0) CheckNccl(ncclRecv(rb + (*v.rd)[q] * es, (*v.rc)[q], nt, q, nccl_, s), "ncclRecv");
        }
    }
    CheckNccl(ncclGroupEnd(), "ncclGroupEnd");
    CommProf().End(rec, s, in_bytes);
}

void Comm::SendRecv(DType t, const void* send, int dest, void* recv, int src, Int count, Device dev, hipStream_t s) {
    const size_t bytes = static_cast<size_t>(count) * DTypeSize(t);
    ELX_REQUIRE(dest >= 0 && dest < size_ && src >= 0 && src < size_, "SendRecv: bad peer ", dest, "/", src, " of ",
                size_);
    auto& st = GlobalCommStats();
    st.calls++;
    if (src != rank_) st.bytes += static_cast<int64_t>(bytes);
    if (count == 0) return;
    if (dest == rank_ && src == rank_) { CopyBytes(dev, recv, send, bytes, s); return; }
    if (kind_ == Kind::RCCL) {
        ELX_REQUIRE(dev == Device::GPU, "RCCL collectives need device buffers");
        const ncclDataType_t nt = NcclType(t);
        CheckNccl(ncclGroupStart(), "ncclGroupStart");
        CheckNccl(ncclSend(send, count, nt, dest, nccl_, s), "ncclSend");
        CheckNccl(ncclRecv(recv, count, nt, src, nccl_, s), "ncclRecv");
        CheckNccl(ncclGroupEnd(), "ncclGroupEnd");
        return;
    }
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
        CheckNccl(ncclAllReduce(flag.data(), flag.data(), 1, ncclFloat32, ncclSum, nccl_, s), "barrier");
        ELX_CHECK_HIP(hipStreamSynchronize(s));
        return;
    }
    HostCall(ELX_COLL_BARRIER, DType::F32, nullptr, nullptr, 0, 0, 0);
}

}  // namespace elx
