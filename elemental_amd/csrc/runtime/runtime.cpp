#include "runtime.hpp"
#include "../kernels/kernels.hpp"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

namespace elx {

Runtime& Runtime::Get() {
    static Runtime* rt = new Runtime();  // intentionally leaked: outlives static dtors
    return *rt;
}

void Runtime::SetDevice(int dev) {
    std::lock_guard<std::mutex> lk(mu_);
    if (gpu_ready_ && dev != device_)
        throw LogicError(Cat("elx: device already initialised as ", device_, "; cannot switch to ", dev));
    device_ = dev;
}

void Runtime::EnsureGPU() {
    if (gpu_ready_) return;
    std::lock_guard<std::mutex> lk(mu_);
    if (gpu_ready_) return;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        throw NoDeviceError("elx: no HIP device visible (the GPU path never falls back to the CPU)");
    if (device_ < 0) {
        // One rank per GPU: LOCAL_RANK (torchrun) or the launcher's local-rank
        // variables pick the device, like ComputeDeviceId (src/hydrogen/device/GPU.cpp:30-50).
        int local = 0;
        for (const char* v : {"LOCAL_RANK", "SLURM_LOCALID", "OMPI_COMM_WORLD_LOCAL_RANK",
                              "MV2_COMM_WORLD_LOCAL_RANK"}) {
            if (const char* s = std::getenv(v)) { local = std::atoi(s); break; }
        }
        device_ = local % n;
    }
    ELX_CHECK_HIP(hipSetDevice(device_));
    hipDeviceProp_t prop;
    ELX_CHECK_HIP(hipGetDeviceProperties(&prop, device_));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
        throw NoDeviceError(Cat("elx: device ", device_, " is ", prop.gcnArchName,
                                "; this build targets gfx950 (MI355X) only"));
    // ELX_COMM_CUS = R > 0: the compute stream (the MFMA panel updates) is
    // masked off R CUs so the comm stream's pack/unpack and RCCL kernels always
    // find free CUs while a full-machine GEMM grid is resident.  The reserved CUs
    // are spread so that both a blocked (i / 32) and an interleaved (i % 8)
    // CU-to-XCD numbering put them on different XCDs.
    const int ncu = prop.multiProcessorCount;
    if (const char* e = std::getenv("ELX_COMM_CUS")) reserved_cus_ = std::max(0, std::atoi(e));
    if (reserved_cus_ > 0 && reserved_cus_ < ncu) {
        std::vector<uint32_t> mask((ncu + 31) / 32, 0);
        for (int i = 0; i < ncu; ++i) mask[i / 32] |= 1u << (i % 32);
        const int slice = ncu / reserved_cus_;
        for (int r = 0; r < reserved_cus_; ++r) {
            const int i = std::min(ncu - 1, r * slice + (r % 8) % std::max(1, slice));
            mask[i / 32] &= ~(1u << (i % 32));
        }
        ELX_CHECK_HIP(hipExtStreamCreateWithCUMask(&compute_, static_cast<uint32_t>(mask.size()), mask.data()));
    } else {
        reserved_cus_ = 0;
        ELX_CHECK_HIP(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking));
    }
    int lo = 0, hi = 0;
    ELX_CHECK_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // communication gets the higher priority so panel broadcasts are not
    // starved by the long-running MFMA update they overlap with
    // (ELX_COMM_PRIORITY=0: the compute stream's priority instead; A/B timing)
    const char* pe = getenv("ELX_COMM_PRIORITY");
    ELX_CHECK_HIP(hipStreamCreateWithPriority(&comm_, hipStreamNonBlocking, pe && atoi(pe) == 0 ? lo : hi));
    // The cache's backing store is hipMalloc / hipFree, as hipCUB's
    // CachingDeviceAllocator's is (cudaMalloc / cudaFree): the driver's
    // stream-ordered pool (hipMallocFromPoolAsync) was measured to corrupt live
    // blocks on this ROCm (runtime.hpp, tools/pool_trim_probe.hip).
    if (!max_cached_set_) {
        // H_CUB_MAX_CACHED_SIZE as the reference reads it (cub.cpp:37-43)
        for (const char* v : {"ELX_POOL_MAX_CACHED", "H_CUB_MAX_CACHED_SIZE"}) {
            if (const char* e = std::getenv(v)) { max_cached_ = std::strtoull(e, nullptr, 10); break; }
        }
    }
    gpu_ready_ = true;
}

namespace {
// The bin geometry (cub.cpp:21-35): ELX's default, or CUB's when any of
// H_CUB_BIN_GROWTH / H_CUB_MIN_BIN / H_CUB_MAX_BIN is set.
struct BinConfig {
    bool cub = false;
    unsigned growth = 2, min_bin = 1, max_bin = ~0u;  // max_bin ~0u: CUB's INVALID_BIN (no limit)
    bool debug = false;
};
unsigned EnvUint(const char* name, unsigned def, bool& set) {
    const char* e = std::getenv(name);
    if (!e || !*e) return def;
    set = true;
    return static_cast<unsigned>(std::strtoul(e, nullptr, 10));
}
const BinConfig& Bins() {
    static const BinConfig c = [] {
        BinConfig b;
        bool set = false;
        b.growth = std::max(2u, EnvUint("H_CUB_BIN_GROWTH", 2, set));
        b.min_bin = EnvUint("H_CUB_MIN_BIN", 1, set);
        b.max_bin = EnvUint("H_CUB_MAX_BIN", ~0u, set);
        b.cub = set;
        bool dset = false;
        b.debug = EnvUint("H_CUB_DEBUG", 0, dset) != 0;
        return b;
    }();
    return c;
}
constexpr size_t kGranule = 512;  // every block is a multiple of 512 B (256-B aligned pointers)
constexpr size_t kSizeMax = std::numeric_limits<size_t>::max();
// round b up to a multiple of g; 0 (no bin) when that does not fit in size_t
size_t RoundUp(size_t b, size_t g) { return b > kSizeMax - (g - 1) ? 0 : (b + g - 1) / g * g; }
size_t MulSat(size_t a, unsigned g) { return a > kSizeMax / g ? kSizeMax : a * g; }
// growth^k, saturating at SIZE_MAX
size_t PowSat(unsigned g, unsigned k) {
    size_t r = 1;
    for (unsigned i = 0; i < k && r != kSizeMax; ++i) r = MulSat(r, g);
    return r;
}
const char* StreamTag(hipStream_t s, hipStream_t compute, hipStream_t comm) {
    return s == compute ? " (compute)" : s == comm ? " (comm)" : "";
}
}  // namespace

// 0 when no bin can hold b (the rounding would overflow size_t); Alloc then
// reports out-of-memory instead of handing out a zero-byte block
size_t Runtime::BinBytes(size_t b, bool* cacheable) {
    const BinConfig& c = Bins();
    if (cacheable) *cacheable = true;
    if (c.cub) {
        // CachingDeviceAllocator::DeviceAllocate: above max_bin_bytes the block
        // is sized exactly and not cached; else the nearest growth^k >= bytes,
        // at least growth^min_bin
        const size_t maxb = c.max_bin == ~0u ? kSizeMax : PowSat(c.growth, c.max_bin);
        if (b > maxb) {
            if (cacheable) *cacheable = false;
            return RoundUp(std::max<size_t>(b, 1), kGranule);
        }
        size_t p = PowSat(c.growth, c.min_bin);
        while (p < b && p != kSizeMax) p = MulSat(p, c.growth);
        if (p < b) return 0;  // saturated below the request: no bin
        return RoundUp(std::max<size_t>(p, 1), kGranule);
    }
    // powers of two up to 1 MiB (CUB bin_growth 2), then eight bins per octave
    if (b <= kGranule) return kGranule;
    if (b <= (size_t(1) << 20)) {
        size_t p = kGranule;
        while (p < b) p <<= 1;
        return p;
    }
    size_t top = size_t(1) << 20;
    while ((top << 1) <= b && top < (size_t(1) << 62)) top <<= 1;
    return RoundUp(b, top / 8);
}

hipEvent_t Runtime::EventLocked() {
    hipEvent_t ev = nullptr;
    if (!spare_events_.empty()) { ev = spare_events_.back(); spare_events_.pop_back(); }
    else ELX_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return ev;
}

void* Runtime::Backing(size_t bin) {
    // called without mu_: hipMalloc never runs under the allocator's lock
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bin);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
        (void)hipGetLastError();
        {  // give the cache back and retry once, after every release has landed
            std::lock_guard<std::mutex> lk(mu_);
            ReleaseCachedLocked(0);
        }
        WaitReleases();
        e = hipMalloc(&p, bin);
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        size_t fr = 0, tot = 0;
        (void)hipMemGetInfo(&fr, &tot);
        throw HIPError(Cat("elx_pool_alloc: ", hipGetErrorString(e), " (", bin, " bytes requested, ",
                           fr, " bytes available, ", tot, " bytes total)"));
    }
    return p;
}

void Runtime::QueueReleaseLocked(void* p, size_t bin, hipEvent_t ready) {
    // The block goes back to the driver once its free's event completed (CUB
    // returns over-cap blocks with a synchronous cudaFree), but neither the
    // event wait nor hipFree (which waits for the whole device) run on the
    // caller's thread or under mu_: the release thread does both.
    pending_.push_back(Pending{p, bin, ready});
    if (!releaser_started_) {
        releaser_started_ = true;
        releaser_ = std::thread([this] { ReleaseLoop(); });
        // drain before the HIP runtime tears down (registered after hipInit, so
        // it runs before the runtime's own exit handlers)
        std::atexit([] { Runtime::Get().StopReleaser(); });
    }
    release_cv_.notify_one();
    if (Bins().debug)
        std::fprintf(stderr, "elx_pool[dev %d]: queued block %p (%zu bytes) for release to the driver "
                             "after event %p (cached %zu, live %zu)\n",
                     device_, p, bin, (void*)ready, cached_, live_bin_);
}

void Runtime::ReleaseLoop() {
    (void)hipSetDevice(device_);
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
        release_cv_.wait(lk, [this] { return !pending_.empty() || stop_; });
        if (pending_.empty()) break;  // stop_ with nothing left
        const Pending x = pending_.front();
        pending_.pop_front();
        releasing_ = true;
        lk.unlock();
        const hipError_t e1 = hipEventSynchronize(x.ready);
        const hipError_t e2 = hipFree(x.p);
        if (e1 != hipSuccess || e2 != hipSuccess)
            std::fprintf(stderr, "elx_pool[dev %d]: releasing block %p failed: %s / %s\n", device_, x.p,
                         hipGetErrorString(e1), hipGetErrorString(e2));
        lk.lock();
        releasing_ = false;
        backing_ -= x.bin;
        spare_events_.push_back(x.ready);
        if (Bins().debug)
            std::fprintf(stderr, "elx_pool[dev %d]: returned block %p (%zu bytes) to the driver (cached %zu, live %zu)\n",
                         device_, x.p, x.bin, cached_, live_bin_);
        idle_cv_.notify_all();
    }
}

void Runtime::WaitReleases() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_cv_.wait(lk, [this] { return pending_.empty() && !releasing_; });
}

void Runtime::StopReleaser() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (!releaser_started_ || stop_) return;
        stop_ = true;
    }
    release_cv_.notify_one();
    if (releaser_.joinable()) releaser_.join();
}

void Runtime::ReleaseCachedLocked(size_t keep) {
    // largest blocks first, each queued for release behind its free's event
    while (cached_ > keep && !cache_.empty()) {
        auto it = std::prev(cache_.end());
        const size_t bin = it->first;
        const Cached c = it->second;
        cached_ -= bin;
        cache_.erase(it);
        QueueReleaseLocked(c.p, bin, c.ready);
    }
}

void* Runtime::Alloc(size_t bytes, hipStream_t s) {
    EnsureGPU();
    if (bytes == 0) return nullptr;
    if (!s) s = compute_;
    bool cacheable = true;
    const size_t bin = BinBytes(bytes, &cacheable);
    if (bin < bytes)  // BinBytes' overflow marker (0): no bin holds the request
        throw HIPError(Cat("elx_pool_alloc: out of memory (", bytes, " bytes requested: larger than any block)"));
    // ELX_POOL_CACHE=0 (debug): no caching, every request from the backing pool
    static const bool nocache = [] { const char* e = std::getenv("ELX_POOL_CACHE"); return e && e[0] == '0'; }();
    void* p = nullptr;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto [lo, hi] = cache_.equal_range(bin);
        if (nocache || !cacheable) lo = hi;
        if (lo != hi) {
            // prefer a block last used on this stream, then one whose free has
            // completed, then any (ordered behind its free's event)
            auto pick = hi;
            for (auto it = lo; it != hi; ++it)
                if (it->second.stream == s) { pick = it; break; }
            if (pick == hi)
                for (auto it = lo; it != hi; ++it)
                    if (hipEventQuery(it->second.ready) == hipSuccess) { pick = it; break; }
            if (pick == hi) pick = lo;
            const bool cross = pick->second.stream != s;
            const bool waits = hipEventQuery(pick->second.ready) != hipSuccess;
            if (waits) ELX_CHECK_HIP(hipStreamWaitEvent(s, pick->second.ready, 0));
            p = pick->second.p;
            if (Bins().debug)
                std::fprintf(stderr,
                             "elx_pool[dev %d]: reused cached block %p (%zu bytes, bin %zu) for stream %p%s "
                             "(freed on stream %p%s, event %p%s)\n",
                             device_, p, bytes, bin, (void*)s, StreamTag(s, compute_, comm_),
                             (void*)pick->second.stream, StreamTag(pick->second.stream, compute_, comm_),
                             (void*)pick->second.ready,
                             cross ? (waits ? ": cross-stream reuse, the new stream waits on the event"
                                            : ": cross-stream reuse, event already complete")
                                   : ": same stream");
            spare_events_.push_back(pick->second.ready);
            cached_ -= bin;
            cache_.erase(pick);
            live_[p] = Live{bytes, bin, cacheable};
            in_use_ += bytes;
            live_bin_ += bin;
        }
    }
    if (!p) {
        p = Backing(bin);
        std::lock_guard<std::mutex> lk(mu_);
        backing_ += bin;
        live_[p] = Live{bytes, bin, cacheable};
        in_use_ += bytes;
        live_bin_ += bin;
        if (Bins().debug)
            std::fprintf(stderr, "elx_pool[dev %d]: allocated new block %p (%zu bytes, bin %zu%s) for stream %p%s\n",
                         device_, p, bytes, bin, cacheable ? "" : ", uncached", (void*)s,
                         StreamTag(s, compute_, comm_));
    }
    // ELX_POOL_POISON=1 (debug): every block handed out is filled with 0xFF
    // bytes (NaN in every float type), so a read before the first write shows up
    static const bool poison = [] { const char* e = std::getenv("ELX_POOL_POISON"); return e && e[0] == '1'; }();
    if (poison) ELX_CHECK_HIP(hipMemsetAsync(p, 0xFF, bin, s));
    return p;
}

void Runtime::Free(void* p, hipStream_t s) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = live_.find(p);
    if (it == live_.end()) throw LogicError("elx_pool_free: pointer not from this pool");
    const Live l = it->second;
    if (!s) s = compute_;
    static const bool nocache = [] { const char* e = std::getenv("ELX_POOL_CACHE"); return e && e[0] == '0'; }();
    hipEvent_t ev = EventLocked();
    ELX_CHECK_HIP(hipEventRecord(ev, s));
    in_use_ -= l.requested;
    live_bin_ -= l.bin;
    live_.erase(it);
    if (nocache || !l.cacheable || cached_ + l.bin > max_cached_) {
        QueueReleaseLocked(p, l.bin, ev);  // over the cap / uncacheable: back to the driver
    } else {
        cache_.emplace(l.bin, Cached{p, s, ev});
        cached_ += l.bin;
        if (Bins().debug)
            std::fprintf(stderr, "elx_pool[dev %d]: returned block %p (%zu bytes) to the cache, stream %p%s, event %p "
                                 "(cached %zu)\n",
                         device_, p, l.bin, (void*)s, StreamTag(s, compute_, comm_), (void*)ev, cached_);
    }
}

void Runtime::Trim(size_t keep) {
    EnsureGPU();
    ELX_CHECK_HIP(hipDeviceSynchronize());
    {
        std::lock_guard<std::mutex> lk(mu_);
        ReleaseCachedLocked(keep);
    }
    WaitReleases();
}

void Runtime::SetMaxCached(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    max_cached_ = bytes;
    max_cached_set_ = true;
    if (gpu_ready_) ReleaseCachedLocked(bytes);
}

size_t Runtime::MaxCached() {
    std::lock_guard<std::mutex> lk(mu_);
    return max_cached_;
}

void Runtime::Stats(size_t& reserved, size_t& in_use) {
    std::lock_guard<std::mutex> lk(mu_);
    reserved = live_bin_ + cached_;
    in_use = in_use_;
}

size_t Runtime::BackingReserved() {
    WaitReleases();
    std::lock_guard<std::mutex> lk(mu_);
    return backing_;
}

namespace kern {
hipError_t workspace_alloc(void** p, size_t bytes, hipStream_t s) {
    try {
        *p = Runtime::Get().Alloc(bytes, s);
        return hipSuccess;
    } catch (...) {
        *p = nullptr;
        return hipErrorOutOfMemory;
    }
}
hipError_t workspace_free(void* p, hipStream_t s) {
    try {
        Runtime::Get().Free(p, s);
        return hipSuccess;
    } catch (...) {
        return hipErrorInvalidValue;
    }
}
}  // namespace kern

void StreamFence(hipStream_t from, hipStream_t to) {
    if (!from || !to || from == to) return;
    hipEvent_t ev;
    ELX_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ELX_CHECK_HIP(hipEventRecord(ev, from));
    ELX_CHECK_HIP(hipStreamWaitEvent(to, ev, 0));
    ELX_CHECK_HIP(hipEventDestroy(ev));
}

void Buffer::Reset(Device d, size_t bytes, hipStream_t s) {
    Release();
    dev_ = d;
    bytes_ = bytes;
    stream_ = s;
    owned_ = true;
    if (bytes == 0) return;
    if (d == Device::GPU) {
        if (!stream_) stream_ = Runtime::Get().ComputeStream();
        ptr_ = Runtime::Get().Alloc(bytes, stream_);
    } else {
        ptr_ = std::aligned_alloc(64, (bytes + 63) / 64 * 64);
        if (!ptr_) throw RuntimeError(Cat("host allocation of ", bytes, " bytes failed"));
    }
}

void Buffer::Release() {
    if (!ptr_) return;
    if (!owned_) {
        ptr_ = nullptr;
        bytes_ = 0;
        owned_ = true;
        return;
    }
    if (dev_ == Device::GPU) {
        try { Runtime::Get().Free(ptr_, stream_); } catch (...) {}
    } else {
        std::free(ptr_);
    }
    ptr_ = nullptr;
    bytes_ = 0;
}

}  // namespace elx
