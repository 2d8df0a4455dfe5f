// Device runtime: device selection, the library's streams, and the caching
// device allocator that replaces the reference's hipCUB CachingDeviceAllocator
// (src/core/imports/cub.cpp:1-75; El::Memory mode 1,
// include/El/core/Memory/impl.hpp:113-187).
//
// Allocator contract (what `elx_pool_*` promise):
//  * sizes are rounded to bins and a freed block is cached under its bin; a
//    request is served from a cached block of exactly its bin.  Default bins:
//    powers of two from 512 B to 1 MiB (at most 2x slack, as CUB's growth 2),
//    then eight per octave (<= 12.5 % slack).  H_CUB_BIN_GROWTH / H_CUB_MIN_BIN /
//    H_CUB_MAX_BIN (src/core/imports/cub.cpp:21-35) switch to CUB's geometric
//    bins growth^k, k >= min_bin; a request above growth^max_bin gets a block of
//    its own size (512-B granules) that is never cached;
//  * reuse is stream-ordered without a host sync: a block freed on stream F and
//    handed out on stream S makes S wait on the event recorded on F at the free
//    (CUB's DeviceFree/DeviceAllocate ready-event rule);
//  * therefore a repeated alloc/free pattern (the SUMMA panel slots, any
//    steady-state loop) reserves nothing new after its first pass, whichever
//    streams it allocates and frees on;
//  * cached bytes are capped by H_CUB_MAX_CACHED_SIZE / ELX_POOL_MAX_CACHED /
//    elx_pool_set_max_cached (default: unbounded, as CUB's INVALID_SIZE); a
//    block that does not fit under the cap, an uncacheable block and, with
//    ELX_POOL_CACHE=0, every block leaves the allocator: it is queued for the
//    allocator's release thread, which waits for the free's event and hipFrees
//    it, so the memory returns to the driver as under CUB's synchronous
//    cudaFree, but the freeing thread returns at once and no event wait or
//    hipFree ever runs under the allocator's lock (a free never stalls the host
//    or another thread's Alloc / Free); Trim, elx_pool_backing_reserved and an
//    out-of-memory retry wait for the queued releases;
//  * a request no bin can hold (its rounding overflows) fails with
//    out-of-memory;
//  * the backing store is hipMalloc / hipFree, as under hipCUB's
//    CachingDeviceAllocator (cudaMalloc / cudaFree); a block goes back to the
//    driver only once the host has seen its free's event complete.  Not the
//    driver's stream-ordered pool (hipMallocFromPoolAsync): round 5 measured it
//    on this ROCm (tools/pool_race_probe.hip, tools/pool_trim_probe.hip,
//    profiles/r05_pool_race_probe.log, profiles/r05_pool_trim_probe.log): a hipFreeAsync'd block whose earlier work
//    is still queued is re-backed or handed out before that work runs; with
//    follow-event-dependencies on, a stream that once waited on an OLDER event
//    of the freeing stream receives the block at once; and even with every
//    free idle, single-stream and the release threshold at max, allocations
//    after frees overwrote blocks that were still live (hipMalloc: clean on the
//    same sequence).  Every device scratch of the library (the split-k
//    partials too, kern::workspace_alloc) comes from this allocator; a failed
//    backing allocation releases the cache and retries once before reporting
//    out-of-memory;
//  * H_CUB_DEBUG=1 (cub.cpp:45-50) logs every allocation, reuse (with the
//    stream it was freed on and the event the new stream waits on), cache
//    return and release to stderr.
#pragma once
#include "../common.hpp"
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace elx {

enum class Device : int { CPU = ELX_DEVICE_CPU, GPU = ELX_DEVICE_GPU };

class Runtime {
public:
    static Runtime& Get();
    // Initialise HIP on first GPU use; throws NoDeviceError without a device.
    void EnsureGPU();
    bool GPUInitialized() const { return gpu_ready_; }
    int DeviceId() const { return device_; }
    void SetDevice(int dev);
    hipStream_t ComputeStream() { EnsureGPU(); return compute_; }
    hipStream_t CommStream() { EnsureGPU(); return comm_; }
    hipStream_t Resolve(void* s) { return s ? static_cast<hipStream_t>(s) : ComputeStream(); }
    // CUs masked off the compute stream for communication kernels (ELX_COMM_CUS)
    int ReservedCUs() { EnsureGPU(); return reserved_cus_; }

    // Stream-ordered caching allocation (contract above).
    void* Alloc(size_t bytes, hipStream_t s);
    void Free(void* p, hipStream_t s);
    void Trim(size_t keep);
    // reserved = live + cached bin bytes; in_use = requested bytes still live
    void Stats(size_t& reserved, size_t& in_use);
    // bytes held from the driver (hipMalloc'd, not yet hipFree'd) once the
    // queued releases have landed (waits for them): live + cached blocks; 0
    // before the first GPU use
    size_t BackingReserved();
    void SetMaxCached(size_t bytes);
    size_t MaxCached();
    // the bin a request of `bytes` is served from; `cacheable` = false for
    // requests above H_CUB_MAX_BIN's bin (own-size blocks, never cached)
    static size_t BinBytes(size_t bytes, bool* cacheable = nullptr);

private:
    struct Cached { void* p; hipStream_t stream; hipEvent_t ready; };
    struct Live { size_t requested, bin; bool cacheable; };
    struct Pending { void* p; size_t bin; hipEvent_t ready; };
    Runtime() = default;
    // hipMalloc a new block (without mu_; on out-of-memory: release the cache,
    // wait for the releases, retry once)
    void* Backing(size_t bin);
    void ReleaseCachedLocked(size_t keep);
    // hand a block to the release thread: hipFree'd once `ready` completed
    void QueueReleaseLocked(void* p, size_t bin, hipEvent_t ready);
    void ReleaseLoop();
    void WaitReleases();  // until every queued release landed (takes mu_)
    void StopReleaser();  // at exit: drain the queue, join the thread
    hipEvent_t EventLocked();
    std::mutex mu_;
    std::condition_variable release_cv_, idle_cv_;
    std::deque<Pending> pending_;
    std::thread releaser_;
    bool releaser_started_ = false, releasing_ = false, stop_ = false;
    bool gpu_ready_ = false;
    int device_ = -1;
    int reserved_cus_ = 0;
    hipStream_t compute_ = nullptr, comm_ = nullptr;
    std::unordered_map<void*, Live> live_;
    std::multimap<size_t, Cached> cache_;  // bin bytes -> freed block
    std::vector<hipEvent_t> spare_events_;
    size_t in_use_ = 0, live_bin_ = 0, cached_ = 0, backing_ = 0;
    size_t max_cached_ = ~size_t(0);
    bool max_cached_set_ = false;
};

// Stream `to` waits for the work queued on `from` so far (no-op when equal or null).
void StreamFence(hipStream_t from, hipStream_t to);

// RAII device or host buffer.  GPU memory comes from the pool on `stream` and is
// returned to it on that stream (stream-ordered reuse, no device sync).
class Buffer {
public:
    Buffer() = default;
    Buffer(Device d, size_t bytes, hipStream_t s = nullptr) { Reset(d, bytes, s); }
    ~Buffer() { Release(); }
    Buffer(const Buffer&) = delete;
    Buffer& operator=(const Buffer&) = delete;
    Buffer(Buffer&& o) noexcept { *this = std::move(o); }
    Buffer& operator=(Buffer&& o) noexcept {
        if (this != &o) {
            Release();
            dev_ = o.dev_; ptr_ = o.ptr_; bytes_ = o.bytes_; stream_ = o.stream_; owned_ = o.owned_;
            o.ptr_ = nullptr; o.bytes_ = 0;
        }
        return *this;
    }
    void Reset(Device d, size_t bytes, hipStream_t s = nullptr);
    // non-owning: caller storage (DistMatrix::Attach); never freed here
    void Wrap(Device d, void* ptr, size_t bytes) { Release(); dev_ = d; ptr_ = ptr; bytes_ = bytes; owned_ = false; }
    void Release();
    // release on `s` from now on (the caller has ordered s after the old stream)
    void Rebind(hipStream_t s) { stream_ = s; }
    void* data() const { return ptr_; }
    // the stream the block is returned to the pool on (GPU blocks we own;
    // nullptr for host memory and wrapped caller storage)
    hipStream_t stream() const { return owned_ && dev_ == Device::GPU ? stream_ : nullptr; }
    size_t bytes() const { return bytes_; }
    Device device() const { return dev_; }

private:
    Device dev_ = Device::CPU;
    void* ptr_ = nullptr;
    size_t bytes_ = 0;
    hipStream_t stream_ = nullptr;
    bool owned_ = true;
};

}  // namespace elx
