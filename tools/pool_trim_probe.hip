// Do releases to the driver disturb memory that is still allocated?  Round-5
// probe behind the allocator's backing-store choice (runtime.hpp).
//
// A random alloc / free sequence keeps ~24 live blocks (4 KiB .. 32 MiB), each
// filled with its own id.  Frees happen only after a device synchronize (the
// block is idle), then, per mode, the memory goes back to the driver:
//   pool_trim  : hipFreeAsync to a hipMemPool (reuse policies off), synchronize,
//                hipMemPoolTrimTo(pool, 0)
//   pool_thr0  : the same pool with release threshold 0 and no explicit trim
//   pool_keep  : threshold max, never trimmed
//   malloc     : hipMalloc / hipFree
// After every step all live blocks are checked on the device (mismatch count)
// and on the host for overlapping address ranges.  Fill paths: a kernel, or a
// host-to-device copy from pinned memory (the copy engines' view of the fresh
// mapping against the compute units' view).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(3);                                                                          \
        }                                                                                          \
    } while (0)

__global__ void fill_u32(uint32_t* p, size_t n, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void check_u32(const uint32_t* p, size_t n, uint32_t v, unsigned long long* bad) {
    unsigned long long b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != v;
    if (b) atomicAdd(bad, b);
}

struct Blk { uint32_t* p; size_t bytes; uint32_t id; };

int main(int argc, char** argv) {
    const int steps = argc > 1 ? std::atoi(argv[1]) : 400;
    const std::string fillp = argc > 2 ? argv[2] : "kernel";  // kernel | h2d | h2d_pageable
    const bool h2d = fillp != "kernel";
    uint32_t* host = nullptr;
    const size_t host_words = (size_t(32) << 20) / 4 + 4096;
    std::vector<uint32_t> pageable;
    if (fillp == "h2d") CK(hipHostMalloc(&host, host_words * 4, hipHostMallocDefault));
    if (fillp == "h2d_pageable") { pageable.resize(host_words); host = pageable.data(); }
    const char* modes[] = {"pool_trim", "pool_thr0", "pool_keep", "malloc"};
    unsigned long long* bad;
    CK(hipMalloc(&bad, sizeof(*bad)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (const char* mode : modes) {
        const std::string m = mode;
        hipMemPool_t pool = nullptr;
        if (m != "malloc") {
            hipMemPoolProps props{};
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = 0;
            CK(hipMemPoolCreate(&pool, &props));
            uint64_t t = m == "pool_thr0" ? 0 : std::numeric_limits<uint64_t>::max();
            CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &t));
            int off = 0;
            CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseFollowEventDependencies, &off));
            CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowOpportunistic, &off));
            CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowInternalDependencies, &off));
        }
        std::mt19937 rng(12345);
        std::vector<Blk> live;
        uint32_t next_id = 1;
        unsigned long long corrupt_steps = 0, overlaps = 0, total_bad = 0;
        for (int step = 0; step < steps; ++step) {
            const bool do_alloc = live.size() < 8 || (live.size() < 40 && rng() % 2);
            if (do_alloc) {
                const int lg = 12 + rng() % 14;  // 4 KiB .. 32 MiB
                size_t bytes = (size_t(1) << lg) + (rng() % 4096) * 4;
                Blk b{nullptr, bytes, next_id++};
                if (m == "malloc") CK(hipMalloc(&b.p, bytes));
                else CK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&b.p), bytes, pool, s));
                if (h2d) {
                    CK(hipStreamSynchronize(s));
                    for (size_t w = 0; w < bytes / 4; ++w) host[w] = b.id;
                    CK(hipMemcpyAsync(b.p, host, bytes / 4 * 4, hipMemcpyHostToDevice, s));
                    CK(hipStreamSynchronize(s));
                } else {
                    fill_u32<<<256, 256, 0, s>>>(b.p, bytes / 4, b.id);
                }
                live.push_back(b);
            } else {
                const size_t i = rng() % live.size();
                Blk b = live[i];
                live.erase(live.begin() + i);
                CK(hipStreamSynchronize(s));  // idle before it leaves
                if (m == "malloc") {
                    CK(hipFree(b.p));
                } else {
                    CK(hipFreeAsync(b.p, s));
                    CK(hipStreamSynchronize(s));
                    if (m == "pool_trim") CK(hipMemPoolTrimTo(pool, 0));
                }
            }
            CK(hipMemsetAsync(bad, 0, sizeof(*bad), s));
            for (const Blk& b : live) check_u32<<<256, 256, 0, s>>>(b.p, b.bytes / 4, b.id, bad);
            unsigned long long h = 0;
            CK(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            if (h) { ++corrupt_steps; total_bad += h; }
            for (size_t a = 0; a < live.size(); ++a)
                for (size_t c = a + 1; c < live.size(); ++c) {
                    const char* pa = (const char*)live[a].p; const char* pc = (const char*)live[c].p;
                    if (pa < pc + live[c].bytes && pc < pa + live[a].bytes) ++overlaps;
                }
        }
        CK(hipStreamSynchronize(s));
        for (const Blk& b : live) {
            if (m == "malloc") CK(hipFree(b.p));
            else CK(hipFreeAsync(b.p, s));
        }
        CK(hipStreamSynchronize(s));
        if (pool) CK(hipMemPoolDestroy(pool));
        std::printf("fill=%s mode=%-9s steps=%d corrupt_steps=%llu bad_words=%llu overlapping_live_pairs=%llu %s\n",
                    fillp.c_str(), mode, steps, corrupt_steps, total_bad, overlaps, corrupt_steps || overlaps ? "CORRUPT" : "ok");
        std::fflush(stdout);
    }
    return 0;
}
