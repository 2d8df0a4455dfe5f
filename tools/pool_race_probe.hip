// Driver-level probe of stream-ordered pool reuse (round-5 hunt for round 4's
// intermittent wrong GEMMs under a release threshold of 0).
//
// Each case: X (one block from a hipMemPool) is filled with 1.0, then a reader
// kernel on stream R spins for `spin_ms` and writes Y = X + 10.  X is freed
// (hipFreeAsync) on stream F after the reader was queued, ordered or not as the
// case says, and a new block of the same size is allocated on stream N and filled
// with 2.0.  A correct runtime never hands X to N before the reader is done when
// N is not ordered after the free, so Y must be all 11 (12: X was handed to N
// and refilled before the reader ran; 10: X read as zero pages; 0: no write).
//   pools: release threshold 0 or max, the driver's reuse policies (follow event
//   dependencies, opportunistic, internal dependencies) on or off; cases:
//    same    : R = F = N (stream order: always legal, Y must be 1)
//    cross   : R = F, N another stream, no dependency (opportunistic reuse is
//              legal only after the free completes)
//    cross_sync : as cross, with hipStreamSynchronize(N) between free and alloc
//    stale_dep  : N waits on an event of F recorded BEFORE the reader and the free
//              (follow-event-dependencies must not treat that as covering the free)
//    dep     : N waits on an event of F recorded AFTER the free (reuse legal, the
//              fill waits for the reader: Y must be 1)
//    dep_hostsync : as dep, and the host waits for that event before the alloc
//    wait_only : no free at all: N waits on the event, then fills X itself (the
//              plain cross-stream ordering a caching allocator relies on)
// Prints one line per case: pointer reused?, Y correct?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(3);                                                            \
        }                                                                            \
    } while (0)

__global__ void spin_copy(const double* x, double* y, size_t n, unsigned long long ticks) {
    if (ticks) {
        const unsigned long long t0 = wall_clock64();
        while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    }
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) y[i] = x[i] + 10.0;
}

__global__ void fill(double* x, size_t n, double v) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) x[i] = v;
}

int main(int argc, char** argv) {
    const size_t n = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (16u << 20)) / sizeof(double);
    const double spin_ms = argc > 2 ? std::atof(argv[2]) : 100.0;
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
    const unsigned long long ticks = (unsigned long long)(spin_ms * clk_khz);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    double* Y;
    CK(hipMalloc(&Y, n * sizeof(double)));
    std::vector<double> h(n);
    int bad_total = 0;
    for (int cfg = 0; cfg < 4; ++cfg) {
        const int thr = cfg & 1, reuse = cfg < 2;
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = 0;
        hipMemPool_t pool;
        CK(hipMemPoolCreate(&pool, &props));
        uint64_t t = thr == 0 ? 0 : std::numeric_limits<uint64_t>::max();
        CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &t));
        int on = reuse;
        CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseFollowEventDependencies, &on));
        CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowOpportunistic, &on));
        CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowInternalDependencies, &on));
        for (const char* c : {"same", "cross", "cross_sync", "stale_dep", "dep", "dep_hostsync", "wait_only"}) {
            const std::string cs = c;
            hipStream_t F = s1, R = s1, N = cs == "same" ? s1 : s2;
            CK(hipDeviceSynchronize());
            CK(hipMemsetAsync(Y, 0, n * sizeof(double), F));
            CK(hipStreamSynchronize(F));
            double* X = nullptr;
            CK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&X), n * sizeof(double), pool, F));
            fill<<<1024, 256, 0, F>>>(X, n, 1.0);
            CK(hipStreamSynchronize(F));
            hipEvent_t early, late;
            CK(hipEventCreateWithFlags(&early, hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&late, hipEventDisableTiming));
            CK(hipEventRecord(early, F));
            spin_copy<<<1024, 256, 0, R>>>(X, Y, n, ticks);
            const bool wait_only = cs == "wait_only";
            if (!wait_only) CK(hipFreeAsync(X, F));
            CK(hipEventRecord(late, F));
            if (cs == "cross_sync") CK(hipStreamSynchronize(N));
            if (cs == "stale_dep") CK(hipStreamWaitEvent(N, early, 0));
            if (cs == "dep" || cs == "dep_hostsync" || wait_only) CK(hipStreamWaitEvent(N, late, 0));
            if (cs == "dep_hostsync") CK(hipEventSynchronize(late));
            double* X2 = X;
            if (!wait_only) CK(hipMallocFromPoolAsync(reinterpret_cast<void**>(&X2), n * sizeof(double), pool, N));
            fill<<<1024, 256, 0, N>>>(X2, n, 2.0);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), Y, n * sizeof(double), hipMemcpyDeviceToHost));
            size_t wrong = 0, v12 = 0, v10 = 0, v0 = 0;
            for (double v : h) { wrong += v != 11.0; v12 += v == 12.0; v10 += v == 10.0; v0 += v == 0.0; }
            std::printf("threshold=%s reuse_policies=%s case=%-12s reused=%d wrong=%zu/%zu (12: %zu, 10: %zu, 0: %zu) %s\n",
                        thr == 0 ? "0" : "max", reuse ? "on " : "off", c, X2 == X, wrong, n, v12, v10, v0,
                        wrong ? "CORRUPT" : "ok");
            bad_total += wrong != 0;
            CK(hipFreeAsync(X2, N));
            CK(hipDeviceSynchronize());
            CK(hipEventDestroy(early));
            CK(hipEventDestroy(late));
        }
        CK(hipMemPoolDestroy(pool));
    }
    std::printf("cases corrupt: %d\n", bad_total);
    return 0;
}
