#include "runtime.hpp"
#include <algorithm>
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
    ELX_CHECK_HIP(hipDeviceGetDefaultMemPool(&pool_, device_));
    uint64_t thresh = std::numeric_limits<uint64_t>::max();  // keep freed blocks cached
    ELX_CHECK_HIP(hipMemPoolSetAttribute(pool_, hipMemPoolAttrReleaseThreshold, &thresh));
    gpu_ready_ = true;
}

void* Runtime::Alloc(size_t bytes, hipStream_t s) {
    EnsureGPU();
    if (bytes == 0) return nullptr;
    void* p = nullptr;
    ELX_CHECK_HIP(hipMallocFromPoolAsync(&p, bytes, pool_, s ? s : compute_));
    std::lock_guard<std::mutex> lk(mu_);
    live_[p] = bytes;
    in_use_ += bytes;
    return p;
}

void Runtime::Free(void* p, hipStream_t s) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = live_.find(p);
        if (it == live_.end()) throw LogicError("elx_pool_free: pointer not from this pool");
        in_use_ -= it->second;
        live_.erase(it);
    }
    ELX_CHECK_HIP(hipFreeAsync(p, s ? s : compute_));
}

void Runtime::Trim(size_t keep) {
    EnsureGPU();
    ELX_CHECK_HIP(hipDeviceSynchronize());
    ELX_CHECK_HIP(hipMemPoolTrimTo(pool_, keep));
}

void Runtime::Stats(size_t& reserved, size_t& in_use) {
    reserved = 0;
    if (gpu_ready_) {
        uint64_t r = 0;
        if (hipMemPoolGetAttribute(pool_, hipMemPoolAttrReservedMemCurrent, &r) == hipSuccess)
            reserved = r;
    }
    std::lock_guard<std::mutex> lk(mu_);
    in_use = in_use_;
}

void Buffer::Reset(Device d, size_t bytes, hipStream_t s) {
    Release();
    dev_ = d;
    bytes_ = bytes;
    stream_ = s;
    owned_ = true;
    if (bytes == 0) return;
    if (d == Device::GPU) {
        ptr_ = Runtime::Get().Alloc(bytes, s);
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
