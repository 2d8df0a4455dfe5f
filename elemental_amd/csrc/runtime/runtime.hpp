// Device runtime: device selection, the library's streams, and the
// hipMallocAsync memory pool that replaces the reference's hipCUB
// CachingDeviceAllocator (src/core/imports/cub.cpp:1-75; El::Memory mode 1,
// include/El/core/Memory/impl.hpp:113-187).
#pragma once
#include "../common.hpp"
#include <mutex>
#include <unordered_map>

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

    // Stream-ordered pool allocation (hipMallocFromPoolAsync / hipFreeAsync).
    void* Alloc(size_t bytes, hipStream_t s);
    void Free(void* p, hipStream_t s);
    void Trim(size_t keep);
    void Stats(size_t& reserved, size_t& in_use);

private:
    Runtime() = default;
    std::mutex mu_;
    bool gpu_ready_ = false;
    int device_ = -1;
    int reserved_cus_ = 0;
    hipStream_t compute_ = nullptr, comm_ = nullptr;
    hipMemPool_t pool_ = nullptr;
    std::unordered_map<void*, size_t> live_;
    size_t in_use_ = 0;
};

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
