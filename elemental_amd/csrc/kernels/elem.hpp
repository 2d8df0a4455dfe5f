// Element-type helpers shared by the HIP kernels: 16-bit types travel as
// uint16_t storage and compute in f32; f32/f64 compute natively.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace elx {
namespace kern {

struct f16_t { uint16_t bits; };
struct bf16_t { uint16_t bits; };

template <typename T> struct Elem;
template <> struct Elem<double> {
    using storage = double;
    using compute = double;
    static __device__ __forceinline__ compute load(double x) { return x; }
    static __device__ __forceinline__ double store(compute x) { return x; }
};
template <> struct Elem<float> {
    using storage = float;
    using compute = float;
    static __device__ __forceinline__ compute load(float x) { return x; }
    static __device__ __forceinline__ float store(compute x) { return x; }
};
template <> struct Elem<f16_t> {
    using storage = uint16_t;
    using compute = float;
    static __device__ __forceinline__ compute load(uint16_t x) {
        return (float)__builtin_bit_cast(_Float16, x);
    }
    static __device__ __forceinline__ uint16_t store(compute x) {
        return __builtin_bit_cast(uint16_t, (_Float16)x);  // RNE
    }
};
template <> struct Elem<bf16_t> {
    using storage = uint16_t;
    using compute = float;
    static __device__ __forceinline__ compute load(uint16_t x) {
        return __builtin_bit_cast(float, (uint32_t)x << 16);
    }
    static __device__ __forceinline__ uint16_t store(compute x) {
        const uint32_t f = __builtin_bit_cast(uint32_t, x);
        if ((f & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((f >> 16) | 0x40);  // NaN stays NaN
        return (uint16_t)((f + 0x7fffu + ((f >> 16) & 1u)) >> 16);                 // RNE
    }
};

// Counter-based hash for grid-independent synthetic inputs (mirrored bit-for-bit
// by oracle/oracle.c:orc_hash_value and elx::HashValue on the host).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ double hash_unit(uint64_t seed, int64_t i, int64_t j) {
    uint64_t h = splitmix64(seed ^ splitmix64((uint64_t)i * 0xD1B54A32D192ED03ull + 0x1234567ull));
    h = splitmix64(h ^ ((uint64_t)j * 0xA0761D6478BD642Full));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);  // [0,1)
}

}  // namespace kern
}  // namespace elx
