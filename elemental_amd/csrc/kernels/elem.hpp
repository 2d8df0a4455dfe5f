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
    static __host__ __device__ __forceinline__ compute load(double x) { return x; }
    static __host__ __device__ __forceinline__ double store(compute x) { return x; }
};
template <> struct Elem<float> {
    using storage = float;
    using compute = float;
    static __host__ __device__ __forceinline__ compute load(float x) { return x; }
    static __host__ __device__ __forceinline__ float store(compute x) { return x; }
};
template <> struct Elem<f16_t> {
    using storage = uint16_t;
    using compute = float;
    static __host__ __device__ __forceinline__ compute load(uint16_t x) {
        return (float)__builtin_bit_cast(_Float16, x);
    }
    static __host__ __device__ __forceinline__ uint16_t store(compute x) {
        return __builtin_bit_cast(uint16_t, (_Float16)x);  // RNE
    }
};
template <> struct Elem<bf16_t> {
    using storage = uint16_t;
    using compute = float;
    static __host__ __device__ __forceinline__ compute load(uint16_t x) {
        return __builtin_bit_cast(float, (uint32_t)x << 16);
    }
    static __host__ __device__ __forceinline__ uint16_t store(compute x) {
        const uint32_t f = __builtin_bit_cast(uint32_t, x);
        if ((f & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((f >> 16) | 0x40);  // NaN stays NaN
        return (uint16_t)((f + 0x7fffu + ((f >> 16) & 1u)) >> 16);                 // RNE
    }
};

// Type-converting element copy, the reference's Copy_GPU_impl<SrcT,DestT>
// (src/hydrogen/blas/gpu/Copy.cu:13-21: `dest = src`, a C++ conversion): the
// exact source value is rounded ONCE, to nearest-even, into the destination
// type.  f64 -> bf16 goes through a round-to-odd f32 (24 >= 8 + 2 significand
// bits, so the second rounding is the correctly rounded result).
__host__ __device__ __forceinline__ float round_to_odd_f32(double d) {
    const float f = (float)d;
    const double b = (double)f;
    if (b == d || b != b) return f;  // exact, or NaN
    uint32_t u = __builtin_bit_cast(uint32_t, f);
    if ((b < 0 ? -b : b) > (d < 0 ? -d : d)) u -= 1;  // rounded away from zero: truncate instead
    return __builtin_bit_cast(float, u | 1u);          // sticky bit
}
template <typename TD> struct Narrow;
template <> struct Narrow<double> {
    static __host__ __device__ __forceinline__ double from(double v) { return v; }
    static __host__ __device__ __forceinline__ double from(float v) { return v; }
};
template <> struct Narrow<float> {
    static __host__ __device__ __forceinline__ float from(double v) { return (float)v; }
    static __host__ __device__ __forceinline__ float from(float v) { return v; }
};
template <> struct Narrow<f16_t> {
    static __host__ __device__ __forceinline__ uint16_t from(double v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }
    static __host__ __device__ __forceinline__ uint16_t from(float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }
};
template <> struct Narrow<bf16_t> {
    static __host__ __device__ __forceinline__ uint16_t from(double v) { return Elem<bf16_t>::store(round_to_odd_f32(v)); }
    static __host__ __device__ __forceinline__ uint16_t from(float v) { return Elem<bf16_t>::store(v); }
};
template <typename TS, typename TD>
__host__ __device__ __forceinline__ typename Elem<TD>::storage convert_elem(typename Elem<TS>::storage x) {
    return Narrow<TD>::from(Elem<TS>::load(x));
}

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
