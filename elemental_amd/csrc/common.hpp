// Shared internals of libelemental_amd: error plumbing, dtype traits, HIP checks.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <sstream>
#include "../../include/elemental_amd.h"

namespace elx {

using Int = int64_t;

// Exception types mirroring the reference's (LogicError / RuntimeError /
// hydrogen::HIPError); the C-ABI maps them to ELX_ERR_* codes.
struct LogicError : std::logic_error { using std::logic_error::logic_error; };
struct RuntimeError : std::runtime_error { using std::runtime_error::runtime_error; };
struct HIPError : std::runtime_error { using std::runtime_error::runtime_error; };
struct CommError : std::runtime_error { using std::runtime_error::runtime_error; };
struct UnsupportedError : std::logic_error { using std::logic_error::logic_error; };
struct NoDeviceError : std::runtime_error { using std::runtime_error::runtime_error; };
// El::SingularMatrixException (include/El/core/environment/decl.hpp:209-214)
struct SingularMatrixError : std::runtime_error {
    SingularMatrixError() : std::runtime_error("Matrix was singular") {}
};

template <typename... Args>
std::string Cat(Args&&... args) {
    std::ostringstream os;
    (os << ... << args);
    return os.str();
}

#define ELX_CHECK_HIP(expr)                                                     \
    do {                                                                        \
        hipError_t _e = (expr);                                                 \
        if (_e != hipSuccess)                                                   \
            throw ::elx::HIPError(::elx::Cat("HIP error ", hipGetErrorName(_e), \
                                             " (", hipGetErrorString(_e),       \
                                             ") at ", __FILE__, ":", __LINE__,  \
                                             ": " #expr));                      \
    } while (0)

#define ELX_REQUIRE(cond, ...)                                                  \
    do { if (!(cond)) throw ::elx::LogicError(::elx::Cat(__VA_ARGS__)); } while (0)

void SetLastError(const std::string& msg);

// Run `f`, translating exceptions into C-ABI status codes.
template <typename F>
int Guard(F&& f) {
    try {
        f();
        return ELX_OK;
    } catch (const UnsupportedError& e) { SetLastError(e.what()); return ELX_ERR_UNSUPPORTED; }
    catch (const LogicError& e)         { SetLastError(e.what()); return ELX_ERR_LOGIC; }
    catch (const HIPError& e)           { SetLastError(e.what()); return ELX_ERR_HIP; }
    catch (const CommError& e)          { SetLastError(e.what()); return ELX_ERR_COMM; }
    catch (const NoDeviceError& e)      { SetLastError(e.what()); return ELX_ERR_NO_DEVICE; }
    catch (const SingularMatrixError& e) { SetLastError(e.what()); return ELX_ERR_SINGULAR; }
    catch (const std::logic_error& e)   { SetLastError(e.what()); return ELX_ERR_LOGIC; }
    catch (const std::exception& e)     { SetLastError(e.what()); return ELX_ERR_RUNTIME; }
    catch (...)                         { SetLastError("unknown exception"); return ELX_ERR_RUNTIME; }
}

// F32..BF16: matrix element types; I32 / I64 / U8: communication buffers only
// (ToCommDType), never a DistMatrix or kernel type (ToDType rejects them)
enum class DType : int {
    F32 = ELX_F32, F64 = ELX_F64, F16 = ELX_F16, BF16 = ELX_BF16, I32 = ELX_I32, I64 = ELX_I64, U8 = ELX_U8
};

inline size_t DTypeSize(DType t) {
    switch (t) {
    case DType::F32: return 4;
    case DType::F64: return 8;
    case DType::F16: return 2;
    case DType::BF16: return 2;
    case DType::I32: return 4;
    case DType::I64: return 8;
    case DType::U8: return 1;
    }
    throw LogicError("bad dtype");
}
inline DType ToDType(int t) {
    if (t < 0 || t > 3) throw LogicError(Cat("invalid dtype ", t));
    return static_cast<DType>(t);
}
inline DType ToCommDType(int t) {
    if (t < 0 || t > ELX_U8) throw LogicError(Cat("invalid dtype ", t, " for a collective"));
    return static_cast<DType>(t);
}
inline const char* DTypeName(DType t) {
    switch (t) {
    case DType::F32: return "f32";
    case DType::F64: return "f64";
    case DType::F16: return "f16";
    case DType::BF16: return "bf16";
    case DType::I32: return "i32";
    case DType::I64: return "i64";
    case DType::U8: return "u8";
    }
    return "?";
}

// Host-side 16-bit float conversions (round-to-nearest-even), used by the CPU
// device path and by scalar conversion at the boundary.
inline float HalfToFloat(uint16_t h) {
    uint32_t sign = (h & 0x8000u) << 16, exp = (h >> 10) & 0x1f, man = h & 0x3ff;
    uint32_t f;
    if (exp == 0) {
        if (man == 0) f = sign;
        else {  // subnormal
            int e = -1;
            do { ++e; man <<= 1; } while (!(man & 0x400));
            f = sign | ((127 - 15 - e) << 23) | ((man & 0x3ff) << 13);
        }
    } else if (exp == 31) f = sign | 0x7f800000u | (man << 13);
    else f = sign | ((exp - 15 + 127) << 23) | (man << 13);
    float out; std::memcpy(&out, &f, 4); return out;
}
inline uint16_t FloatToHalf(float x) {
    uint32_t f; std::memcpy(&f, &x, 4);
    uint32_t sign = (f >> 16) & 0x8000u;
    uint32_t absf = f & 0x7fffffffu;
    if (absf >= 0x7f800000u)  // inf / nan
        return static_cast<uint16_t>(sign | 0x7c00u | (absf > 0x7f800000u ? 0x200u : 0));
    if (absf >= 0x477ff000u) return static_cast<uint16_t>(sign | 0x7c00u);  // overflow -> inf
    if (absf < 0x33000001u) return static_cast<uint16_t>(sign);            // underflow -> 0
    int e = static_cast<int>(absf >> 23);
    uint32_t man = (absf & 0x7fffffu) | 0x800000u;
    if (e < 113) {  // subnormal half: m = round(man * 2^(e-126))
        const int shift = 126 - e;  // 14..24
        uint32_t m = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (m & 1))) ++m;
        return static_cast<uint16_t>(sign | m);
    }
    uint32_t h = ((e - 112) << 10) | ((man >> 13) & 0x3ff);
    uint32_t rem = man & 0x1fff;
    if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) ++h;
    return static_cast<uint16_t>(sign | h);
}
inline float BF16ToFloat(uint16_t b) {
    uint32_t f = static_cast<uint32_t>(b) << 16; float out; std::memcpy(&out, &f, 4); return out;
}
inline uint16_t FloatToBF16(float x) {
    uint32_t f; std::memcpy(&f, &x, 4);
    if ((f & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((f >> 16) | 0x40);  // keep NaN
    uint32_t r = f + 0x7fffu + ((f >> 16) & 1u);
    return static_cast<uint16_t>(r >> 16);
}

}  // namespace elx
