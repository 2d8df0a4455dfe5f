// Distributed matrix file I/O.  The reference gathers to [CIRC,CIRC] and the
// root writes (Write.cpp:70-86); reading is either sequential (root reads,
// Copy scatters) or every rank seeks its own entries (Read/Binary.hpp:40-95).
// Here both directions go through [CIRC,CIRC] on the host of the root (one
// redistribution, one contiguous file access); the element values are moved,
// never recomputed, so the files are byte-identical to the reference's.
#include "io.hpp"
#include "redist.hpp"
#include <cstdio>
#include <cstring>
#include <vector>

namespace elx {

namespace {

std::string Extension(int format) { return format == FILE_BINARY ? "bin" : "dat"; }  // File.cpp:34-35

int Detect(const std::string& filename) {  // DetectFormat (File.cpp): by extension
    const auto dot = filename.rfind('.');
    const std::string ext = dot == std::string::npos ? "" : filename.substr(dot + 1);
    if (ext == "bin") return FILE_BINARY;
    if (ext == "dat") return FILE_BINARY_FLAT;
    throw RuntimeError(Cat("Could not detect the format of ", filename));
}

void CheckFormat(int format, int intBytes) {
    if (format != FILE_BINARY && format != FILE_BINARY_FLAT) throw LogicError("Invalid file format");
    ELX_REQUIRE(intBytes == 4 || intBytes == 8, "sizeof(Int) must be 4 or 8, got ", intBytes);
}

// element size on file: 16-bit types are widened to float
size_t FileElem(DType t) { return t == DType::F16 || t == DType::BF16 ? 4 : DTypeSize(t); }

void ToFile(DType t, const void* src, void* dst, size_t count) {
    if (t == DType::F16 || t == DType::BF16) {
        const uint16_t* s = static_cast<const uint16_t*>(src);
        float* d = static_cast<float*>(dst);
        for (size_t i = 0; i < count; ++i) d[i] = t == DType::F16 ? HalfToFloat(s[i]) : BF16ToFloat(s[i]);
    } else {
        std::memcpy(dst, src, count * DTypeSize(t));
    }
}

void FromFile(DType t, const void* src, void* dst, size_t count) {
    if (t == DType::F16 || t == DType::BF16) {
        const float* s = static_cast<const float*>(src);
        uint16_t* d = static_cast<uint16_t*>(dst);
        for (size_t i = 0; i < count; ++i) d[i] = t == DType::F16 ? FloatToHalf(s[i]) : FloatToBF16(s[i]);
    } else {
        std::memcpy(dst, src, count * DTypeSize(t));
    }
}

struct File {
    FILE* f = nullptr;
    File(const std::string& name, const char* mode) : f(std::fopen(name.c_str(), mode)) {
        if (!f) throw RuntimeError(Cat("Could not open ", name));
    }
    ~File() { if (f) std::fclose(f); }
};

}  // namespace

void Write(const DistMatrix& A, const std::string& basename, int format, int intBytes) {
    CheckFormat(format, intBytes);
    const Int m = A.Height(), n = A.Width();
    // gather to VC rank 0 (every rank takes part in the redistribution), on the
    // device the grid's communicator moves data on
    DistMatrix R(A.GridPtr(), A.Type(), Dist::CIRC, Dist::CIRC, A.G().CommDevice(), 0);
    Copy(A, R);
    if (A.G().VCRank() != 0) return;
    std::vector<unsigned char> local(static_cast<size_t>(m * n) * A.ElemSize());
    if (m > 0 && n > 0) R.GetLocal(local.data(), m);
    std::vector<unsigned char> data(static_cast<size_t>(m * n) * FileElem(A.Type()));
    ToFile(A.Type(), local.data(), data.data(), static_cast<size_t>(m * n));
    File file(basename + "." + Extension(format), "wb");
    if (format == FILE_BINARY) {
        const int64_t h64 = m, w64 = n;
        const int32_t h32 = static_cast<int32_t>(m), w32 = static_cast<int32_t>(n);
        std::fwrite(intBytes == 8 ? (const void*)&h64 : (const void*)&h32, intBytes, 1, file.f);
        std::fwrite(intBytes == 8 ? (const void*)&w64 : (const void*)&w32, intBytes, 1, file.f);
    }
    if (!data.empty() && std::fwrite(data.data(), 1, data.size(), file.f) != data.size())
        throw RuntimeError(Cat("short write to ", basename));
}

void Read(DistMatrix& A, const std::string& filename, int format, int intBytes) {
    if (format == FILE_AUTO) format = Detect(filename);
    CheckFormat(format, intBytes);
    // every rank checks the file (same answer, same exception everywhere)
    File file(filename, "rb");
    std::fseek(file.f, 0, SEEK_END);
    const int64_t bytes = std::ftell(file.f);
    std::fseek(file.f, 0, SEEK_SET);
    Int m = A.Height(), n = A.Width();
    int64_t meta = 0;
    if (format == FILE_BINARY) {
        int64_t h = 0, w = 0;
        int32_t h32 = 0, w32 = 0;
        const bool ok = intBytes == 8 ? std::fread(&h, 8, 1, file.f) == 1 && std::fread(&w, 8, 1, file.f) == 1
                                      : std::fread(&h32, 4, 1, file.f) == 1 && std::fread(&w32, 4, 1, file.f) == 1;
        if (!ok) throw RuntimeError(Cat("Could not read the header of ", filename));
        m = intBytes == 8 ? h : h32;
        n = intBytes == 8 ? w : w32;
        meta = 2 * intBytes;
    }
    const int64_t expect = meta + m * n * static_cast<int64_t>(FileElem(A.Type()));
    if (bytes != expect) throw RuntimeError(Cat("Expected file to be ", expect, " bytes but found ", bytes));
    DistMatrix R(A.GridPtr(), A.Type(), Dist::CIRC, Dist::CIRC, A.G().CommDevice(), 0);
    R.Resize(m, n);
    // only the root reads the body: its success is broadcast before the
    // collective scatter, so a failure raises on every rank instead of leaving
    // the others waiting in the redistribution
    std::string err;
    if (A.G().VCRank() == 0 && m > 0 && n > 0) {
        try {
            std::vector<unsigned char> data(static_cast<size_t>(m * n) * FileElem(A.Type()));
            if (std::fread(data.data(), 1, data.size(), file.f) != data.size())
                throw RuntimeError(Cat("short read from ", filename));
            std::vector<unsigned char> local(static_cast<size_t>(m * n) * A.ElemSize());
            FromFile(A.Type(), data.data(), local.data(), static_cast<size_t>(m * n));
            R.SetLocal(local.data(), m);
        } catch (const std::exception& e) {
            err = e.what();
            if (err.empty()) err = "read failed";
        }
    }
    if (GridBcast(A.G(), err.empty() ? 1.0 : 0.0, 0) == 0.0)
        throw RuntimeError(err.empty() ? Cat("short read from ", filename, " on the root rank") : err);
    Copy(R, A);
}

}  // namespace elx
