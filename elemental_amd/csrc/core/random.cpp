// El's random test inputs: the process-global std::mt19937 (seeded
// (secs << 16) | rank, secs = 21 when deterministic: src/core/random.cpp:24-35)
// and Uniform / MakeUniform (src/matrices/random/independent/Uniform.cpp:18-66):
// RedundantRank 0 of each redundant group draws SampleBall(center, radius) =
// uniform_real_distribution(center - radius, center + radius)
// (include/El/core/random/impl.hpp:113-139,230-231) for every local entry in
// column-major order (EntrywiseFill, include/El/blas_like/level1/EntrywiseFill.hpp:20-35),
// the GPU copy is that host fill moved to the device, and the result is
// broadcast over the redundant group.  The same <random> of the same libstdc++
// gives the reference's values bit for bit on the same grid.
#include "random.hpp"
#include "exec.hpp"
#include <ctime>
#include <random>
#include <vector>

namespace elx {

namespace {
std::mt19937& Generator() {
    static std::mt19937 gen;
    return gen;
}

// The ranks holding the same local block as this one: the dimension(s) of the
// grid that neither distribution covers (ElementalMatrix RedundantComm).
Comm* RedundantComm(const DistMatrix& A) {
    const Grid& g = A.G();
    // [MD,*], [*,MD], [CIRC,CIRC]: self (MD_STAR.cpp:170-171, CIRC_CIRC.cpp:54-55)
    if (A.ColDist() == Dist::MD || A.RowDist() == Dist::MD || A.ColDist() == Dist::CIRC) return nullptr;
    auto covers_mc = [](Dist d) { return d == Dist::MC || d == Dist::VC || d == Dist::VR; };
    auto covers_mr = [](Dist d) { return d == Dist::MR || d == Dist::VC || d == Dist::VR; };
    const bool mc = covers_mc(A.ColDist()) || covers_mc(A.RowDist());
    const bool mr = covers_mr(A.ColDist()) || covers_mr(A.RowDist());
    if (mc && mr) return nullptr;
    if (mc) return &g.MR();   // same grid row: differ only in mr
    if (mr) return &g.MC();
    return &g.VC();           // [STAR,STAR]: everyone
}
}  // namespace

void InitializeRandom(bool deterministic, int worldRank) {
    const long secs = deterministic ? 21 : static_cast<long>(time(nullptr));
    const long seed = (secs << 16) | (worldRank & 0xFFFF);
    Generator().seed(static_cast<std::mt19937::result_type>(seed));
}

void MakeUniform(DistMatrix& A, double center, double radius) {
    if (A.ColDist() == Dist::CIRC || A.RowDist() == Dist::CIRC) {
        ELX_REQUIRE(A.ColDist() == A.RowDist(), "MakeUniform: bad distribution");
    }
    const Int m = A.LocalHeight(), n = A.LocalWidth();
    Comm* red = A.Participating() ? RedundantComm(A) : nullptr;
    const bool drawer = A.Participating() && (red == nullptr || red->Rank() == 0);
    if (drawer && m > 0 && n > 0) {
        auto& gen = Generator();
        std::vector<unsigned char> host(static_cast<size_t>(m * n) * A.ElemSize());
        switch (A.Type()) {
        case DType::F64: {
            std::uniform_real_distribution<double> uni(center - radius, center + radius);
            double* h = reinterpret_cast<double*>(host.data());
            for (Int j = 0; j < n; ++j)
                for (Int i = 0; i < m; ++i) h[i + j * m] = uni(gen);
            break;
        }
        case DType::F32: {
            const float c = static_cast<float>(center), r = static_cast<float>(radius);
            std::uniform_real_distribution<float> uni(c - r, c + r);  // SampleBall<float>: float arithmetic
            float* h = reinterpret_cast<float*>(host.data());
            for (Int j = 0; j < n; ++j)
                for (Int i = 0; i < m; ++i) h[i + j * m] = uni(gen);
            break;
        }
        case DType::F16: {  // cpu_half_type: half arithmetic for the bounds, float draw, RNE to half
            const float c = HalfToFloat(FloatToHalf(static_cast<float>(center)));
            const float r = HalfToFloat(FloatToHalf(static_cast<float>(radius)));
            const float lo = HalfToFloat(FloatToHalf(c - r)), hi = HalfToFloat(FloatToHalf(c + r));
            std::uniform_real_distribution<float> uni(lo, hi);
            uint16_t* h = reinterpret_cast<uint16_t*>(host.data());
            for (Int j = 0; j < n; ++j)
                for (Int i = 0; i < m; ++i) h[i + j * m] = FloatToHalf(uni(gen));
            break;
        }
        case DType::BF16: {  // no reference type: the float draw rounded to bf16
            const float c = static_cast<float>(center), r = static_cast<float>(radius);
            std::uniform_real_distribution<float> uni(c - r, c + r);
            uint16_t* h = reinterpret_cast<uint16_t*>(host.data());
            for (Int j = 0; j < n; ++j)
                for (Int i = 0; i < m; ++i) h[i + j * m] = FloatToBF16(uni(gen));
            break;
        }
        default:
            throw LogicError(Cat("MakeUniform: dtype ", DTypeName(A.Type()), " is not a matrix type"));
        }
        A.SetLocal(host.data(), m);
    }
    if (red && red->Size() > 1 && m > 0 && n > 0) {
        if (red->kind() == Comm::Kind::RCCL && A.Dev() == Device::CPU) {
            // CPU matrices on an RCCL grid: stage through device memory
            std::vector<unsigned char> host(static_cast<size_t>(m * n) * A.ElemSize());
            if (drawer) A.GetLocal(host.data(), m);
            hipStream_t s = Runtime::Get().CommStream();
            Buffer tmp(Device::GPU, host.size(), s);
            if (drawer) ELX_CHECK_HIP(hipMemcpyAsync(tmp.data(), host.data(), host.size(), hipMemcpyHostToDevice, s));
            red->Bcast(A.Type(), tmp.data(), m * n, 0, Device::GPU, s);
            ELX_CHECK_HIP(hipMemcpyAsync(host.data(), tmp.data(), host.size(), hipMemcpyDeviceToHost, s));
            ELX_CHECK_HIP(hipStreamSynchronize(s));
            A.SetLocal(host.data(), m);
        } else {  // RCCL on device memory, or the host backend (which stages device buffers itself)
            red->Bcast(A.Type(), A.Buffer(), A.LDim() * n, 0, A.Dev(), A.Stream());
        }
    }
}

void Uniform(DistMatrix& A, Int m, Int n, double center, double radius) {
    A.Resize(m, n);
    MakeUniform(A, center, radius);
}

}  // namespace elx
