// Functor-generic El::EntrywiseMap / El::Combine on GPU matrices
// (include/El/EntrywiseMap.hip.hpp, the reference's EntrywiseMapImpl /
// CombineImpl device templates): user device lambdas and a functor struct on
// Matrix<T,GPU>, DistMatrix local blocks, a cross-distribution DistMatrix map
// and the in-place form, checked entry by entry on the host.  Built by
// __graft_entry__.build() with hipcc; run by tests/test_gpu_dist.py.
#include <El.hpp>

#include <cmath>
#include <cstdio>
#include <vector>

static int failures = 0;
#define EXPECT(cond)                                                                        \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            std::fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                                     \
        }                                                                                   \
    } while (0)

// the device may contract a*b+c into one fused multiply-add (one rounding where
// the host rounds twice): compare to a few ulps
static bool Near(double got, double want) { return std::fabs(got - want) <= 4e-16 * (std::fabs(want) + 1.0); }

struct LeakyRelu {  // a functor type with state
    float slope;
    __host__ __device__ float operator()(float x) const { return x > 0.f ? x : slope * x; }
};

template <typename T, El::Dist U, El::Dist V>
static std::vector<T> Local(const El::DistMatrix<T, U, V, El::ELEMENT, El::Device::GPU>& A) {
    std::vector<T> h(std::max<El::Int>(A.LocalHeight() * A.LocalWidth(), 1));
    A.GetLocalBlock(h.data(), std::max<El::Int>(A.LocalHeight(), 1));
    return h;
}

int main() {
    using El::Int;
    using GPUMat = El::DistMatrix<double, El::MC, El::MR, El::ELEMENT, El::Device::GPU>;
    El::Grid g;
    const Int m = 1531, n = 67;  // a ragged last row chunk (1531 = 1024 + 507)
    GPUMat A(m, n, g), B(g);
    El::HashFill(A, 5, 0.0, 2.0);
    const auto a = Local(A);

    // a device lambda on local matrices: an owned Matrix<double,GPU> is resized to A's block
    El::Matrix<double, El::Device::GPU> Bm;
    El::EntrywiseMap(A.LockedMatrix(), Bm, [] __device__(double x) { return 3.0 * x * x - 1.0; });
    EXPECT(Bm.Height() == m && Bm.Width() == n && Near(Bm.Get(7, 3), 3.0 * a[7 + 3 * m] * a[7 + 3 * m] - 1.0));
    (void)B;
    GPUMat B2(m, n, g);
    El::EntrywiseMap(A, B2, [] __device__(double x) { return 3.0 * x * x - 1.0; });
    auto b = Local(B2);
    bool ok = true;
    for (Int i = 0; i < m * n; ++i) ok &= Near(b[i], 3.0 * a[i] * a[i] - 1.0);
    EXPECT(ok);

    // Combine: B2 := a * B2 + 1 (binary lambda), then in place B2 := -B2
    El::Combine(A, B2, [] __device__(double x, double y) { return x * y + 1.0; });
    El::EntrywiseMap(B2, [] __host__ __device__(double y) { return -y; });
    b = Local(B2);
    ok = true;
    for (Int i = 0; i < m * n; ++i) ok &= Near(b[i], -(a[i] * (3.0 * a[i] * a[i] - 1.0) + 1.0));
    EXPECT(ok);

    // type-changing map with a functor struct: double [MC,MR] -> float [STAR,VR]
    // (A redistributed to B's distribution first, EntrywiseMap.hpp:90-137)
    El::DistMatrix<float, El::STAR, El::VR, El::ELEMENT, El::Device::GPU> F(g);
    El::DistMatrix<double, El::STAR, El::VR, El::ELEMENT, El::Device::GPU> Astar(g);
    Astar = A;
    El::EntrywiseMap(A, F, [] __device__(double x) { return LeakyRelu{0.25f}(static_cast<float>(x)); });
    const auto f = Local(F);
    const auto as = Local(Astar);
    ok = F.Height() == m && F.Width() == n && F.LocalHeight() == Astar.LocalHeight();
    for (Int i = 0; i < F.LocalHeight() * F.LocalWidth() && ok; ++i)
        ok &= f[i] == LeakyRelu{0.25f}(static_cast<float>(as[i]));
    EXPECT(ok);

    // Matrix<T,GPU> directly, with a caller stream (created before and destroyed
    // after the matrices that use it: Y's buffer is released on it)
    void* s = nullptr;
    elx_stream_create(&s);
    {
    El::Matrix<float, El::Device::GPU> X(300, 5), Y;
    El::Fill(X, 2.0f);
    Y.SetStream(s);
    El::EntrywiseMap(X, Y, LeakyRelu{0.5f});
    El::Combine(X, Y, [] __device__(float x, float y) { return x - 4.f * y; });  // 2 - 8 = -6
    (void)hipStreamSynchronize(static_cast<hipStream_t>(s));
    EXPECT(Y.Height() == 300 && Y.Width() == 5 && Y.Get(0, 0) == -6.f && Y.Get(299, 4) == -6.f);
    bool threw = false;
    try {
        El::Matrix<float, El::Device::GPU> Z(3, 3);
        El::Combine(X, Z, [] __device__(float x, float y) { return x + y; });
    } catch (const El::RuntimeError&) {
        threw = true;
    }
    EXPECT(threw);
    }
    (void)hipDeviceSynchronize();
    elx_stream_destroy(s);
    if (failures) {
        std::fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    std::printf("functor EntrywiseMap/Combine test OK\n");
    std::fflush(stdout);
    return 0;
}
