// Compiled check of the drop-in C++ surface (include/El.hpp) over a 1x1 grid:
// it must compile the way reference callers write El::Gemm code
// (tests/blas_like/Gemm.cpp:20-140 shape) and give the same answers as a plain
// triple loop.  Built and run on Device::CPU matrices by tests/test_capi_cpu.py
// and, with -DEL_TEST_GPU, on Device::GPU matrices by tests/test_gpu_dist.py.
#include <El.hpp>
#include <unistd.h>
#include <cstdio>
#include <string>

#include <cmath>
#include <cstdio>
#include <vector>

#ifdef EL_TEST_GPU
constexpr El::Device kDev = El::Device::GPU;
#else
constexpr El::Device kDev = El::Device::CPU;
#endif
template <typename T, El::Dist U = El::MC, El::Dist V = El::MR>
using DM = El::DistMatrix<T, U, V, El::ELEMENT, kDev>;

static int failures = 0;
#define EXPECT(cond)                                                        \
    do {                                                                    \
        if (!(cond)) {                                                      \
            std::fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                     \
        }                                                                   \
    } while (0)

template <typename T, El::Dist U, El::Dist V>
static std::vector<T> Local(const DM<T, U, V>& A) {
    std::vector<T> h(std::max<El::Int>(A.LocalHeight() * A.LocalWidth(), 1));
    A.GetLocalBlock(h.data(), std::max<El::Int>(A.LocalHeight(), 1));
    return h;
}

// host copy of a local matrix (entry by entry: small test sizes only)
template <typename T>
static std::vector<T> HostOf(const El::Matrix<T, kDev>& M) {
    std::vector<T> h(M.LDim() * M.Width());
    for (El::Int j = 0; j < M.Width(); ++j)
        for (El::Int i = 0; i < M.Height(); ++i) h[i + j * M.LDim()] = M.Get(i, j);
    return h;
}

int main() {
    using El::Int;
    El::Initialize();
    El::Grid g;  // 1x1 over COMM_SELF
    EXPECT(g.Height() == 1 && g.Width() == 1 && g.Size() == 1);
    EXPECT(El::Grid::DefaultHeight(8) == 2 && El::Grid::DefaultHeight(4) == 2 && El::Grid::DefaultHeight(2) == 1);

    const Int m = 37, n = 29, k = 41;
    DM<double> A(m, k, g), B(k, n, g), C(m, n, g);
    El::HashFill(A, 11, 0.0, 1.0);
    El::HashFill(B, 12, 0.0, 1.0);
    El::HashFill(C, 13, 0.0, 1.0);
    EXPECT(A.Height() == m && A.Width() == k && A.LocalHeight() == m && A.LDim() >= m);
    EXPECT(A.ColDist() == El::MC && A.RowDist() == El::MR && A.GetLocalDevice() == kDev);
    const auto a = Local(A), b = Local(B), c0 = Local(C);

    // C := 0.5 A B - 0.25 C
    El::Gemm(El::NORMAL, El::NORMAL, 0.5, A, B, -0.25, C);
    auto c = Local(C);
    double err = 0, ref = 0;
    for (Int j = 0; j < n; ++j)
        for (Int i = 0; i < m; ++i) {
            double s = 0;
            for (Int l = 0; l < k; ++l) s += a[i + l * m] * b[l + j * k];
            const double want = 0.5 * s - 0.25 * c0[i + j * m];
            err = std::max(err, std::fabs(c[i + j * m] - want));
            ref = std::max(ref, std::fabs(want));
        }
    EXPECT(err <= 1e-13 * (ref + 1));

    // beta-less form resizes C; transpose orientation: D := A^T A  (k x k)
    DM<double> D(g);
    El::Gemm(El::TRANSPOSE, El::NORMAL, 1.0, A, A, D, El::GEMM_SUMMA_C);
    EXPECT(D.Height() == k && D.Width() == k);
    auto d = Local(D);
    err = 0;
    for (Int j = 0; j < k; ++j)
        for (Int i = 0; i < k; ++i) {
            double s = 0;
            for (Int l = 0; l < m; ++l) s += a[l + i * m] * a[l + j * m];
            err = std::max(err, std::fabs(d[i + j * k] - s));
        }
    EXPECT(err <= 1e-12);

    // Syrk (beta-less): E := tril(A^T A); its strict upper triangle stays zero
    DM<double> E(g);
    El::Syrk(El::LOWER, El::TRANSPOSE, 1.0, A, E);
    EXPECT(E.Height() == k && E.Width() == k);
    auto e = Local(E);
    err = 0;
    for (Int j = 0; j < k; ++j)
        for (Int i = 0; i < k; ++i)
            err = std::max(err, std::fabs(e[i + j * k] - (i >= j ? d[i + j * k] : 0.0)));
    EXPECT(err <= 1e-12);
    // Herk with beta: the upper triangle is scaled and updated, the lower untouched
    El::Herk(El::UPPER, El::TRANSPOSE, 1.0, A, 2.0, E);
    e = Local(E);
    err = 0;
    for (Int j = 0; j < k; ++j)
        for (Int i = 0; i < k; ++i)
            err = std::max(err, std::fabs(e[i + j * k] - (i > j ? d[i + j * k] : i == j ? 3.0 * d[i + j * k] : d[i + j * k])));
    EXPECT(err <= 1e-12);

    // Trsm: solve tril(E) Y = 2 R (R: k x n right-hand sides taken from C; E's
    // diagonal is 3 d_ii > 0 after the Herk above); check tril(E) Y == 2 R
    {
        const auto c_now = Local(C);
        std::vector<double> rhs(k * n);
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < k; ++i) rhs[i + j * k] = c_now[(i % m) + j * m];
        DM<double> Y(k, n, g);
        Y.SetLocalBlock(rhs.data(), k);
        El::Trsm(El::LEFT, El::LOWER, El::NORMAL, El::NON_UNIT, 2.0, E, Y);
        const auto y = Local(Y);
        double rerr = 0, rref = 0;
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < k; ++i) {
                double s = 0;
                for (Int l = 0; l <= i; ++l) s += e[i + l * k] * y[l + j * k];
                rerr = std::max(rerr, std::fabs(s - 2.0 * rhs[i + j * k]));
                rref = std::max(rref, std::fabs(rhs[i + j * k]));
            }
        EXPECT(rerr <= 1e-10 * (rref + 1));
    }

    // redistribution + transpose + view are bit-exact
    DM<double, El::STAR, El::STAR> S(A);
    EXPECT(Local(S) == a);
    DM<double, El::VR, El::STAR> R(g);
    R = A;
    EXPECT(Local(R) == a);
    DM<double> T(g);
    El::Transpose(A, T);
    auto t = Local(T);
    bool tok = T.Height() == k && T.Width() == m;
    for (Int j = 0; j < m && tok; ++j)
        for (Int i = 0; i < k; ++i) tok &= t[i + j * k] == a[j + i * m];
    EXPECT(tok);
    auto Av = A(El::IR(3, 10), El::IR(5, 9));
    EXPECT(Av.Height() == 7 && Av.Width() == 4 && Av.Viewing());
    DM<double> W(Av);
    auto w = Local(W);
    bool vok = true;
    for (Int j = 0; j < 4; ++j)
        for (Int i = 0; i < 7; ++i) vok &= w[i + j * 7] == a[(3 + i) + (5 + j) * m];
    EXPECT(vok);

    // level-1 front doors
    DM<double> Y(S);
    El::Axpy(2.0, A, Y);   // Y = 3A
    El::Scale(0.5, Y);     // Y = 1.5A
    auto y = Local(Y);
    bool aok = true;
    for (size_t i = 0; i < a.size(); ++i) aok &= std::fabs(y[i] - 1.5 * a[i]) <= 1e-15 * std::fabs(a[i]) + 1e-300;
    EXPECT(aok);
    El::EntrywiseMap(A, Y, El::EntrywiseFn::SQUARE);
    DM<double> H(g);
    H.Resize(m, k);
    El::Hadamard(A, A, H);
    EXPECT(Local(H) == Local(Y));
    El::Combine(A, H, El::CombineFn::SUB);  // H := H - A = A.*A - A
    {
        auto h = Local(H);
        bool cok = true;
        for (size_t i = 0; i < a.size(); ++i) cok &= h[i] == a[i] * a[i] - a[i];
        EXPECT(cok);
    }
    El::Zero(H);
    for (double v : Local(H)) EXPECT(v == 0.0);

    // float path
    DM<float> Af(8, 8, g), Bf(8, 8, g), Cf(8, 8, g);
    El::HashFill(Af, 1, 0.0, 1.0);
    El::HashFill(Bf, 2, 0.0, 1.0);
    El::Gemm(El::NORMAL, El::TRANSPOSE, 1.0f, Af, Bf, 0.0f, Cf);
    auto af = Local(Af), bf = Local(Bf), cf = Local(Cf);
    float ferr = 0;
    for (int j = 0; j < 8; ++j)
        for (int i = 0; i < 8; ++i) {
            float s = 0;
            for (int l = 0; l < 8; ++l) s += af[i + l * 8] * bf[j + l * 8];
            ferr = std::max(ferr, std::fabs(cf[i + j * 8] - s));
        }
    EXPECT(ferr <= 1e-5f);

    // error mapping: nonconformal Gemm is a LogicError, as Gemm.cpp:279-283
    bool threw = false;
    try {
        El::Gemm(El::NORMAL, El::NORMAL, 1.0, A, A, 0.0, C);
    } catch (const El::LogicError&) {
        threw = true;
    }
    EXPECT(threw);

    // Attach: caller storage (an El::Matrix on the same device) with ldim > height, computed into in place
    El::Matrix<double, kDev> Cm(m + 2, n);
    El::Fill(Cm, 9.0);
    DM<double> Ca(g);
    Ca.Attach(m, n, g, 0, 0, Cm.Buffer(), m + 2);
    EXPECT(Ca.Viewing() && Ca.LDim() == m + 2);
    El::Gemm(El::NORMAL, El::NORMAL, 0.5, A, B, 0.0, Ca);
    Ca.Synchronize();
    const std::vector<double> cbuf = HostOf(Cm);
    bool tok2 = true;
    for (Int j = 0; j < n; ++j) {
        for (Int i = 0; i < m; ++i) {
            double s = 0;
            for (Int l = 0; l < k; ++l) s += a[i + l * m] * b[l + j * k];
            tok2 &= std::fabs(cbuf[i + j * (m + 2)] - 0.5 * s) <= 1e-13;
        }
        tok2 &= cbuf[m + j * (m + 2)] == 9.0 && cbuf[m + 1 + j * (m + 2)] == 9.0;
    }
    EXPECT(tok2);

    // El::Write / El::Read round trip (BINARY: Int h, Int w, column-major data)
    {
        const std::string base = "/tmp/elx_api_test_" + std::to_string(::getpid());
        El::Write(A, base, El::BINARY);
        DM<double, El::VC, El::STAR> R(g);
        El::Read(R, base + ".bin");
        EXPECT(R.Height() == m && R.Width() == k && Local(R) == Local(A));
        std::remove((base + ".bin").c_str());
    }

    // El::Matrix<T,D> and Gemm on local matrices (level3.hpp:37-65): the local
    // blocks of A and B through LockedMatrix(), into an owned Matrix
    {
        El::Matrix<double, kDev> L(m, n);
        El::Gemm(El::NORMAL, El::NORMAL, 0.5, A.LockedMatrix(), B.LockedMatrix(), 0.0, L);
        EXPECT(A.LockedMatrix().Height() == m && A.LockedMatrix().Width() == k && A.LockedMatrix().Viewing());
        El::Matrix<double, kDev> L2;  // beta-less form resizes
        El::Gemm(El::TRANSPOSE, El::NORMAL, 1.0, A.LockedMatrix(), A.LockedMatrix(), L2);
        EXPECT(L2.Height() == k && L2.Width() == k);
        const auto l = HostOf(L), l2 = HostOf(L2);
        double lerr = 0;
        for (Int j = 0; j < n; ++j)
            for (Int i = 0; i < m; ++i) {
                double s = 0;
                for (Int q = 0; q < k; ++q) s += a[i + q * m] * b[q + j * k];
                lerr = std::max(lerr, std::fabs(l[i + j * m] - 0.5 * s));
            }
        for (Int j = 0; j < k; ++j)
            for (Int i = 0; i < k; ++i) lerr = std::max(lerr, std::fabs(l2[i + j * k] - d[i + j * k]));
        EXPECT(lerr <= 1e-12);
        // level-1 on Matrix and on the DistMatrix's local block
        El::Matrix<double, kDev> X(L);  // deep copy
        El::Axpy(-1.0, L, X);           // X = 0
        for (double v : HostOf(X)) EXPECT(v == 0.0);
        El::Scale(2.0, A.Matrix());     // A's local block doubled in place ...
        EXPECT(A.Get(3, 5) == 2.0 * a[3 + 5 * m]);
        El::Scale(0.5, A.Matrix());     // ... and back (exact)
        EXPECT(Local(A) == a);
        bool threw_k = false;
        try { El::Gemm(El::NORMAL, El::NORMAL, 1.0, A.LockedMatrix(), A.LockedMatrix(), 0.0, L); }
        catch (const El::LogicError&) { threw_k = true; }
        EXPECT(threw_k);
    }

    // DistMatrix entry access (Get collective, Set / Update local) and El::Fill
    {
        EXPECT(A.Get(3, 5) == a[3 + 5 * m] && A.Get(m - 1, k - 1) == a[(m - 1) + (k - 1) * m]);
        DM<double> F(4, 3, g);
        El::Fill(F, 2.5);
        for (double v : Local(F)) EXPECT(v == 2.5);
        F.Set(1, 2, -7.0);
        F.Update(1, 2, 0.5);
        EXPECT(F.Get(1, 2) == -6.5 && F.Get(0, 0) == 2.5);
        DM<El::gpu_half_type> Hh(3, 3, g);
        El::Fill(Hh, El::gpu_half_type{0x3c00});  // 1.0
        Hh.Set(2, 1, El::gpu_half_type{0xc000});   // -2.0
        EXPECT(Hh.Get(0, 0).x == 0x3c00 && Hh.Get(2, 1).x == 0xc000);
        DM<El::bfloat16> Bh(2, 2, g);
        Bh.Set(1, 1, El::bfloat16{0x4040});        // 3.0
        EXPECT(Bh.Get(1, 1).x == 0x4040);
    }

    // Trsm's checkIfSingular (Trsm.cpp:60-68): an exact zero on a NON_UNIT
    // diagonal raises SingularMatrixException; UNIT diagonals are not checked
    {
        DM<double> Z(5, 5, g), Y(5, 2, g);
        El::Fill(Z, 1.0);
        El::Fill(Y, 1.0);
        Z.Set(3, 3, 0.0);
        bool sing = false;
        try { El::Trsm(El::LEFT, El::LOWER, El::NORMAL, El::NON_UNIT, 1.0, Z, Y, true); }
        catch (const El::SingularMatrixException&) { sing = true; }
        EXPECT(sing);
        El::Trsm(El::LEFT, El::LOWER, El::NORMAL, El::UNIT, 1.0, Z, Y, true);
        EXPECT(Y.Get(0, 0) == 1.0 && Y.Get(1, 0) == 0.0);
    }

    El::SetBlocksize(64);
    EXPECT(El::Blocksize() == 64);
    El::SetBlocksize(128);

    // blocksize stack (environment/decl.hpp:88-94, blocksizes.cpp:38-72)
    {
        El::PushBlocksizeStack(32);
        EXPECT(El::Blocksize() == 32);
        El::SetBlocksize(48);  // SetBlocksize rewrites the top only
        EXPECT(El::Blocksize() == 48);
        El::PopBlocksizeStack();
        EXPECT(El::Blocksize() == 128);
        El::EmptyBlocksizeStack();
        bool threw_b = false;
        try { (void)El::Blocksize(); } catch (const El::LogicError&) { threw_b = true; }
        EXPECT(threw_b);
        El::PushBlocksizeStack(128);
        EXPECT(El::Blocksize() == 128);
    }

    // El::mpi::COMM_WORLD (imports/mpi.hpp:86): a grid over it, and Grid()
    {
        El::Grid gw(El::mpi::COMM_WORLD);
        EXPECT(gw.Size() == El::mpi::Size(El::mpi::COMM_WORLD) && gw.Size() == 1);
        EXPECT(El::mpi::Rank() == 0 && El::mpi::COMM_WORLD.Rank() == 0);
        El::mpi::Barrier(El::mpi::COMM_WORLD);
        DM<double> Wm(5, 4, gw);
        El::Fill(Wm, 1.5);
        EXPECT(Wm.Get(4, 3) == 1.5);
    }

    // SyncInfo / SyncInfoFromMatrix / SetSyncInfo / MultiSync
    // (Matrix/decl.hpp:287-296,478-479,521-533, rocm/SyncInfo.hpp:15-81, MultiSync.hpp:33-78)
    {
        El::Matrix<double, kDev> Mx(4, 4);
        auto si = El::SyncInfoFromMatrix(Mx);
        El::SetSyncInfo(Mx, si);
        auto ms = El::MakeMultiSync(si, El::SyncInfoFromMatrix(A.LockedMatrix()));
        (void)ms;
        El::Synchronize(si);
        EXPECT(si == El::SyncInfoFromMatrix(Mx));
    }
    // El::mpi typed collectives on SyncInfo-tagged buffers over COMM_WORLD and
    // COMM_SELF (imports/mpi.hpp:593-1400): buffers of the test's device
    {
        const int n = 6;
        const auto& comm = El::mpi::COMM_WORLD;
        const int p = El::mpi::Size(comm), me = El::mpi::Rank(comm);
        El::Matrix<double, kDev> S(n, 1), R(n * p, 1), T(n, 1);
        auto si = El::SyncInfoFromMatrix(S);
        for (int i = 0; i < n; ++i) S.Set(i, 0, 10.0 * me + i - 2.0);
        El::mpi::AllGather(S.LockedBuffer(), n, R.Buffer(), n, comm, si);
        bool ok = true;
        for (int q = 0; q < p; ++q)
            for (int i = 0; i < n; ++i) ok &= R.Get(q * n + i, 0) == 10.0 * q + i - 2.0;
        EXPECT(ok);
        El::mpi::AllReduce(S.LockedBuffer(), T.Buffer(), n, El::mpi::MAX, comm, si);
        for (int i = 0; i < n; ++i) EXPECT(T.Get(i, 0) == 10.0 * (p - 1) + i - 2.0);
        El::mpi::AllReduce(T.Buffer(), n, comm, si);  // in place, SUM
        for (int i = 0; i < n; ++i) EXPECT(T.Get(i, 0) == p * (10.0 * (p - 1) + i - 2.0));
        El::mpi::AllReduce(S.LockedBuffer(), T.Buffer(), n, El::mpi::MIN, comm, si);
        for (int i = 0; i < n; ++i) EXPECT(T.Get(i, 0) == i - 2.0);
        EXPECT(El::mpi::AllReduce(3.0, El::mpi::PROD, comm, si) == std::pow(3.0, p));
        EXPECT(El::mpi::AllReduce(2.5, comm, si) == 2.5 * p);
        El::Matrix<double, kDev> RS(n * p, 1), Ro(n, 1);
        for (int i = 0; i < n * p; ++i) RS.Set(i, 0, i + 1.0);
        El::mpi::ReduceScatter(RS.LockedBuffer(), Ro.Buffer(), n, comm, si);
        for (int i = 0; i < n; ++i) EXPECT(Ro.Get(i, 0) == p * (me * n + i + 1.0));
        El::mpi::ReduceScatter(RS.LockedBuffer(), Ro.Buffer(), n, El::mpi::MAX, comm, si);
        for (int i = 0; i < n; ++i) EXPECT(Ro.Get(i, 0) == me * n + i + 1.0);
        El::Matrix<double, kDev> A2(n * p, 1);
        El::mpi::AllToAll(RS.LockedBuffer(), n, A2.Buffer(), n, comm, si);
        for (int i = 0; i < n; ++i) EXPECT(A2.Get(i, 0) == me * n + i + 1.0);
        El::Matrix<double, kDev> B(n, 1);
        for (int i = 0; i < n; ++i) B.Set(i, 0, me == 0 ? 7.0 + i : -1.0);
        El::mpi::Broadcast(B.Buffer(), n, 0, comm, si);
        for (int i = 0; i < n; ++i) EXPECT(B.Get(i, 0) == 7.0 + i);
        El::mpi::SendRecv(S.LockedBuffer(), n, (me + 1) % p, T.Buffer(), n, (me + p - 1) % p, comm, si);
        for (int i = 0; i < n; ++i) EXPECT(T.Get(i, 0) == 10.0 * ((me + p - 1) % p) + i - 2.0);
        El::mpi::SendRecv(B.Buffer(), n, (me + 1) % p, (me + p - 1) % p, comm, si);  // in place
        for (int i = 0; i < n; ++i) EXPECT(B.Get(i, 0) == 7.0 + i);
        {  // in-place SendRecv of Int and byte buffers on the test's device
            El::Matrix<El::Int, kDev> I(3, 1);
            El::Matrix<unsigned char, kDev> U(5, 1);
            for (int i = 0; i < 3; ++i) I.Set(i, 0, 100 * me + i);
            for (int i = 0; i < 5; ++i) U.Set(i, 0, static_cast<unsigned char>(10 * me + i));
            El::mpi::SendRecv(I.Buffer(), 3, (me + 1) % p, (me + p - 1) % p, comm, El::SyncInfoFromMatrix(I));
            El::mpi::SendRecv(U.Buffer(), 5, (me + 1) % p, (me + p - 1) % p, comm, El::SyncInfoFromMatrix(U));
            const int src = (me + p - 1) % p;
            for (int i = 0; i < 3; ++i) EXPECT(I.Get(i, 0) == 100 * src + i);
            for (int i = 0; i < 5; ++i) EXPECT(U.Get(i, 0) == static_cast<unsigned char>(10 * src + i));
        }
        double scalar = me == 0 ? 4.25 : 0.0;
        El::mpi::Broadcast(scalar, 0, comm, El::SyncInfo<El::Device::CPU>{});
        EXPECT(scalar == 4.25);
        bool threw_c = false;
        try { El::mpi::AllGather(S.LockedBuffer(), n, R.Buffer(), n - 1, comm, si); }
        catch (const El::LogicError&) { threw_c = true; }
        EXPECT(threw_c);
        threw_c = false;
        try { El::mpi::Broadcast(B.Buffer(), n, p, comm, si); }
        catch (const El::LogicError&) { threw_c = true; }
        EXPECT(threw_c);
        // Int / int / byte buffers (host memory, any device tag)
        {
            const El::Int xi = me + 1;
            EXPECT(El::mpi::AllReduce(xi, El::mpi::SUM, comm, El::SyncInfo<El::Device::CPU>{}) ==
                   (El::Int)p * (p + 1) / 2);
            std::int32_t v32[3] = {me, -me, 7};
            El::mpi::AllReduce(v32, 3, El::mpi::MAX, comm, El::SyncInfo<El::Device::CPU>{});
            EXPECT(v32[0] == p - 1 && v32[1] == 0 && v32[2] == 7);
            std::vector<unsigned char> bytes(4 * p), mine = {1, 2, 3, (unsigned char)me};
            El::mpi::AllGather(mine.data(), 4, bytes.data(), 4, comm, El::SyncInfo<El::Device::CPU>{});
            EXPECT(bytes[4 * (p - 1) + 3] == (unsigned char)(p - 1) && bytes[1] == 2);
        }
        // a split-off self communicator works the same way
        const El::mpi::Comm self = El::mpi::COMM_SELF();
        El::mpi::AllReduce(S.LockedBuffer(), T.Buffer(), n, El::mpi::SUM, self, si);
        for (int i = 0; i < n; ++i) EXPECT(T.Get(i, 0) == 10.0 * me + i - 2.0);
        El::Synchronize(si);
    }
#ifdef EL_TEST_GPU
    {
        using GPU = El::SyncInfo<El::Device::GPU>;
        const GPU& dflt = El::gpu::DefaultSyncInfo();
        EXPECT(dflt.Stream() != nullptr && dflt.Event() != nullptr);
        EXPECT(GPU{} == dflt);
        GPU si1 = El::CreateNewSyncInfo<El::Device::GPU>();
        GPU si2 = El::CreateNewSyncInfo<El::Device::GPU>();
        EXPECT(si1.Stream() && si1.Event() && si1.Stream() != si2.Stream() && si1 != si2);
        // Merge keeps the parts the argument leaves null
        GPU part(si1.Stream(), nullptr);
        GPU merged = dflt;
        merged.Merge(part);
        EXPECT(merged.Stream() == si1.Stream() && merged.Event() == dflt.Event());

        // event-fenced hand-off: X is produced on si1 by a ~2 ms GEMM, consumed
        // on si2 right after; the fence is what makes the consumer see it
        const Int nn = 4096;
        El::Matrix<double, El::Device::GPU> P(nn, nn), Q(nn, nn), X(nn, nn), Yh(nn, nn);
        for (auto* M : {&P, &Q, &X, &Yh}) El::SetSyncInfo(*M, si1);
        EXPECT(El::SyncInfoFromMatrix(X).Stream() == si1.Stream() && El::SyncInfoFromMatrix(X).Event() == si1.Event());
        El::Fill(P, 1.0);
        El::Fill(Q, 0.5);
        El::Fill(X, -1.0);
        El::Fill(Yh, -3.0);
        El::Synchronize(si1);
        El::Gemm(El::NORMAL, El::NORMAL, 1.0, P, Q, 0.0, X);  // X = 2048 everywhere (exact), on si1
        El::AddSynchronizationPoint(si1, si2);                // si2 waits for si1's queued work
        El::SetSyncInfo(Yh, si2);                              // Yh moves to si2 (fenced after si1)
        {
            auto fence = El::MakeMultiSync(si2, si1);           // on exit si1 waits for si2
            El::Copy(X, Yh);                                    // on Yh's stream, si2; X on si1 is fenced in too
        }
        El::Synchronize(si1);                                  // si1 now covers si2's copy
        EXPECT(Yh.Get(0, 0) == 2048.0 && Yh.Get(nn - 1, nn - 1) == 2048.0 && Yh.Get(nn / 2, 17) == 2048.0);

        // local Gemm with A and B on a stream other than C's (Gemm.cpp:178-180
        // MakeMultiSync(C, A, B)): C on si2 must see P written on si1
        El::Matrix<double, El::Device::GPU> Cg(64, 64);
        El::SetSyncInfo(Cg, si2);
        El::Fill(Cg, 0.0);
        El::Synchronize(si2);
        El::Scale(2.0, P);                                    // P = 2 (on si1), queued behind nothing long ...
        El::Gemm(El::NORMAL, El::NORMAL, 1.0, Q, P, 0.0, X);   // ... then a long GEMM on si1 rewrites X = 4096
        El::Matrix<double, El::Device::GPU> Xv;
        Xv.LockedAttach(64, nn, X.LockedBuffer(), X.LDim());   // a view of X's first 64 rows, on si1
        El::SetSyncInfo(Xv, si1);
        El::Matrix<double, El::Device::GPU> Pv;
        Pv.LockedAttach(nn, 64, P.LockedBuffer(), P.LDim());
        El::SetSyncInfo(Pv, si1);
        El::Gemm(El::NORMAL, El::NORMAL, 1.0, Xv, Pv, 0.0, Cg); // on si2: Cg = 4096 * 2 * 4096
        El::Synchronize(si2);
        EXPECT(Cg.Get(0, 0) == 4096.0 * 2.0 * 4096.0 && Cg.Get(63, 63) == 4096.0 * 2.0 * 4096.0);

        // a DistMatrix's local block: SetSyncInfo on Matrix() moves the DistMatrix
        DM<double> Ds(6, 5, g);
        El::SetSyncInfo(Ds.Matrix(), si1);
        EXPECT(Ds.Stream() == static_cast<void*>(si1.Stream()));
        EXPECT(El::SyncInfoFromMatrix(Ds.LockedMatrix()).Stream() == si1.Stream());
        El::Fill(Ds, 4.0);
        EXPECT(Ds.Get(5, 4) == 4.0);
        El::SetSyncInfo(Ds.Matrix(), dflt);
        EXPECT(Ds.Stream() == static_cast<void*>(dflt.Stream()));

        // a moved-from matrix keeps a usable SyncInfo and serves as an output
        // fenced against operands on another stream (LocalFence records on it)
        {
            El::Matrix<double, El::Device::GPU> Src(8, 8);
            El::Fill(Src, 1.0);
            El::Matrix<double, El::Device::GPU> Dst(std::move(Src));
            EXPECT(Src.GetSyncInfo().Event() != nullptr && Src.GetSyncInfo().Stream() != nullptr);
            El::Matrix<double, El::Device::GPU> Qv;
            Qv.LockedAttach(8, 8, Q.LockedBuffer(), Q.LDim());
            El::SetSyncInfo(Qv, si1);
            El::Gemm(El::NORMAL, El::NORMAL, 1.0, Dst, Qv, Src);  // beta-less: Src resized, = 8 * 0.5
            El::Synchronize(El::SyncInfoFromMatrix(Src));
            EXPECT(Src.Height() == 8 && Src.Get(0, 0) == 4.0 && Src.Get(7, 7) == 4.0);
        }
        {
            // the fenced call throws after the fence is set up (a locked output)
            // with operands on another stream: a catchable LogicError, not a
            // terminate from the fence's destructor
            El::Matrix<double, El::Device::GPU> Cw(8, 8), Qv, Cl;
            El::SetSyncInfo(Cw, si2);
            Qv.LockedAttach(8, 8, Q.LockedBuffer(), Q.LDim());
            El::SetSyncInfo(Qv, si1);
            Cl.LockedAttach(8, 8, Cw.LockedBuffer(), Cw.LDim());
            El::SetSyncInfo(Cl, si2);
            bool threw_f = false;
            try { El::Gemm(El::NORMAL, El::NORMAL, 1.0, Qv, Qv, 0.0, Cl); }
            catch (const El::LogicError&) { threw_f = true; }
            EXPECT(threw_f);
        }

        for (auto* M : {&P, &Q, &X, &Yh, &Cg}) El::SetSyncInfo(*M, dflt);
        El::Synchronize(dflt);
        El::Synchronize(si1);
        El::Synchronize(si2);
        El::DestroySyncInfo(si1);
        El::DestroySyncInfo(si2);
        EXPECT(si1.Stream() == nullptr && si1.Event() == nullptr);
    }
#endif
    El::Finalize();
    if (failures) {
        std::fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    std::printf("El.hpp API test OK\n");
    return 0;
}
