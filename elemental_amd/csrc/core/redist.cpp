// The redistribution engine.
//
// The reference dispatches each (source, target) distribution pair to one of
// ~20 hand-written routines (include/El/blas_like/level1/Copy/*.hpp:
// RowAllGather, ColAllGather, PartialRow/ColAllGather, Col/RowAllToAllDemote/
// Promote, Exchange, Filter, Scatter, Gather, TranslateBetweenGrids, ...),
// each one pack -> MPI collective -> unpack, chained over up to three hops for
// pairs without a direct routine (e.g. MC_MR.cpp:85-139).
//
// Here every pair goes through ONE plan, computed from the layout formulas:
// for each peer pair (s -> d) the elements s sends to d are a Cartesian product
// I(s,d) x J(s,d) of two residue classes (CRT on the two cyclic patterns), so
// the pack and the unpack are single strided 2-D block moves.  Replicated
// sources send from one designated owner (the one that shares the receiver's
// free grid coordinates, i.e. the receiver itself whenever it already holds
// the data), so each element crosses the network at most once per receiver -
// the same bytes as the reference's AllGather/AllToAll/SendRecv chains, in one
// hop.  Execution: one batched pack launch, one grouped RCCL send/recv over the
// VC communicator (direct xGMI peer links), one batched unpack launch.  The
// result is bit-exact by construction (pure data movement).
#include "redist.hpp"
#include "exec.hpp"
#include "../runtime/trace.hpp"
#include <cstring>
#include <numeric>
#include <cmath>
#include <vector>

namespace elx {

namespace {

struct DimXfer {
    Int count = 0;
    Int src0 = 0, src_step = 1;  // first local index / step in the source
    Int dst0 = 0, dst_step = 1;  // ... in the target
};

Int Gcd(Int a, Int b) { while (b) { Int t = a % b; a = b; b = t; } return a; }

// Global indices in [0,n) held by source coordinate rs (stride ss, align as)
// AND wanted by target coordinate rd (stride sd, align ad).
DimXfer Intersect(Int n, int ss, int rs, int as, int sd, int rd, int ad) {
    DimXfer x;
    if (rs < 0 || rd < 0 || n == 0) return x;
    const Int shs = Shift(rs, as, ss), shd = Shift(rd, ad, sd);
    const Int L = ss / Gcd(ss, sd) * sd;
    for (Int z = shs; z < L; z += ss) {
        if (Mod(z - shd, sd) == 0) {
            x.count = Length(n, z, L);
            x.src0 = (z - shs) / ss;
            x.src_step = L / ss;
            x.dst0 = (z - shd) / sd;
            x.dst_step = L / sd;
            return x;
        }
    }
    return x;
}

// does the distribution pin a rank's grid row / column?  (an MD index names one
// rank of the root diagonal, so it pins both)
bool FixesMC(Dist d) { return d == Dist::MC || d == Dist::VC || d == Dist::VR || d == Dist::MD; }
bool FixesMR(Dist d) { return d == Dist::MR || d == Dist::VC || d == Dist::VR || d == Dist::MD; }

// Is source rank s the designated sender of A's data to receiver d?
bool Designated(const DistMatrix& A, int s, int d) {
    if (!A.ParticipatingOf(s)) return false;
    if (A.ColDist() == Dist::CIRC) return true;
    const Grid& g = A.G();
    const bool fmc = FixesMC(A.ColDist()) || FixesMC(A.RowDist());
    const bool fmr = FixesMR(A.ColDist()) || FixesMR(A.RowDist());
    return (fmc || g.MCOf(s) == g.MCOf(d)) && (fmr || g.MROf(s) == g.MROf(d));
}

struct PairPlan {
    DimXfer rows, cols;
    Int count() const { return rows.count * cols.count; }
};

PairPlan Plan(const DistMatrix& A, const DistMatrix& B, int s, int d) {
    PairPlan p;
    p.rows = Intersect(A.Height(), A.ColStride(), A.ColRankOf(s), A.ColAlign(), B.ColStride(), B.ColRankOf(d),
                       B.ColAlign());
    p.cols = Intersect(A.Width(), A.RowStride(), A.RowRankOf(s), A.RowAlign(), B.RowStride(), B.RowRankOf(d),
                       B.RowAlign());
    if (p.rows.count == 0 || p.cols.count == 0) p.rows.count = p.cols.count = 0;
    return p;
}

char* At(const DistMatrix& M, Int iLoc, Int jLoc) {
    return static_cast<char*>(M.Buffer()) + (iLoc + jLoc * M.LDim()) * static_cast<Int>(M.ElemSize());
}

// Order B's stream after A's pending work (the reference's MultiSync fencing,
// include/hydrogen/MultiSync.hpp:33-78).
void Fence(const DistMatrix& A, const DistMatrix& B) {
    if (A.Dev() != Device::GPU || B.Dev() != Device::GPU || A.Stream() == B.Stream()) return;
    hipEvent_t ev;
    ELX_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ELX_CHECK_HIP(hipEventRecord(ev, A.Stream()));
    ELX_CHECK_HIP(hipStreamWaitEvent(B.Stream(), ev, 0));
    ELX_CHECK_HIP(hipEventDestroy(ev));
}

// Alignment an unconstrained target adopts from its source, per dimension,
// following the one-hop copy routines: same dist -> same align
// (Copy/Translate); target is the partial of the source (VC->MC) -> align mod
// stride (ColAllToAllPromote.hpp:26, PartialColAllGather.hpp:43); source is the
// partial of the target (MC->VC) -> same align (ColAllToAllDemote.hpp:25);
// STAR -> 0; the source's other dimension of the same dist -> its align
// (transposing pairs, AlignColsWith ElementMatrix.cpp:243-269); else unchanged.
int AdoptAlign(Dist target, int stride, int cur, Dist srcSame, int alignSame, Dist srcOther, int alignOther) {
    auto partial = [](Dist u) { return u == Dist::VC ? Dist::MC : (u == Dist::VR ? Dist::MR : u); };
    if (target == Dist::STAR || target == Dist::CIRC) return 0;
    if (srcSame == target) return alignSame % stride;
    if (partial(srcSame) == target) return alignSame % stride;
    if (partial(target) == srcSame) return alignSame % stride;
    if (srcOther == target) return alignOther % stride;
    return cur;
}

void PrepareTarget(const DistMatrix& A, DistMatrix& B) {
    if (!B.Viewing()) {
        if (!B.ColConstrained())
            B.AlignCols(AdoptAlign(B.ColDist(), B.ColStride(), B.ColAlign(), A.ColDist(), A.ColAlign(), A.RowDist(),
                                   A.RowAlign()), false);
        if (!B.RowConstrained())
            B.AlignRows(AdoptAlign(B.RowDist(), B.RowStride(), B.RowAlign(), A.RowDist(), A.RowAlign(), A.ColDist(),
                                   A.ColAlign()), false);
    }
    B.Resize(A.Height(), A.Width());
}

void CheckCompatible(const DistMatrix& A, const DistMatrix& B) {
    ELX_REQUIRE(A.Type() == B.Type(), "redistribution between different types (", DTypeName(A.Type()), " -> ",
                DTypeName(B.Type()), ")");
    ELX_REQUIRE(&A.G() == &B.G(), "matrices live on different grids");
}

// Cross-device copy of A's local data into an identically distributed matrix on `dev`.
std::shared_ptr<DistMatrix> OnDevice(const DistMatrix& A, Device dev, hipStream_t s) {
    auto T = std::make_shared<DistMatrix>(A.GridPtr(), A.Type(), A.ColDist(), A.RowDist(), dev, A.Root());
    T->Align(A.ColAlign(), A.RowAlign(), true);
    T->Resize(A.Height(), A.Width());
    if (T->LocalHeight() > 0 && T->LocalWidth() > 0) {
        const size_t es = A.ElemSize();
        const hipMemcpyKind kind = dev == Device::GPU ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
        hipStream_t st = dev == Device::GPU ? T->Stream() : A.Stream();
        if (dev == Device::CPU) A.Synchronize();
        ELX_CHECK_HIP(hipMemcpy2DAsync(T->Buffer(), T->LDim() * es, A.Buffer(), A.LDim() * es,
                                       A.LocalHeight() * es, A.LocalWidth(), kind, st));
        ELX_CHECK_HIP(hipStreamSynchronize(st));
    }
    (void)s;
    return T;
}

// Shared transfer for Copy (designated senders, overwrite) and AxpyContract
// (every owner sends, receiver sums in rank order), in three stages so several
// transfers can share one exchange (CopyGroup): Prepare (plans, buffers, pack
// and the local portion, on B's stream), the AllToAllV over the VC
// communicator, Finish (unpack / rank-ordered sums).
struct TransferJob {
    const DistMatrix* A;
    DistMatrix* B;
    bool contract;
    double alpha;
    std::vector<PairPlan> out, in;
    std::vector<Int> sc, sd, rc, rd;
    bool cross = false;  // does any rank exchange data with another? (same answer on every rank)
    elx::Buffer sbuf, rbuf;
};

void TransferPrepare(TransferJob& j) {
    const DistMatrix& A = *j.A;
    DistMatrix& B = *j.B;
    const Grid& g = A.G();
    const int p = g.Size(), me = g.VCRank();
    const DType t = A.Type();
    const Device dev = B.Dev();
    const size_t es = A.ElemSize();
    hipStream_t st = B.Stream();
    Fence(A, B);

    auto sends_to = [&](int s, int d) { return j.contract ? A.ParticipatingOf(s) : Designated(A, s, d); };
    for (int s = 0; s < p && !j.cross; ++s)
        for (int d = 0; d < p && !j.cross; ++d)
            if (s != d && sends_to(s, d) && Plan(A, B, s, d).count() > 0) j.cross = true;

    j.out.assign(p, PairPlan{});
    j.in.assign(p, PairPlan{});
    j.sc.assign(p, 0); j.sd.assign(p, 0); j.rc.assign(p, 0); j.rd.assign(p, 0);
    Int stot = 0, rtot = 0;
    for (int q = 0; q < p; ++q) {
        if (sends_to(me, q)) j.out[q] = Plan(A, B, me, q);
        if (sends_to(q, me)) j.in[q] = Plan(A, B, q, me);
        if (q == me) continue;
        j.sc[q] = j.out[q].count(); j.sd[q] = stot; stot += j.sc[q];
        j.rc[q] = j.in[q].count();  j.rd[q] = rtot; rtot += j.rc[q];
    }
    if (j.cross) {
        j.sbuf.Reset(dev, static_cast<size_t>(stot) * es, st);
        j.rbuf.Reset(dev, static_cast<size_t>(rtot) * es, st);
        std::vector<kern::Copy2D> pack;
        for (int q = 0; q < p; ++q) {
            if (q == me || j.sc[q] == 0) continue;
            const PairPlan& pl = j.out[q];
            pack.push_back({pl.rows.count, pl.cols.count, At(A, pl.rows.src0, pl.cols.src0), pl.rows.src_step,
                            pl.cols.src_step * A.LDim(), static_cast<char*>(j.sbuf.data()) + j.sd[q] * es, 1,
                            pl.rows.count});
        }
        exec::Copy2DBatch(dev, t, pack.data(), static_cast<int>(pack.size()), false, 0.0, st);
    }
    // the local portion moves directly (never through the send buffer)
    if (!j.contract && j.out[me].count() > 0) {
        const PairPlan& pl = j.out[me];
        kern::Copy2D d{pl.rows.count, pl.cols.count, At(A, pl.rows.src0, pl.cols.src0), pl.rows.src_step,
                       pl.cols.src_step * A.LDim(), At(B, pl.rows.dst0, pl.cols.dst0), pl.rows.dst_step,
                       pl.cols.dst_step * B.LDim()};
        exec::Copy2DBatch(dev, t, &d, 1, false, 0.0, st);
    }
}

void TransferFinish(TransferJob& j) {
    const DistMatrix& A = *j.A;
    DistMatrix& B = *j.B;
    const int p = A.G().Size(), me = A.G().VCRank();
    const DType t = A.Type();
    const Device dev = B.Dev();
    const size_t es = A.ElemSize();
    hipStream_t st = B.Stream();
    auto unpack_desc = [&](int q) {
        const PairPlan& pl = j.in[q];
        return kern::Copy2D{pl.rows.count, pl.cols.count, static_cast<char*>(j.rbuf.data()) + j.rd[q] * es, 1,
                            pl.rows.count, At(B, pl.rows.dst0, pl.cols.dst0), pl.rows.dst_step,
                            pl.cols.dst_step * B.LDim()};
    };
    if (!j.contract) {
        std::vector<kern::Copy2D> unpack;
        for (int q = 0; q < p; ++q)
            if (q != me && j.rc[q] > 0) unpack.push_back(unpack_desc(q));
        exec::Copy2DBatch(dev, t, unpack.data(), static_cast<int>(unpack.size()), false, 0.0, st);
    } else {
        // sum contributions in rank order (deterministic).  When every source
        // covers the same destination pattern (the reduce-scatters of SUMMA_A /
        // B / Dot: each source holds all of what the receiver owns) one launch
        // reads every portion and B once (AxpyContract.hpp:475-478's single
        // InterleaveMatrixUpdate); otherwise one axpy launch per source, so two
        // sources never update the same element concurrently.  Both round to the
        // storage type after each source: identical results.
        std::vector<int> srcs;
        for (int q = 0; q < p; ++q)
            if (q == me ? j.in[me].count() > 0 : j.rc[q] > 0) srcs.push_back(q);
        auto same_dst = [&](const PairPlan& a, const PairPlan& b) {
            return a.rows.count == b.rows.count && a.cols.count == b.cols.count && a.rows.dst0 == b.rows.dst0 &&
                   a.cols.dst0 == b.cols.dst0 && a.rows.dst_step == b.rows.dst_step &&
                   a.cols.dst_step == b.cols.dst_step;
        };
        bool fused = srcs.size() > 1;
        for (size_t i = 1; i < srcs.size() && fused; ++i) fused = same_dst(j.in[srcs[0]], j.in[srcs[i]]);
        auto source_desc = [&](int q) {
            if (q == me) {
                const PairPlan& pl = j.in[me];
                return kern::Copy2D{pl.rows.count, pl.cols.count, At(A, pl.rows.src0, pl.cols.src0), pl.rows.src_step,
                                    pl.cols.src_step * A.LDim(), At(B, pl.rows.dst0, pl.cols.dst0), pl.rows.dst_step,
                                    pl.cols.dst_step * B.LDim()};
            }
            return unpack_desc(q);
        };
        if (fused) {
            std::vector<exec::ContractSource> cs;
            for (int q : srcs) {
                const kern::Copy2D d = source_desc(q);
                cs.push_back({d.src, d.scs, d.srs});
            }
            const kern::Copy2D d0 = source_desc(srcs[0]);
            exec::ContractSum(dev, t, d0.m, d0.n, d0.dst, d0.dcs, d0.drs, cs.data(), static_cast<int>(cs.size()),
                              j.alpha, st);
        } else {
            for (int q : srcs) {
                const kern::Copy2D d = source_desc(q);
                exec::Copy2DBatch(dev, t, &d, 1, true, j.alpha, st);
            }
        }
    }
    // sbuf/rbuf return to the pool stream-ordered on B's stream
}

Comm::VSet ExchangeOf(TransferJob& j) {
    return Comm::VSet{j.A->Type(), j.sbuf.data(), &j.sc, &j.sd, j.rbuf.data(), &j.rc, &j.rd};
}

void Transfer(const DistMatrix& A, DistMatrix& B, bool contract, double alpha) {
    TransferJob j{&A, &B, contract, alpha};
    TransferPrepare(j);
    if (j.cross) A.G().VC().AllToAllV(A.Type(), j.sbuf.data(), j.sc, j.sd, j.rbuf.data(), j.rc, j.rd, B.Dev(), B.Stream());
    TransferFinish(j);
}

void LocalTransposeInto(const DistMatrix& A, DistMatrix& T) {
    // T's local block is A's local block transposed
    if (T.LocalHeight() == 0 || T.LocalWidth() == 0) return;
    kern::Copy2D d{T.LocalHeight(), T.LocalWidth(), A.Buffer(), A.LDim(), 1, T.Buffer(), 1, T.LDim()};
    Fence(A, T);
    exec::Copy2DBatch(T.Dev(), T.Type(), &d, 1, false, 0.0, T.Stream());
}

std::shared_ptr<DistMatrix> LocalTransposed(const DistMatrix& A) {
    auto T = A.Like(A.RowDist(), A.ColDist());
    T->Align(A.RowAlign(), A.ColAlign(), true);
    T->Resize(A.Width(), A.Height());
    LocalTransposeInto(A, *T);
    return T;
}

}  // namespace

bool SameLocalLayout(const DistMatrix& A, Dist cd, Dist rd, int calign, int ralign) {
    const Grid& g = A.G();
    if (A.ColDist() == Dist::CIRC || cd == Dist::CIRC) return false;
    // root-dependent participation: never reinterpret in place
    if (A.ColDist() == Dist::MD || A.RowDist() == Dist::MD || cd == Dist::MD || rd == Dist::MD) return false;
    if (g.Stride(cd) != A.ColStride() || g.Stride(rd) != A.RowStride()) return false;
    for (int q = 0; q < g.Size(); ++q) {
        if (Shift(g.DistRankOf(cd, q), calign, g.Stride(cd)) != Shift(A.ColRankOf(q), A.ColAlign(), A.ColStride()))
            return false;
        if (Shift(g.DistRankOf(rd, q), ralign, g.Stride(rd)) != Shift(A.RowRankOf(q), A.RowAlign(), A.RowStride()))
            return false;
    }
    return true;
}

// El::Copy(ElementalMatrix<S> const& A, DistMatrix<T,U,V>& B) with S != T
// (include/El/blas_like/level1/CopyDistMatrix.hpp:28-57): when A already has
// B's distribution, root and (adoptable) alignment, convert the local block in
// place of a redistribution; otherwise redistribute in S to a temporary aligned
// with B, then convert locally.
void CopyConvert(const DistMatrix& A, DistMatrix& B) {
    ELX_REQUIRE(&A.G() == &B.G(), "matrices live on different grids");
    const DistMatrix* src = &A;
    std::shared_ptr<DistMatrix> T;
    bool direct = false;
    if (A.ColDist() == B.ColDist() && A.RowDist() == B.RowDist() && A.Dev() == B.Dev() && A.Root() == B.Root()) {
        if (!B.Viewing()) {
            if (!B.ColConstrained()) B.AlignCols(A.ColAlign(), false);
            if (!B.RowConstrained()) B.AlignRows(A.RowAlign(), false);
        }
        direct = A.ColAlign() == B.ColAlign() && A.RowAlign() == B.RowAlign();
    }
    if (!direct) {
        T = std::make_shared<DistMatrix>(A.GridPtr(), A.Type(), B.ColDist(), B.RowDist(), B.Dev(), B.Root());
        T->Align(B.ColAlign(), B.RowAlign(), true);
        T->SetStream(B.Stream());  // produced, consumed and released on B's stream
        Copy(A, *T);
        src = T.get();
    }
    B.Resize(A.Height(), A.Width());
    if (B.LocalHeight() == 0 || B.LocalWidth() == 0) return;
    Fence(*src, B);
    kern::Copy2D d{B.LocalHeight(), B.LocalWidth(), src->Buffer(), 1, src->LDim(), B.Buffer(), 1, B.LDim()};
    exec::Convert2D(B.Dev(), src->Type(), B.Type(), d, B.Stream());
}

void Copy(const DistMatrix& A, DistMatrix& B) {
    ELX_TRACE("El::Copy (redistribution)");
    if (A.Type() != B.Type()) { CopyConvert(A, B); return; }
    CheckCompatible(A, B);
    if (A.Dev() != B.Dev()) {
        auto T = OnDevice(A, B.Dev(), B.Stream());
        Copy(*T, B);
        return;
    }
    PrepareTarget(A, B);
    if (B.Height() == 0 || B.Width() == 0) return;
    Transfer(A, B, false, 0.0);
}

void CopyGroup(const std::vector<std::pair<const DistMatrix*, DistMatrix*>>& pairs) {
    // one shared exchange only when every pair is a same-type, same-device
    // redistribution on one grid with its target on one stream
    bool group = pairs.size() > 1;
    for (const auto& pr : pairs) {
        const DistMatrix& A = *pr.first;
        DistMatrix& B = *pr.second;
        group = group && A.Type() == B.Type() && A.Dev() == B.Dev() && &A.G() == &pairs[0].first->G() &&
                &B.G() == &A.G() && B.Stream() == pairs[0].second->Stream();
    }
    if (!group) {
        for (const auto& pr : pairs) Copy(*pr.first, *pr.second);
        return;
    }
    ELX_TRACE("El::Copy (grouped redistributions)");
    std::vector<TransferJob> jobs;
    jobs.reserve(pairs.size());
    for (const auto& pr : pairs) {
        CheckCompatible(*pr.first, *pr.second);
        PrepareTarget(*pr.first, *pr.second);
        if (pr.second->Height() == 0 || pr.second->Width() == 0) continue;
        jobs.push_back(TransferJob{pr.first, pr.second, false, 0.0});
    }
    for (auto& j : jobs) TransferPrepare(j);
    std::vector<Comm::VSet> sets;
    for (auto& j : jobs)
        if (j.cross) sets.push_back(ExchangeOf(j));
    if (!sets.empty()) jobs[0].A->G().VC().AllToAllVGroup(sets, jobs[0].B->Dev(), jobs[0].B->Stream());
    for (auto& j : jobs) TransferFinish(j);
}

void Transpose(const DistMatrix& A, DistMatrix& B) {
    CheckCompatible(A, B);
    if (A.Dev() == B.Dev() && B.ColDist() == A.RowDist() && B.RowDist() == A.ColDist()) {
        // direct local transpose when B can hold A^T with matching alignment
        const bool colOk = B.Viewing() || B.ColConstrained() ? B.ColAlign() == A.RowAlign() : true;
        const bool rowOk = B.Viewing() || B.RowConstrained() ? B.RowAlign() == A.ColAlign() : true;
        if (colOk && rowOk) {
            if (!B.Viewing()) {
                if (!B.ColConstrained()) B.AlignCols(A.RowAlign(), false);
                if (!B.RowConstrained()) B.AlignRows(A.ColAlign(), false);
            }
            B.Resize(A.Width(), A.Height());
            LocalTransposeInto(A, B);
            return;
        }
    }
    auto T = LocalTransposed(A);
    Copy(*T, B);
}

void AxpyContract(double alpha, const DistMatrix& A, DistMatrix& B) {
    CheckCompatible(A, B);
    ELX_REQUIRE(A.Height() == B.Height() && A.Width() == B.Width(), "AxpyContract: ", A.Height(), "x", A.Width(),
                " vs ", B.Height(), "x", B.Width());
    if (A.Dev() != B.Dev()) {
        auto T = OnDevice(A, B.Dev(), B.Stream());
        AxpyContract(alpha, *T, B);
        return;
    }
    if (B.Height() == 0 || B.Width() == 0) return;
    Transfer(A, B, true, alpha);
}

void TransposeAxpyContract(double alpha, const DistMatrix& A, DistMatrix& B) {
    auto T = LocalTransposed(A);
    AxpyContract(alpha, *T, B);
}

void Axpy(double alpha, const DistMatrix& X, DistMatrix& Y) {
    CheckCompatible(X, Y);
    ELX_REQUIRE(X.Height() == Y.Height() && X.Width() == Y.Width(), "Axpy: nonconformal ", X.Height(), "x",
                X.Width(), " vs ", Y.Height(), "x", Y.Width());
    if (X.Dev() == Y.Dev() && X.ColDist() == Y.ColDist() && X.RowDist() == Y.RowDist() &&
        X.ColAlign() == Y.ColAlign() && X.RowAlign() == Y.RowAlign()) {
        if (Y.LocalHeight() == 0 || Y.LocalWidth() == 0) return;
        kern::Copy2D d{Y.LocalHeight(), Y.LocalWidth(), X.Buffer(), 1, X.LDim(), Y.Buffer(), 1, Y.LDim()};
        Fence(X, Y);
        exec::Copy2DBatch(Y.Dev(), Y.Type(), &d, 1, true, alpha, Y.Stream());
        return;
    }
    auto T = Y.Like(Y.ColDist(), Y.RowDist());
    T->Align(Y.ColAlign(), Y.RowAlign(), true);
    Copy(X, *T);
    Axpy(alpha, *T, Y);
}

void Zero(DistMatrix& A) {
    if (A.LocalHeight() == 0 || A.LocalWidth() == 0) return;
    exec::Fill(A.Dev(), A.Type(), A.LocalHeight(), A.LocalWidth(), 0.0, A.Buffer(), A.LDim(), A.Stream());
}

void Scale(double alpha, DistMatrix& A) {  // include/El/blas_like/level1/Scale.hpp:18-31
    if (alpha == 0.0) { Zero(A); return; }
    if (alpha == 1.0) return;
    if (A.LocalHeight() == 0 || A.LocalWidth() == 0) return;
    exec::Scale(A.Dev(), A.Type(), A.LocalHeight(), A.LocalWidth(), alpha, A.Buffer(), A.LDim(), A.Stream());
}

void Hadamard(const DistMatrix& A, const DistMatrix& B, DistMatrix& C) {  // Hadamard.hpp:107-131
    CheckCompatible(A, B);
    CheckCompatible(A, C);
    ELX_REQUIRE(A.ColDist() == B.ColDist() && A.RowDist() == B.RowDist() && A.ColDist() == C.ColDist() &&
                    A.RowDist() == C.RowDist(), "Hadamard: A, B and C must share a distribution");
    ELX_REQUIRE(A.ColAlign() == B.ColAlign() && A.RowAlign() == B.RowAlign(), "Hadamard: A and B not aligned");
    ELX_REQUIRE(A.Height() == B.Height() && A.Width() == B.Width(), "Hadamard: nonconformal");
    ELX_REQUIRE(A.Dev() == B.Dev() && A.Dev() == C.Dev(), "Hadamard: mixed devices");
    if (&C != &A && &C != &B) {
        if (!C.Viewing()) {
            if (!C.ColConstrained()) C.AlignCols(A.ColAlign(), false);
            if (!C.RowConstrained()) C.AlignRows(A.RowAlign(), false);
        }
        ELX_REQUIRE(C.ColAlign() == A.ColAlign() && C.RowAlign() == A.RowAlign(), "Hadamard: C not aligned");
        C.Resize(A.Height(), A.Width());
    }
    if (C.LocalHeight() == 0 || C.LocalWidth() == 0) return;
    Fence(A, C);
    Fence(B, C);
    exec::Hadamard(C.Dev(), C.Type(), C.LocalHeight(), C.LocalWidth(), A.Buffer(), A.LDim(), B.Buffer(), B.LDim(),
                   C.Buffer(), C.LDim(), C.Stream());
}

void EntrywiseMap(int fn, const DistMatrix& A, DistMatrix& B) {  // EntrywiseMap.hpp:90-137
    CheckCompatible(A, B);
    const DistMatrix* src = &A;
    std::shared_ptr<DistMatrix> T;
    if (A.ColDist() == B.ColDist() && A.RowDist() == B.RowDist() && A.Dev() == B.Dev()) {
        if (!B.Viewing()) {
            if (!B.ColConstrained()) B.AlignCols(A.ColAlign(), false);
            if (!B.RowConstrained()) B.AlignRows(A.RowAlign(), false);
        }
    }
    if (!(A.ColDist() == B.ColDist() && A.RowDist() == B.RowDist() && A.ColAlign() == B.ColAlign() &&
          A.RowAlign() == B.RowAlign() && A.Dev() == B.Dev())) {
        T = B.Like(B.ColDist(), B.RowDist());
        T->Align(B.ColAlign(), B.RowAlign(), true);
        Copy(A, *T);
        src = T.get();
    }
    B.Resize(A.Height(), A.Width());
    if (B.LocalHeight() == 0 || B.LocalWidth() == 0) return;
    Fence(*src, B);
    exec::Map(B.Dev(), B.Type(), fn, B.LocalHeight(), B.LocalWidth(), src->Buffer(), src->LDim(), B.Buffer(),
              B.LDim(), B.Stream());
}

void Combine(int fn, const DistMatrix& A, DistMatrix& B) {
    if (A.Height() != B.Height() || A.Width() != B.Width())
        throw RuntimeError("A and B must be the same size for Combine.");
    CheckCompatible(A, B);
    ELX_REQUIRE(A.ColDist() == B.ColDist() && A.RowDist() == B.RowDist() && A.ColAlign() == B.ColAlign() &&
                    A.RowAlign() == B.RowAlign() && A.Dev() == B.Dev(),
                "Combine: A and B must share distribution, alignment and device");
    if (B.LocalHeight() == 0 || B.LocalWidth() == 0) return;
    Fence(A, B);
    exec::Combine(B.Dev(), B.Type(), fn, B.LocalHeight(), B.LocalWidth(), A.Buffer(), A.LDim(), B.Buffer(), B.LDim(),
                  B.Stream());
}

// ---------------------------------------------------------------------------
// Entry access (ElementMatrix/setup.hpp:463-610) and grid-wide scalars.
// ---------------------------------------------------------------------------
namespace {

// one double through a grid communicator: device buffers when the comm is RCCL
template <typename F>
double ScalarColl(const Grid& g, double v, F&& coll) {
    if (g.Size() == 1) return v;
    if (g.CommDevice() == Device::GPU) {
        hipStream_t s = Runtime::Get().CommStream();
        elx::Buffer b(Device::GPU, sizeof(double), s);
        ELX_CHECK_HIP(hipMemcpyAsync(b.data(), &v, sizeof(double), hipMemcpyHostToDevice, s));
        coll(b.data(), Device::GPU, s);
        ELX_CHECK_HIP(hipMemcpyAsync(&v, b.data(), sizeof(double), hipMemcpyDeviceToHost, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
        return v;
    }
    coll(&v, Device::CPU, nullptr);
    return v;
}

// does rank vc hold global entry (i, j) of A?
bool HoldsOf(const DistMatrix& A, int vc, Int i, Int j) {
    if (!A.ParticipatingOf(vc)) return false;
    const Int cs = Shift(A.ColRankOf(vc), A.ColAlign(), A.ColStride());
    const Int rs = Shift(A.RowRankOf(vc), A.RowAlign(), A.RowStride());
    return Mod(i - cs, A.ColStride()) == 0 && Mod(j - rs, A.RowStride()) == 0;
}

char* LocalEntry(const DistMatrix& A, Int i, Int j) {
    const Int iLoc = (i - A.ColShift()) / A.ColStride(), jLoc = (j - A.RowShift()) / A.RowStride();
    return At(A, iLoc, jLoc);
}

double ReadEntry(const DistMatrix& A, const char* p) {
    alignas(8) unsigned char tmp[8];
    const size_t es = A.ElemSize();
    if (A.Dev() == Device::GPU) {
        ELX_CHECK_HIP(hipMemcpyAsync(tmp, p, es, hipMemcpyDeviceToHost, A.Stream()));
        ELX_CHECK_HIP(hipStreamSynchronize(A.Stream()));
    } else {
        std::memcpy(tmp, p, es);
    }
    return exec::LoadScalar(A.Type(), tmp);
}

void WriteEntry(DistMatrix& A, char* p, double v) {
    alignas(8) unsigned char tmp[8];
    exec::StoreScalar(A.Type(), tmp, v);
    const size_t es = A.ElemSize();
    if (A.Dev() == Device::GPU) {
        ELX_CHECK_HIP(hipMemcpyAsync(p, tmp, es, hipMemcpyHostToDevice, A.Stream()));
        ELX_CHECK_HIP(hipStreamSynchronize(A.Stream()));
    } else {
        std::memcpy(p, tmp, es);
    }
}

void CheckIndex(const DistMatrix& A, Int i, Int j) {
    ELX_REQUIRE(i >= 0 && i < A.Height() && j >= 0 && j < A.Width(), "entry (", i, ",", j,
                ") out of bounds of ", A.Height(), " x ", A.Width());
}

}  // namespace

double GridAllReduceSum(const Grid& g, double v) {
    return ScalarColl(g, v, [&](void* p, Device d, hipStream_t s) { g.VC().AllReduce(DType::F64, p, p, 1, d, s); });
}

// max over the grid (NaN wins): every rank's value gathered over VC
double GridAllReduceMax(const Grid& g, double v) {
    const int p = g.Size();
    if (p == 1) return v;
    std::vector<double> all(p);
    if (g.CommDevice() == Device::GPU) {
        hipStream_t s = Runtime::Get().CommStream();
        elx::Buffer b(Device::GPU, sizeof(double) * (p + 1), s);
        double* d = static_cast<double*>(b.data());
        ELX_CHECK_HIP(hipMemcpyAsync(d, &v, sizeof(double), hipMemcpyHostToDevice, s));
        g.VC().AllGather(DType::F64, d, d + 1, 1, Device::GPU, s);
        ELX_CHECK_HIP(hipMemcpyAsync(all.data(), d + 1, sizeof(double) * p, hipMemcpyDeviceToHost, s));
        ELX_CHECK_HIP(hipStreamSynchronize(s));
    } else {
        g.VC().AllGather(DType::F64, &v, all.data(), 1, Device::CPU, nullptr);
    }
    double r = all[0];
    for (double x : all) r = r != r ? r : x != x ? x : std::max(r, x);
    return r;
}

double GridBcast(const Grid& g, double v, int rootVC) {
    return ScalarColl(g, v, [&](void* p, Device d, hipStream_t s) { g.VC().Bcast(DType::F64, p, 1, rootVC, d, s); });
}

// El::DistMatrix::Get (ElementMatrix/setup.hpp:463-490): collective over the
// grid; the lowest VC rank holding (i, j) reads it and broadcasts it.
double Get(const DistMatrix& A, Int i, Int j) {
    CheckIndex(A, i, j);
    const Grid& g = A.G();
    int owner = -1;
    for (int q = 0; q < g.Size() && owner < 0; ++q)
        if (HoldsOf(A, q, i, j)) owner = q;
    double v = 0.0;
    if (owner == g.VCRank()) v = ReadEntry(A, LocalEntry(A, i, j));
    return GridBcast(g, v, owner);
}

// El::DistMatrix::Set / Update (setup.hpp:552-604): every rank holding (i, j)
// writes its copy; no communication.
void Set(DistMatrix& A, Int i, Int j, double v) {
    CheckIndex(A, i, j);
    if (HoldsOf(A, A.G().VCRank(), i, j)) WriteEntry(A, LocalEntry(A, i, j), v);
}

void Update(DistMatrix& A, Int i, Int j, double v) {
    CheckIndex(A, i, j);
    if (!HoldsOf(A, A.G().VCRank(), i, j)) return;
    char* p = LocalEntry(A, i, j);
    WriteEntry(A, p, ReadEntry(A, p) + v);
}

// El::Fill (include/El/blas_like/level1/Fill.hpp:20-70): every local entry := v
void Fill(DistMatrix& A, double v) {
    if (A.LocalHeight() == 0 || A.LocalWidth() == 0) return;
    exec::Fill(A.Dev(), A.Type(), A.LocalHeight(), A.LocalWidth(), v, A.Buffer(), A.LDim(), A.Stream());
}

// El::FrobeniusNorm (src/lapack_like/props/Norm/Frobenius.cpp:20-60): the
// reference's scaled sum of squares (UpdateScaledSquare) with one scale, the
// grid-wide max |a|, so no entry overflows or underflows the squares; both
// passes are device reductions over the local block.  Replicated copies of a
// local block (e.g. [STAR,STAR]) count once.
double FrobeniusNorm(const DistMatrix& A) {
    const Int lh = A.LocalHeight(), lw = A.LocalWidth();
    const bool mine = A.Participating() && lh > 0 && lw > 0;
    const double amax = GridAllReduceMax(
        A.G(), mine ? exec::AbsMax(A.Dev(), A.Type(), lh, lw, A.Buffer(), A.LDim(), A.Stream()) : 0.0);
    if (amax == 0.0 || !std::isfinite(amax)) return amax;
    double local = 0.0;
    if (mine) {
        local = exec::ScaledSumSq(A.Dev(), A.Type(), lh, lw, A.Buffer(), A.LDim(), amax, A.Stream());
        int copies = 0;  // ranks holding this same local block (replicated distributions)
        for (int q = 0; q < A.G().Size(); ++q)
            if (A.ColRankOf(q) == A.ColRank() && A.RowRankOf(q) == A.RowRank()) ++copies;
        local /= copies;
    }
    return amax * std::sqrt(GridAllReduceSum(A.G(), local));
}

// Trsm's checkIfSingular (src/blas_like/level3/Trsm.cpp:60-68): is any diagonal
// entry of A exactly zero?  The local diagonal entries form one arithmetic
// progression (global index step lcm(colStride, rowStride)), gathered by one
// strided copy; the per-rank answers are summed over the grid.
bool DiagonalHasZero(const DistMatrix& A) {
    const Int n = std::min(A.Height(), A.Width());
    double zeros = 0;
    if (A.Participating() && n > 0) {
        const Int cs = A.ColShift(), rs = A.RowShift(), cstr = A.ColStride(), rstr = A.RowStride();
        const Int L = cstr / Gcd(cstr, rstr) * rstr;
        Int z = -1;
        for (Int t = cs; t < cs + L; t += cstr)
            if (Mod(t - rs, rstr) == 0) { z = t; break; }
        const Int count = z < 0 ? 0 : Length(n, z, L);
        if (count > 0) {
            const size_t es = A.ElemSize();
            std::vector<unsigned char> host(count * es);
            const Int step = L / cstr + (L / rstr) * A.LDim();
            elx::Buffer tmp(A.Dev(), count * es, A.Stream());
            kern::Copy2D d{count, 1, At(A, (z - cs) / cstr, (z - rs) / rstr), step, 0, tmp.data(), 1, count};
            exec::Copy2DBatch(A.Dev(), A.Type(), &d, 1, false, 0.0, A.Stream());
            if (A.Dev() == Device::GPU) {
                ELX_CHECK_HIP(hipMemcpyAsync(host.data(), tmp.data(), count * es, hipMemcpyDeviceToHost, A.Stream()));
                ELX_CHECK_HIP(hipStreamSynchronize(A.Stream()));
            } else {
                std::memcpy(host.data(), tmp.data(), count * es);
            }
            for (Int q = 0; q < count; ++q)
                if (exec::LoadScalar(A.Type(), host.data() + q * es) == 0.0) zeros += 1;
        }
    }
    return GridAllReduceSum(A.G(), zeros) > 0;
}

}  // namespace elx
