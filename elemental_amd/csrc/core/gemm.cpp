// SUMMA drivers for El::Gemm on DistMatrices.
//
// Mirrors src/blas_like/level3/Gemm.cpp:273-302 (front door: Scale(beta,C) then
// dispatch on orientation) and src/blas_like/level3/Gemm/{NN,NT,TN,TT}.hpp
// (A-, B-, C-stationary and Dot variants + the 2/10 weight heuristic).
//
// What is MI355X-specific:
//  * C-stationary (the hot path, configs C1/C2/C3): every panel gather is a
//    single-hop redistribution (redist.cpp) straight into the layout the local
//    MFMA update reads ([MC,*] and [*,MR] for NN - no transpose pass), enqueued
//    on a dedicated high-priority comm stream into one of two panel slots while
//    the MFMA kernel consumes the other slot on the compute stream (event
//    fenced both ways).  This is what the reference's off-by-default
//    multistream variants approximate (NN_Multistream.hpp:262-412) without
//    their S extra copies of C.
//  * communication panel (Blocksize(), default 128) and compute panel are
//    decoupled: ComputePanel() consecutive columns of A / rows of B are moved
//    per step (EffectivePanel: K/8 for f64/f32, K/4 for f16/bf16, clamped to
//    [2048, 8192]; whole k on a 1x1 grid where the "gathers" are local
//    views), so the fp64 update runs at k >= 2048 instead of k = 128 and
//    C's HBM round trip per panel stays a few % of the MFMA time.  Only the
//    summation order changes (normwise tolerance); data movement is bit-exact.
//  * the _MS algorithm ids are the reference's multistream variants: with a
//    stream pool (H_STREAMPOOL_SIZE > 1) panels round-robin over teams, each with
//    its own stream and duplicated RCCL communicators (SummaCMultistream,
//    SummaA/SummaB with teams); NT/TN included (the reference's ROCm build
//    rejects those, TN.hpp:124-128).
#include "gemm.hpp"
#include <cstdlib>
#include "redist.hpp"
#include "exec.hpp"
#include <algorithm>
#include <functional>
#include "../runtime/trace.hpp"
#include <initializer_list>
#include <vector>

namespace elx {

namespace {
// the algorithmic blocksize stack (src/blas_like/blocksizes.cpp:16,38-72);
// Initialize() leaves one entry, 128 (src/core/environment.cpp:314-315)
std::vector<Int>& BlocksizeStack() {
    static std::vector<Int> s{128};
    return s;
}
Int g_compute_panel = 0;    // 0 = automatic
int g_last_alg = ELX_GEMM_DEFAULT;
constexpr Int kDotBlock = 2000;  // NN.hpp:578 (hard-coded in the reference)
// On the GPU the Dot block is 2048, the reference's 2000 rounded up to the
// 128-wide tile grid: a C block's elements are the same k-sums whatever the
// m/n blocking, and 2000-wide blocks leave a ragged last tile per block and
// 192-wide remainders (C4's 8192 = 4 x 2000 + 192).  C4 on one MI355X: 2000 ->
// 124.4 TF, 2048 -> 131.1, 4096 -> 120.9, 8192 -> 121.4 (fewer, longer-k
// launches over more tiles run slower: profiles/r01_dot_block.log).
constexpr Int kDotBlockGPU = 2048;
Int DotBlockGPU() {  // ELX_DOT_BLOCK overrides (tuning experiments)
    static const Int v = [] { const char* e = getenv("ELX_DOT_BLOCK"); return e ? (Int)atoll(e) : kDotBlockGPU; }();
    return v;
}

bool IsN(int o) { return o == ELX_NORMAL; }

// Event-bracketed profiling of the local updates and panel transfers.
struct Profiler {
    struct Rec { hipEvent_t a, b; double work; int call = -1; };
    bool on = false;
    int calls = 0;  // SummaC invocations (groups consecutive panel updates)
    std::vector<Rec> gemm, comm;
    void Clear() {
        for (auto* v : {&gemm, &comm})
            for (auto& r : *v) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
        gemm.clear();
        comm.clear();
    }
    Rec Begin(hipStream_t s) {
        Rec r{};
        ELX_CHECK_HIP(hipEventCreate(&r.a));
        ELX_CHECK_HIP(hipEventCreate(&r.b));
        ELX_CHECK_HIP(hipEventRecord(r.a, s));
        return r;
    }
    void End(Rec r, hipStream_t s, double work, std::vector<Rec>& into, int call = -1) {
        ELX_CHECK_HIP(hipEventRecord(r.b, s));
        r.work = work;
        r.call = call;
        into.push_back(r);
    }
};
Profiler& Prof() {
    static Profiler p;
    return p;
}

void FenceStreams(hipStream_t from, hipStream_t to) {
    if (!from || !to || from == to) return;
    hipEvent_t ev;
    ELX_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ELX_CHECK_HIP(hipEventRecord(ev, from));
    ELX_CHECK_HIP(hipStreamWaitEvent(to, ev, 0));
    ELX_CHECK_HIP(hipEventDestroy(ev));
}

// MultiSync (include/hydrogen/MultiSync.hpp:33-78): on entry the master stream
// waits for the others' queued work; on exit the others wait for the master, so
// a caller that reuses A or B on its own stream, and every temporary released
// on those streams, is ordered after the reads issued here.
class MultiSync {
public:
    MultiSync(hipStream_t master, std::initializer_list<hipStream_t> others) : master_(master), others_(others) {
        for (hipStream_t o : others_) FenceStreams(o, master_);
    }
    ~MultiSync() {
        for (hipStream_t o : others_) {
            try { FenceStreams(master_, o); } catch (...) {}
        }
    }
    MultiSync(const MultiSync&) = delete;
    MultiSync& operator=(const MultiSync&) = delete;

private:
    hipStream_t master_;
    std::vector<hipStream_t> others_;
};

// DistMatrixReadProxy<T,T,cd,rd,ELEMENT,D> (include/El/core/Proxy.hpp:174-300):
// the operands are brought to the device of `tgt` (the matrix being written,
// as Gemm/NN.hpp:357-359 proxies A and B onto C's device) and every read is
// queued on tgt's stream.  A itself (as a view on that stream) when it already
// has dist (cd,rd), that device [and the requested alignment]; else a
// redistributed copy, moved across devices when needed.
std::shared_ptr<const DistMatrix> ReadProxy(const DistMatrix& A, const DistMatrix& tgt, Dist cd, Dist rd,
                                            int calign = -1, int ralign = -1) {
    const bool ok = A.Dev() == tgt.Dev() && A.ColDist() == cd && A.RowDist() == rd &&
                    (calign < 0 || A.ColAlign() == calign) && (ralign < 0 || A.RowAlign() == ralign);
    if (ok) {
        if (A.Dev() != Device::GPU || A.Stream() == tgt.Stream())
            return std::shared_ptr<const DistMatrix>(&A, [](const DistMatrix*) {});
        auto V = DistMatrix::View(A, 0, A.Height(), 0, A.Width());
        V->SetStream(tgt.Stream());
        return V;
    }
    auto T = A.LikeOn(cd, rd, tgt.Dev());
    T->SetStream(tgt.Stream());
    // A's local block already holds exactly the (cd,rd) block on every rank
    // (e.g. [MC,MR] -> [VC,*] on a 1x1 grid): relabel it in place, no copy
    const int ca = calign >= 0 ? calign : 0, ra = ralign >= 0 ? ralign : 0;
    if (A.Dev() == tgt.Dev() && A.Root() == 0 && SameLocalLayout(A, cd, rd, ca, ra)) {
        T->Attach(A.Height(), A.Width(), ca, ra, const_cast<void*>(A.Buffer()), A.LDim(), 0);
        if (A.Dev() == Device::GPU) FenceStreams(A.Stream(), tgt.Stream());
        return T;
    }
    if (calign >= 0) T->AlignCols(calign, true);
    if (ralign >= 0) T->AlignRows(ralign, true);
    Copy(A, *T);
    return T;
}

// DistMatrixReadWriteProxy for C: work in [MC,MR]; copy back on Finish().
struct RWProxy {
    DistMatrix& orig;
    std::shared_ptr<DistMatrix> tmp;
    explicit RWProxy(DistMatrix& C) : orig(C) {
        if (C.ColDist() != Dist::MC || C.RowDist() != Dist::MR) {
            tmp = C.Like(Dist::MC, Dist::MR);
            Copy(C, *tmp);
        }
    }
    DistMatrix& Get() { return tmp ? *tmp : orig; }
    void Finish() { if (tmp) Copy(*tmp, orig); }
};

void Check(bool cond, const char* what) {
    if (!cond) throw LogicError(Cat("LocalGemm: ", what));
}

// ---------------------------------------------------------------------------
// Multistream teams: hydrogen::SyncInfoPool (SyncInfoPool.hpp:23-195) and
// GetSyncInfoPool / InitializeComms (Gemm.cpp:17-90).  H_STREAMPOOL_SIZE
// streams, each with its own duplicate of the grid's communicators: an RCCL
// communicator's operations are ordered, so concurrent panels on different
// streams need different communicators (the reference gets one Aluminum
// communicator per SyncInfo the same way).  Built collectively, once per grid,
// on first use.  A host-backend grid (blocking collectives, program order) is
// shared by every team; only the streams differ.
// ---------------------------------------------------------------------------
int g_pool_size = -1;  // -1: read H_STREAMPOOL_SIZE (Gemm.cpp:22-29, default 1)

struct Team {
    std::shared_ptr<Grid> grid;
    hipStream_t stream = nullptr;
};
struct TeamSet {
    std::weak_ptr<Grid> base;
    std::vector<Team> teams;
};

std::vector<TeamSet>& TeamCache() {
    static auto* c = new std::vector<TeamSet>();  // leaked: outlives static destructors
    return *c;
}

const std::vector<Team>& Teams(const std::shared_ptr<Grid>& g, Device dev, int n) {
    auto& cache = TeamCache();
    for (auto it = cache.begin(); it != cache.end();) {  // drop teams of destroyed grids
        if (it->base.expired()) {
            for (auto& t : it->teams)
                if (t.stream) (void)hipStreamDestroy(t.stream);
            it = cache.erase(it);
        } else {
            ++it;
        }
    }
    TeamSet* ts = nullptr;
    for (auto& e : cache)
        if (e.base.lock() == g) ts = &e;
    if (!ts) {
        cache.push_back(TeamSet{g, {}});
        ts = &cache.back();
    }
    const bool gpu = dev == Device::GPU;
    while (static_cast<int>(ts->teams.size()) < n) {
        Team t;
        if (g->World().kind() == Comm::Kind::RCCL) {
            auto dup = g->WorldPtr()->Split(0, g->World().Rank());  // collective on every rank
            t.grid = std::make_shared<Grid>(dup, g->Height(), g->Order());
        } else {
            t.grid = g;
        }
        if (gpu) ELX_CHECK_HIP(hipStreamCreateWithFlags(&t.stream, hipStreamNonBlocking));
        ts->teams.push_back(t);
    }
    if (gpu)
        for (auto& t : ts->teams)
            if (!t.stream) ELX_CHECK_HIP(hipStreamCreateWithFlags(&t.stream, hipStreamNonBlocking));
    return ts->teams;
}

// Per-team views of the (proxied) operands: team t's A, B and C are views on
// its grid, queued on its stream, every team stream ordered after C's stream on
// entry.  S == 1: the operands themselves.
struct TeamViews {
    struct V {
        std::shared_ptr<const DistMatrix> A, B;
        std::shared_ptr<DistMatrix> C;
        hipStream_t s = nullptr;
    };
    std::vector<V> v;
    hipStream_t cs;
    TeamViews(const DistMatrix& A, const DistMatrix& B, DistMatrix& C, int S) : cs(C.Stream()) {
        if (S <= 1) {
            v.push_back({std::shared_ptr<const DistMatrix>(&A, [](const DistMatrix*) {}),
                         std::shared_ptr<const DistMatrix>(&B, [](const DistMatrix*) {}),
                         std::shared_ptr<DistMatrix>(&C, [](DistMatrix*) {}), cs});
            return;
        }
        const auto& teams = Teams(C.GridPtr(), C.Dev(), S);
        for (int t = 0; t < S; ++t) {
            V x;
            x.s = teams[t].stream;
            FenceStreams(cs, x.s);
            auto a = DistMatrix::ViewOn(A, teams[t].grid);
            auto b = DistMatrix::ViewOn(B, teams[t].grid);
            x.C = DistMatrix::ViewOn(C, teams[t].grid);
            a->SetStream(x.s);
            b->SetStream(x.s);
            x.C->SetStream(x.s);
            x.A = a;
            x.B = b;
            v.push_back(x);
        }
    }
    const V& operator[](Int p) const { return v[static_cast<size_t>(p % static_cast<Int>(v.size()))]; }
    // C's stream waits for every team
    void Join() const {
        for (auto& x : v) FenceStreams(x.s, cs);
    }
    // teams' temporaries are released on their streams: order them after C's
    ~TeamViews() {
        for (auto& x : v) {
            try { FenceStreams(cs, x.s); } catch (...) {}
        }
    }
};

// number of teams for `panels` panels (NN_Multistream.hpp:288-291: the pool
// size, at most one team per panel; a pool of one means no teams)
int TeamCount(const DistMatrix& C, Int panels) {
    const int pool = StreamPoolSize();
    if (C.Dev() != Device::GPU || pool <= 1) return 1;
    return static_cast<int>(std::max<Int>(1, std::min<Int>(pool, panels)));
}

Int EffectivePanel(const Grid& g, Int K, DType t) {
    const Int nb = std::max<Int>(1, Blocksize());
    Int kc = g_compute_panel;
    // automatic: C's HBM round trip per panel (read + write, 2s bytes per
    // element) against the panel's 2*kc FLOP per element.
    //  f64 / f32: K/8 in [2048, 8192]: C3 on one GPU (K = 65536) runs 72.9 TF at
    //    kc = 8192 vs 71.9 at 4096 (profiles/r02_trsm_kc.log); the deeper first
    //    panel's gather is cut to a quarter by SummaC's ramp.
    //  f16 / bf16: the MFMAs are 16-32x faster per element for only 4x fewer C
    //    bytes, so the round trip weighs ~8x more: K/4 in [2048, 8192]. C5's
    //    local panel on 2x4 (16384 x 8192 x kc bf16) runs 1058 / 1256 / 1390 /
    //    1458 TF at kc = 4096 / 8192 / 16384 / 32768 (profiles/r02_panel_depth.log);
    //    past 8192 the gather of the panel after the (quarter-depth) first one
    //    outgrows the first panel's update (each panel moves 8192*kc B per link
    //    at 2x4), which costs more than the deeper update gains at ~50 GB/s/link.
    const bool h16 = t == DType::F16 || t == DType::BF16;
    if (kc <= 0)
        kc = (g.Size() == 1) ? K : std::min<Int>(8192, std::max<Int>(2048, h16 ? K / 4 : K / 8));
    kc = std::max<Int>(nb, (kc + nb - 1) / nb * nb);  // whole communication panels
    return std::max<Int>(1, kc);
}

// ---------------------------------------------------------------------------
// LocalTrrk (Trrk/Local.hpp:124-300): C_loc += alpha op(a) op(b) on the part of
// C's local block whose GLOBAL index lies in the lower (gi >= gj) or upper
// (gi <= gj) triangle.  Local indices map monotonically to global ones, so the
// triangle is a staircase in local index space.  It is cut recursively (halving
// the column range): every rectangle entirely inside the triangle is one MFMA
// GEMM straight into C (beta = 1) - square-ish, large launches - and only the
// leaves on the diagonal (<= TrrkCols() = 1024 columns, rows rounded out to
// whole 128-row tiles) are computed into a
// workspace and folded in by the trapezoid kernel (the reference's "temporary
// copy" + AxpyTrapezoid, Local.hpp:155-163).  Rows entirely outside are never
// touched; the wasted FLOPs are half the leaves': ~TrrkCols() / 2n of the update.
// ---------------------------------------------------------------------------
constexpr Int kTrrkColsDefault = 1024;
Int TrrkCols() {  // ELX_TRRK_COLS overrides (tests exercise many ragged leaves)
    static const Int v = [] {
        const char* e = getenv("ELX_TRRK_COLS");
        return e && atoll(e) > 0 ? (Int)atoll(e) : kTrrkColsDefault;
    }();
    return v;
}

Int TrrkRowAlign() {  // ELX_TRRK_ROWS overrides (tests: 1 exercises every rectangle)
    static const Int v = [] {
        const char* e = getenv("ELX_TRRK_ROWS");
        return e && atoll(e) > 0 ? (Int)atoll(e) : Int(128);
    }();
    return v;
}

void TrrkLocal(bool lower, bool ta, bool tb, Int k, double alpha, const void* a, Int lda, const void* b, Int ldb,
               DistMatrix& C, hipStream_t s, Buffer& tmp) {
    const Int m = C.LocalHeight(), n = C.LocalWidth();
    if (m == 0 || n == 0) return;
    const Int cs = C.ColShift(), cstr = C.ColStride(), rs = C.RowShift(), rstr = C.RowStride();
    const Device dev = C.Dev();
    const DType t = C.Type();
    const size_t es = DTypeSize(t);
    const Int bw = TrrkCols(), ra = TrrkRowAlign();
    // local rows whose global row index is < x
    auto rows_below = [&](Int x) { return x <= cs ? Int(0) : std::min<Int>(m, (x - cs + cstr - 1) / cstr); };
    auto gcol = [&](Int j) { return rs + j * rstr; };
    // column j's inside rows: lower [R(j), m), upper [0, R(j))
    auto R = [&](Int j) { return rows_below(lower ? gcol(j) : gcol(j) + 1); };
    // rectangle/leaf row boundaries sit on multiples of ra (128: whole MFMA tiles,
    // 16-B aligned operands, so every rectangle takes the LDS-DMA kernels); the
    // rows a rounding moves out of a rectangle go to the masked leaf instead
    auto up = [&](Int i) { return std::min<Int>(m, (i + ra - 1) / ra * ra); };
    auto down = [&](Int i) { return i / ra * ra; };
    auto arow = [&](Int i) { return static_cast<const char*>(a) + (ta ? i * lda : i) * es; };
    auto bcol = [&](Int j) { return static_cast<const char*>(b) + (tb ? j : j * ldb) * es; };
    auto cptr = [&](Int i, Int j) { return static_cast<char*>(C.Buffer()) + (i + j * C.LDim()) * es; };
    auto rect = [&](Int i0, Int i1, Int j0, Int j1) {
        if (i1 > i0 && j1 > j0)
            exec::Gemm(dev, t, ta, tb, i1 - i0, j1 - j0, k, alpha, arow(i0), lda, bcol(j0), ldb, 1.0, cptr(i0, j0),
                       C.LDim(), s);
    };
    auto leaf = [&](Int i0, Int i1, Int j0, Int j1) {
        const Int h = i1 - i0, w = j1 - j0;
        if (h <= 0 || w <= 0) return;
        const size_t bytes = static_cast<size_t>(h) * w * es;
        if (tmp.bytes() < bytes) tmp.Reset(dev, bytes, s);
        exec::Gemm(dev, t, ta, tb, h, w, k, alpha, arow(i0), lda, bcol(j0), ldb, 0.0, tmp.data(), h, s);
        exec::Trapezoid(dev, t, lower, h, w, 1.0, tmp.data(), h, 1.0, cptr(i0, j0), C.LDim(), cs + i0 * cstr, cstr,
                        gcol(j0), rstr, 0, s);
    };
    // Lower: the strip of columns [j0, j1) is rows [R(j0), end) (rows >= end belong
    // to an enclosing rectangle; end >= R(j1-1)).  Halving: left columns' rows
    // [up(R(jm-1)), end) are inside -> rectangle; the rest recurses.
    std::function<void(Int, Int, Int)> strip_lower = [&](Int j0, Int j1, Int end) {
        if (j1 - j0 <= bw) return leaf(down(R(j0)), end, j0, j1);
        const Int jm = j0 + ((j1 - j0 + 1) / 2 + bw - 1) / bw * bw;
        const Int mid = std::min(end, up(R(jm - 1)));
        rect(mid, end, j0, jm);
        strip_lower(j0, jm, mid);
        strip_lower(jm, j1, end);
    };
    // Upper: the strip of columns [j0, j1) is rows [beg, R(j1-1)) (rows < beg belong
    // to an enclosing rectangle; beg <= R(j0)).  Right columns' rows
    // [beg, down(R(jm))) are inside -> rectangle; the rest recurses.
    std::function<void(Int, Int, Int)> strip_upper = [&](Int j0, Int j1, Int beg) {
        if (j1 - j0 <= bw) return leaf(beg, up(R(j1 - 1)), j0, j1);
        const Int jm = j0 + ((j1 - j0 + 1) / 2 + bw - 1) / bw * bw;
        const Int mid = std::max(beg, down(R(jm)));
        rect(beg, mid, jm, j1);
        strip_upper(j0, jm, beg);
        strip_upper(jm, j1, mid);
    };
    if (lower) {
        const Int b0 = up(R(n - 1));  // rows inside for every column
        rect(b0, m, 0, n);
        strip_lower(0, n, b0);
    } else {
        const Int b0 = down(R(0));
        rect(0, b0, 0, n);
        strip_upper(0, n, b0);
    }
}

// ---------------------------------------------------------------------------
// C-stationary SUMMA, all four orientations (NN.hpp:341-385, NT.hpp:251-294,
// TN.hpp:252-291, TT.hpp:195-240), pipelined over two panel slots.
//   op(A) panel: NORMAL -> A(:,k) as [MC,*];   TRANSPOSE -> A(k,:) as [*,MC]
//   op(B) panel: NORMAL -> B(k,:) as [*,MR];   TRANSPOSE -> B(:,k) as [MR,*]
// ---------------------------------------------------------------------------
// beta is folded into the first panel's update (the reference scales C in a
// separate pass first, Gemm.cpp:282; one fewer HBM round trip of C here).
// uplo >= 0 (Syrk/Herk, Syrk/{LN,LT,UN,UT}.hpp): only C's lower (ELX_LOWER) or
// upper (ELX_UPPER) triangle is updated, through TrrkLocal.
void SummaC(int oA, int oB, double alpha, const DistMatrix& APre, const DistMatrix& BPre, double beta,
            DistMatrix& CPre, int uplo = -1) {
    ELX_TRACE(uplo >= 0 ? "El::Trrk SUMMA_C" : "El::Gemm SUMMA_C");
    MultiSync sync(CPre.Stream(), {APre.Stream(), BPre.Stream()});
    auto Ap = ReadProxy(APre, CPre, Dist::MC, Dist::MR);
    auto Bp = ReadProxy(BPre, CPre, Dist::MC, Dist::MR);
    RWProxy Cp(CPre);
    const DistMatrix& A = *Ap;
    const DistMatrix& B = *Bp;
    DistMatrix& C = Cp.Get();
    const Int K = IsN(oA) ? A.Width() : A.Height();
    const Grid& g = C.G();
    const Device dev = C.Dev();
    const bool gpu = dev == Device::GPU;
    hipStream_t cs = C.Stream();
    hipStream_t ms = gpu ? Runtime::Get().CommStream() : nullptr;
    const Int kc = EffectivePanel(g, K, C.Type());
    const Dist a_cd = IsN(oA) ? Dist::MC : Dist::STAR, a_rd = IsN(oA) ? Dist::STAR : Dist::MC;
    const Dist b_cd = IsN(oB) ? Dist::STAR : Dist::MR, b_rd = IsN(oB) ? Dist::MR : Dist::STAR;

    // One rank and one compute panel: the whole product is ONE local update with
    // beta folded in (no panel slots, comm-stream fences or events; saves ~45 us
    // of host work per call, which is most of a 1024^3 call)
    if (g.Size() == 1 && uplo < 0 && K > 0 && kc >= K) {
        const Int m = C.LocalHeight(), n = C.LocalWidth();
        if (m > 0 && n > 0) {
            const bool prof = gpu && Prof().on;
            const int call_id = Prof().calls++;
            Profiler::Rec rec{};
            if (prof) rec = Prof().Begin(cs);
            exec::Gemm(dev, C.Type(), !IsN(oA), !IsN(oB), m, n, K, alpha, A.Buffer(), A.LDim(), B.Buffer(), B.LDim(),
                       beta, C.Buffer(), C.LDim(), cs);
            if (prof) Prof().End(rec, cs, 2.0 * m * n * K, Prof().gemm, call_id);
        }
        Cp.Finish();
        return;
    }

    // inputs (and beta*C) must be complete before the comm stream reads them
    if (gpu) {
        FenceStreams(A.Stream(), ms);
        FenceStreams(B.Stream(), ms);
        FenceStreams(cs, ms);
    }

    struct Slot {
        std::shared_ptr<DistMatrix> a, b;                 // gathered panels (owned temporaries)
        // the panel's views of A and B on the comm stream: kept until the slot
        // is refilled, so that the owner-stream fence each one issues when it
        // goes (~DistMatrix) lands behind work the updates already wait for
        std::shared_ptr<DistMatrix> va, vb;
        std::shared_ptr<const DistMatrix> ua, ub;         // what the update reads (temporary or view)
        hipEvent_t ready = nullptr, done = nullptr;
        bool pending = false;                             // done recorded, not yet waited by comm
    } slot[2];
    for (auto& s : slot) {
        s.a = A.Like(a_cd, a_rd);
        s.b = B.Like(b_cd, b_rd);
        s.a->SetStream(ms);
        s.b->SetStream(ms);
        // AlignWith(C): A1 rows follow C's rows, B1 cols follow C's cols
        if (IsN(oA)) s.a->AlignCols(C.ColAlign(), true); else s.a->AlignRows(C.ColAlign(), true);
        if (IsN(oB)) s.b->AlignRows(C.RowAlign(), true); else s.b->AlignCols(C.RowAlign(), true);
        if (gpu) {
            ELX_CHECK_HIP(hipEventCreateWithFlags(&s.ready, hipEventDisableTiming));
            ELX_CHECK_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        }
    }
    // Panel p covers [kb[p], kb[p+1]).  On grids larger than 1x1 the panels ramp
    // up kc/4, kc/2, kc, kc, ... (whole communication panels): the first gather
    // is the one transfer no update hides, and each later gather runs behind
    // the previous panel's update, which the doubling keeps long enough for it
    // (a single quarter-depth step left the second, full-depth gather exposed
    // where a panel's transfer and update take similar time: 16-bit C5 at 2x4).
    // A 1x1 grid uses its panels in place: no ramp.
    const Int nb = std::max<Int>(1, Blocksize());
    std::vector<Int> kb{0};
    if (g.Size() > 1 && kc >= 4 * nb && K > kc) {
        for (Int d : {kc / 4, kc / 2}) {
            d = std::max<Int>(nb, d / nb * nb);
            if (kb.back() < K) kb.push_back(std::min<Int>(K, kb.back() + d));
        }
    }
    while (kb.back() < K) kb.push_back(std::min<Int>(K, kb.back() + kc));
    const int np = static_cast<int>(kb.size()) - 1;
    auto kbeg = [&](int p) { return kb[static_cast<size_t>(p)]; };
    const int call_id = Prof().calls++;
    Buffer trrk_tmp;

    auto issue = [&](int p) {
        ELX_TRACE("SUMMA_C panel gather");
        Slot& s = slot[p & 1];
        const Int k0 = kbeg(p), k1 = kbeg(p + 1);
        if (gpu && s.pending) ELX_CHECK_HIP(hipStreamWaitEvent(ms, s.done, 0));
        auto Av = IsN(oA) ? DistMatrix::View(A, 0, A.Height(), k0, k1) : DistMatrix::View(A, k0, k1, 0, A.Width());
        auto Bv = IsN(oB) ? DistMatrix::View(B, k0, k1, 0, B.Width()) : DistMatrix::View(B, 0, B.Height(), k0, k1);
        Av->SetStream(ms);
        Bv->SetStream(ms);
        s.ua.reset();
        s.ub.reset();
        s.va = Av;  // releases panel p-1's views (their fence: see Slot)
        s.vb = Bv;
        const bool prof = gpu && Prof().on;
        Profiler::Rec rec{};
        const int64_t bytes0 = GlobalCommStats().bytes;
        if (prof) rec = Prof().Begin(ms);
        // a panel whose local block already IS the gathered layout (e.g. every
        // panel on a 1x1 grid) is used in place: no copy at all (ELX_SUMMA_COPY=1
        // copies anyway: the N > 1 pipeline's stream pattern on one GPU, for tests
        // and timing studies)
        // The A and B gathers share ONE grouped exchange: they reach disjoint
        // peers (the grid row and the grid column), so their xGMI links carry
        // them concurrently instead of one after the other
        static const bool force_copy = [] { const char* e = getenv("ELX_SUMMA_COPY"); return e && atoi(e) > 0; }();
        std::vector<std::pair<const DistMatrix*, DistMatrix*>> gathers;
        if (!force_copy && SameLocalLayout(*Av, a_cd, a_rd, s.a->ColAlign(), s.a->RowAlign())) s.ua = Av;
        else { gathers.push_back({Av.get(), s.a.get()}); s.ua = s.a; }
        if (!force_copy && SameLocalLayout(*Bv, b_cd, b_rd, s.b->ColAlign(), s.b->RowAlign())) s.ub = Bv;
        else { gathers.push_back({Bv.get(), s.b.get()}); s.ub = s.b; }
        CopyGroup(gathers);
        if (prof) Prof().End(rec, ms, static_cast<double>(GlobalCommStats().bytes - bytes0), Prof().comm);
        if (gpu) ELX_CHECK_HIP(hipEventRecord(s.ready, ms));
    };
    auto compute = [&](int p) {
        ELX_TRACE("SUMMA_C panel update");
        Slot& s = slot[p & 1];
        const DistMatrix& a = *s.ua;
        const DistMatrix& b = *s.ub;
        if (gpu) ELX_CHECK_HIP(hipStreamWaitEvent(cs, s.ready, 0));
        const Int m = C.LocalHeight(), n = C.LocalWidth();
        const Int k = IsN(oA) ? a.LocalWidth() : a.LocalHeight();
        const double b_p = p == 0 ? beta : 1.0;
        if (m > 0 && n > 0 && k > 0) {
            const bool prof = gpu && Prof().on;
            Profiler::Rec rec{};
            if (prof) rec = Prof().Begin(cs);
            if (uplo >= 0)
                TrrkLocal(uplo == ELX_LOWER, !IsN(oA), !IsN(oB), k, alpha, a.Buffer(), a.LDim(), b.Buffer(), b.LDim(),
                          C, cs, trrk_tmp);
            else
                exec::Gemm(dev, C.Type(), !IsN(oA), !IsN(oB), m, n, k, alpha, a.Buffer(), a.LDim(), b.Buffer(),
                           b.LDim(), b_p, C.Buffer(), C.LDim(), cs);
            if (prof) Prof().End(rec, cs, 2.0 * m * n * k, Prof().gemm, call_id);
        } else if (p == 0) {
            Scale(beta, C);
        }
        if (gpu) {
            ELX_CHECK_HIP(hipEventRecord(s.done, cs));
            s.pending = true;
        }
    };
    if (np == 0) Scale(beta, C);
    if (np > 0) issue(0);
    for (int p = 0; p < np; ++p) {
        if (p + 1 < np) issue(p + 1);
        compute(p);
    }
    if (gpu) {
        // temporaries are freed on the comm stream: order that after the last update
        FenceStreams(cs, ms);
        for (auto& s : slot) {
            s.ua.reset();
            s.ub.reset();
            s.va.reset();
            s.vb.reset();
            s.a.reset();
            s.b.reset();
            ELX_CHECK_HIP(hipEventDestroy(s.ready));
            ELX_CHECK_HIP(hipEventDestroy(s.done));
        }
    }
    Cp.Finish();
}

// ---------------------------------------------------------------------------
// C-stationary multistream (NN_Multistream.hpp:262-412, NT/TN siblings): panel
// p is gathered and applied by team p mod S, each on its own stream with its own
// communicators, panel slots and copy of C (team 0 updates C itself, the others
// zero-initialised copies, NN_Multistream.hpp:340-355), summed into C at the end
// (:408-411).  Panels are ComputePanel() deep, as in the pipelined driver.
// ---------------------------------------------------------------------------
void SummaCMultistream(int oA, int oB, double alpha, const DistMatrix& APre, const DistMatrix& BPre, double beta,
                       DistMatrix& CPre) {
    ELX_TRACE("El::Gemm SUMMA_C_MS");
    MultiSync sync(CPre.Stream(), {APre.Stream(), BPre.Stream()});
    auto Ap = ReadProxy(APre, CPre, Dist::MC, Dist::MR);
    auto Bp = ReadProxy(BPre, CPre, Dist::MC, Dist::MR);
    RWProxy Cp(CPre);
    DistMatrix& C0 = Cp.Get();
    const Int K = IsN(oA) ? Ap->Width() : Ap->Height();
    const Int kc = EffectivePanel(C0.G(), K, C0.Type());
    const Int np = (K + kc - 1) / kc;
    Scale(beta, C0);  // Gemm.cpp:282; the team copies start from zero
    TeamViews tv(*Ap, *Bp, C0, TeamCount(C0, np));
    const int S = static_cast<int>(tv.v.size());
    const Dist a_cd = IsN(oA) ? Dist::MC : Dist::STAR, a_rd = IsN(oA) ? Dist::STAR : Dist::MC;
    const Dist b_cd = IsN(oB) ? Dist::STAR : Dist::MR, b_rd = IsN(oB) ? Dist::MR : Dist::STAR;
    struct TeamData { std::shared_ptr<DistMatrix> c, a, b; };
    std::vector<TeamData> td(S);
    for (int t = 0; t < S; ++t) {
        const DistMatrix& Ct = *tv.v[t].C;
        if (t == 0) {
            td[t].c = tv.v[t].C;
        } else {
            td[t].c = Ct.Like(Dist::MC, Dist::MR);
            td[t].c->Align(Ct.ColAlign(), Ct.RowAlign(), true);
            td[t].c->Resize(Ct.Height(), Ct.Width());
            Zero(*td[t].c);
        }
        td[t].a = tv.v[t].A->Like(a_cd, a_rd);
        td[t].b = tv.v[t].B->Like(b_cd, b_rd);
        if (IsN(oA)) td[t].a->AlignCols(Ct.ColAlign(), true); else td[t].a->AlignRows(Ct.ColAlign(), true);
        if (IsN(oB)) td[t].b->AlignRows(Ct.RowAlign(), true); else td[t].b->AlignCols(Ct.RowAlign(), true);
    }
    const Device dev = C0.Dev();
    const int call_id = Prof().calls++;
    for (Int p = 0; p < np; ++p) {
        const int t = static_cast<int>(p % S);
        const auto& v = tv.v[t];
        const DistMatrix& A = *v.A;
        const DistMatrix& B = *v.B;
        DistMatrix& Ct = *td[t].c;
        const Int k0 = p * kc, k1 = std::min(K, k0 + kc);
        auto Av = IsN(oA) ? DistMatrix::View(A, 0, A.Height(), k0, k1) : DistMatrix::View(A, k0, k1, 0, A.Width());
        auto Bv = IsN(oB) ? DistMatrix::View(B, k0, k1, 0, B.Width()) : DistMatrix::View(B, 0, B.Height(), k0, k1);
        std::shared_ptr<const DistMatrix> ua = Av, ub = Bv;
        if (!SameLocalLayout(*Av, a_cd, a_rd, td[t].a->ColAlign(), td[t].a->RowAlign())) {
            Copy(*Av, *td[t].a);
            ua = td[t].a;
        }
        if (!SameLocalLayout(*Bv, b_cd, b_rd, td[t].b->ColAlign(), td[t].b->RowAlign())) {
            Copy(*Bv, *td[t].b);
            ub = td[t].b;
        }
        const Int m = Ct.LocalHeight(), n = Ct.LocalWidth();
        const Int k = IsN(oA) ? ua->LocalWidth() : ua->LocalHeight();
        if (m > 0 && n > 0 && k > 0) {
            const bool prof = dev == Device::GPU && Prof().on;
            Profiler::Rec rec{};
            if (prof) rec = Prof().Begin(v.s);
            exec::Gemm(dev, Ct.Type(), !IsN(oA), !IsN(oB), m, n, k, alpha, ua->Buffer(), ua->LDim(), ub->Buffer(),
                       ub->LDim(), 1.0, Ct.Buffer(), Ct.LDim(), v.s);
            if (prof) Prof().End(rec, v.s, 2.0 * m * n * k, Prof().gemm, call_id);
        }
    }
    tv.Join();
    // C += sum of the other teams' copies (in team order, on C's stream)
    for (int t = 1; t < S; ++t) {
        const DistMatrix& Ct = *td[t].c;
        if (C0.LocalHeight() == 0 || C0.LocalWidth() == 0) break;
        kern::Copy2D d{C0.LocalHeight(), C0.LocalWidth(), Ct.Buffer(), 1, Ct.LDim(), C0.Buffer(), 1, C0.LDim()};
        exec::Copy2DBatch(dev, C0.Type(), &d, 1, true, 1.0, C0.Stream());
    }
    // the copies are released on their teams' streams: after the sums read them
    for (auto& x : tv.v) FenceStreams(tv.cs, x.s);
    td.clear();
    Cp.Finish();
}

// ---------------------------------------------------------------------------
// A-stationary (keeps A, reduces partial C panels): NN.hpp:107-154, NT.hpp:19-59,
// TN.hpp:19-61, TT.hpp:17-61.  Loop over column panels of C.
// ---------------------------------------------------------------------------
// ms: the multistream variant (NN_Multistream.hpp:5-130 and the NT/TN
// siblings): panel p runs on team p mod S, each team with its own stream,
// communicators and temporaries; the C panels are disjoint, so no C copies.
void SummaA(int oA, int oB, double alpha, const DistMatrix& APre, const DistMatrix& BPre, DistMatrix& CPre,
            bool ms = false) {
    ELX_TRACE("El::Gemm SUMMA_A");
    MultiSync sync(CPre.Stream(), {APre.Stream(), BPre.Stream()});
    auto Ap = ReadProxy(APre, CPre, Dist::MC, Dist::MR);
    auto Bp = ReadProxy(BPre, CPre, Dist::MC, Dist::MR);
    RWProxy Cp(CPre);
    const Int n = Cp.Get().Width(), nb = std::max<Int>(1, Blocksize());
    TeamViews tv(*Ap, *Bp, Cp.Get(), ms ? TeamCount(Cp.Get(), (n + nb - 1) / nb) : 1);
    for (Int k = 0; k < n; k += nb) {
        const auto& tm = tv[k / nb];
        const DistMatrix& A = *tm.A;
        const DistMatrix& B = *tm.B;
        DistMatrix& C = *tm.C;
        const Int k1 = std::min(n, k + nb);
        auto C1 = DistMatrix::View(C, 0, C.Height(), k, k1);
        if (IsN(oA)) {
            // D1[MC,*] := alpha A[MC,MR] op(B)1[MR,*];  C1 += sum over MR
            auto B1 = IsN(oB) ? DistMatrix::View(B, 0, B.Height(), k, k1) : DistMatrix::View(B, k, k1, 0, B.Width());
            auto B1T = B.Like(Dist::STAR, Dist::MR);  // (op(B)1)^T with cols over MR
            B1T->AlignWith(A, true);
            if (IsN(oB)) Transpose(*B1, *B1T); else Copy(*B1, *B1T);
            auto D1 = A.Like(Dist::MC, Dist::STAR);
            D1->AlignWith(A, true);
            LocalGemmResize(ELX_NORMAL, ELX_TRANSPOSE, alpha, A, *B1T, *D1);
            AxpyContract(1.0, *D1, *C1);
        } else {
            // D1[MR,*] := alpha A^T[MR,MC] op(B)1[MC,*];  C1 += sum over MC, transposed dist
            auto B1 = IsN(oB) ? DistMatrix::View(B, 0, B.Height(), k, k1) : DistMatrix::View(B, k, k1, 0, B.Width());
            auto B1m = B.Like(Dist::MC, Dist::STAR);  // op(B)1 rows over MC
            B1m->AlignWith(A, true);
            if (IsN(oB)) Copy(*B1, *B1m); else Transpose(*B1, *B1m);
            auto D1 = A.Like(Dist::MR, Dist::STAR);
            D1->AlignWith(A, true);
            LocalGemmResize(ELX_TRANSPOSE, ELX_NORMAL, alpha, A, *B1m, *D1);
            AxpyContract(1.0, *D1, *C1);  // [MR,*] -> [MC,MR]: reduce over MC + exchange
        }
    }
    tv.Join();
    Cp.Finish();
}

// ---------------------------------------------------------------------------
// B-stationary (keeps B, reduces partial C row panels): NN.hpp:226-270,
// NT.hpp:134-176, TN.hpp:137-176, TT.hpp:105-152.  Loop over row panels of C.
// ---------------------------------------------------------------------------
void SummaB(int oA, int oB, double alpha, const DistMatrix& APre, const DistMatrix& BPre, DistMatrix& CPre,
            bool ms = false) {
    ELX_TRACE("El::Gemm SUMMA_B");
    MultiSync sync(CPre.Stream(), {APre.Stream(), BPre.Stream()});
    auto Ap = ReadProxy(APre, CPre, Dist::MC, Dist::MR);
    auto Bp = ReadProxy(BPre, CPre, Dist::MC, Dist::MR);
    RWProxy Cp(CPre);
    const Int m = Cp.Get().Height(), nb = std::max<Int>(1, Blocksize());
    TeamViews tv(*Ap, *Bp, Cp.Get(), ms ? TeamCount(Cp.Get(), (m + nb - 1) / nb) : 1);
    for (Int k = 0; k < m; k += nb) {
        const auto& tm = tv[k / nb];
        const DistMatrix& A = *tm.A;
        const DistMatrix& B = *tm.B;
        DistMatrix& C = *tm.C;
        const Int k1 = std::min(m, k + nb);
        auto C1 = DistMatrix::View(C, k, k1, 0, C.Width());
        // op(A)1 = rows k..k1 of op(A)
        auto A1 = IsN(oA) ? DistMatrix::View(A, k, k1, 0, A.Width()) : DistMatrix::View(A, 0, A.Height(), k, k1);
        if (IsN(oB)) {
            // D1^T[MR,*] := alpha B^T[MR,MC] (op(A)1)^T[MC,*]; C1 += transposed sum over MC
            auto A1T = A.Like(Dist::STAR, Dist::MC);  // op(A)1 with cols over MC
            A1T->AlignWith(B, true);
            if (IsN(oA)) Copy(*A1, *A1T); else Transpose(*A1, *A1T);
            auto D1T = B.Like(Dist::MR, Dist::STAR);
            D1T->AlignWith(B, true);
            LocalGemmResize(ELX_TRANSPOSE, ELX_TRANSPOSE, alpha, B, *A1T, *D1T);
            TransposeAxpyContract(1.0, *D1T, *C1);
        } else {
            // D1[*,MC] := alpha op(A)1[*,MR] B^T[MR,MC]; C1 += sum over MR then redistribute
            auto A1r = A.Like(Dist::STAR, Dist::MR);
            A1r->AlignWith(B, true);
            if (IsN(oA)) Copy(*A1, *A1r); else Transpose(*A1, *A1r);
            auto D1 = B.Like(Dist::STAR, Dist::MC);
            D1->AlignWith(B, true);
            LocalGemmResize(ELX_NORMAL, ELX_TRANSPOSE, alpha, *A1r, B, *D1);
            AxpyContract(1.0, *D1, *C1);
        }
    }
    tv.Join();
    Cp.Finish();
}

// ---------------------------------------------------------------------------
// Dot (1-D inner products over all p ranks): NN.hpp:461-511, NT.hpp:373-418,
// TN.hpp:371-416 (config C4), TT.hpp:287-333.  op(A) -> k distributed VC,
// 2000x2000 blocks of C summed with a reduce-scatter over all ranks.
// ---------------------------------------------------------------------------
void SummaDot(int oA, int oB, double alpha, const DistMatrix& APre, const DistMatrix& BPre, DistMatrix& CPre,
              Int bs) {
    ELX_TRACE("El::Gemm SUMMA_DOT");
    const Int m = CPre.Height(), n = CPre.Width();
    MultiSync sync(CPre.Stream(), {APre.Stream(), BPre.Stream()});
    // k must be distributed VC on both: op(A) = A ([*,VC]) or A^T ([VC,*])
    auto Ap = IsN(oA) ? ReadProxy(APre, CPre, Dist::STAR, Dist::VC) : ReadProxy(APre, CPre, Dist::VC, Dist::STAR);
    const int kAlign = IsN(oA) ? Ap->RowAlign() : Ap->ColAlign();
    auto Bp = IsN(oB) ? ReadProxy(BPre, CPre, Dist::VC, Dist::STAR, kAlign, -1)
                      : ReadProxy(BPre, CPre, Dist::STAR, Dist::VC, -1, kAlign);
    RWProxy Cp(CPre);
    const DistMatrix& A = *Ap;
    const DistMatrix& B = *Bp;
    DistMatrix& C = Cp.Get();
    // (one C11 for all blocks, everything on C's stream: a two-slot variant with
    // the contractions on the comm stream measured no faster on one GPU and 10 %
    // slower with event profiling on, profiles/r02_dot_overlap.log)
    auto C11 = C.Like(Dist::STAR, Dist::STAR);
    for (Int i0 = 0; i0 < m; i0 += bs) {
        const Int i1 = std::min(m, i0 + bs);
        auto A1 = IsN(oA) ? DistMatrix::View(A, i0, i1, 0, A.Width()) : DistMatrix::View(A, 0, A.Height(), i0, i1);
        for (Int j0 = 0; j0 < n; j0 += bs) {
            const Int j1 = std::min(n, j0 + bs);
            auto B1 = IsN(oB) ? DistMatrix::View(B, 0, B.Height(), j0, j1) : DistMatrix::View(B, j0, j1, 0, B.Width());
            auto C1 = DistMatrix::View(C, i0, i1, j0, j1);
            LocalGemmResize(oA, oB, alpha, *A1, *B1, *C11);
            AxpyContract(1.0, *C11, *C1);
        }
    }
    Cp.Finish();
}

// ---------------------------------------------------------------------------
// Cannon's algorithm, NN only (NN.hpp:21-104; dispatched from Gemm.cpp:284-285).
// Square grids, width(A) a multiple of sqrt(p).  The reference runs it on the
// CPU only (NN.hpp:30-31); here on either device: packages are contiguous
// copies of the local blocks, the ring shifts are SendRecv over the MR (grid
// row) and MC (grid column) communicators (RCCL on the GPU), and each step is
// one local MFMA update with beta = 1.
// ---------------------------------------------------------------------------
void Cannon(double alpha, const DistMatrix& APre, const DistMatrix& BPre, DistMatrix& CPre) {
    ELX_TRACE("El::Gemm CANNON");
    const Grid& g = CPre.G();
    if (g.Height() != g.Width()) throw LogicError("Process grid must be square for Cannon's");
    MultiSync sync(CPre.Stream(), {APre.Stream(), BPre.Stream()});
    RWProxy Cp(CPre);
    DistMatrix& C = Cp.Get();
    // A aligned with C's rows, B with C's columns (NN.hpp:43-48)
    auto Ap = ReadProxy(APre, C, Dist::MC, Dist::MR, C.ColAlign(), -1);
    auto Bp = ReadProxy(BPre, C, Dist::MC, Dist::MR, -1, C.RowAlign());
    const DistMatrix& A = *Ap;
    const DistMatrix& B = *Bp;
    const int q = g.Height();
    if (A.Width() % q != 0) throw LogicError("For now, width(A) must be integer multiple of sqrt(p)");
    const Device dev = C.Dev();
    const DType t = C.Type();
    hipStream_t s = C.Stream();
    const Int lhA = A.LocalHeight(), lwA = A.LocalWidth(), lhB = B.LocalHeight(), lwB = B.LocalWidth();
    const Int sizeA = lhA * lwA, sizeB = lhB * lwB;
    const size_t es = DTypeSize(t);
    Buffer pA[2], pB[2];
    for (int i = 0; i < 2; ++i) {
        pA[i].Reset(dev, std::max<size_t>(1, sizeA * es), s);
        pB[i].Reset(dev, std::max<size_t>(1, sizeB * es), s);
    }
    // the initial packages: contiguous copies of the local blocks (NN.hpp:60-71)
    exec::Copy2D d[2] = {{lhA, lwA, A.Buffer(), 1, A.LDim(), pA[0].data(), 1, std::max<Int>(lhA, 1)},
                   {lhB, lwB, B.Buffer(), 1, B.LDim(), pB[0].data(), 1, std::max<Int>(lhB, 1)}};
    for (auto& x : d)
        if (x.m > 0 && x.n > 0) exec::Copy2DBatch(dev, t, &x, 1, false, 0.0, s);
    const int row = g.MCRank(), col = g.MRRank();
    int a = 0, b = 0;
    auto shift = [&](int aTo, int aFrom, int bTo, int bFrom) {
        g.MR().SendRecv(t, pA[a].data(), aTo, pA[a ^ 1].data(), aFrom, sizeA, dev, s);
        g.MC().SendRecv(t, pB[b].data(), bTo, pB[b ^ 1].data(), bFrom, sizeB, dev, s);
        a ^= 1;
        b ^= 1;
    };
    // initial circular shifts so the A and B packages align (NN.hpp:73-84)
    const Int colShiftB = B.ColShift(), rowShiftA = A.RowShift();
    shift((int)Mod(col - colShiftB, q), (int)Mod(col + colShiftB, q), (int)Mod(row - rowShiftA, q),
          (int)Mod(row + rowShiftA, q));
    const int aboveRow = (int)Mod(row - 1, q), belowRow = (int)Mod(row + 1, q);
    const int leftCol = (int)Mod(col - 1, q), rightCol = (int)Mod(col + 1, q);
    for (int step = 0; step < q; ++step) {
        const Int m = C.LocalHeight(), n = C.LocalWidth();
        if (m > 0 && n > 0 && lwA > 0)
            exec::Gemm(dev, t, false, false, m, n, lwA, alpha, pA[a].data(), std::max<Int>(lhA, 1), pB[b].data(),
                       std::max<Int>(lhB, 1), 1.0, C.Buffer(), C.LDim(), s);
        if (step != q - 1) shift(leftCol, rightCol, aboveRow, belowRow);
    }
    Cp.Finish();
}

int Heuristic(Int m, Int n, Int k) {  // NN.hpp:583-600 (same weights in NT/TN/TT)
    const double wC = 2.0, wDot = 10.0;
    if (wDot * m <= k && wDot * n <= k) return ELX_GEMM_SUMMA_DOT;
    if (m <= n && wC * m <= k) return ELX_GEMM_SUMMA_B;
    if (n <= m && wC * n <= k) return ELX_GEMM_SUMMA_A;
    return ELX_GEMM_SUMMA_C;
}

}  // namespace

// an empty stack is a LogicError here (the reference checks it in debug builds only)
void SetBlocksize(Int nb) {
    ELX_REQUIRE(nb > 0, "blocksize must be positive");
    ELX_REQUIRE(!BlocksizeStack().empty(), "Attempted to set blocksize at top of empty stack");
    BlocksizeStack().back() = nb;
}
Int Blocksize() {
    ELX_REQUIRE(!BlocksizeStack().empty(), "Attempted to extract blocksize from empty stack");
    return BlocksizeStack().back();
}
void PushBlocksizeStack(Int nb) {
    ELX_REQUIRE(nb > 0, "blocksize must be positive");
    BlocksizeStack().push_back(nb);
}
void PopBlocksizeStack() {
    ELX_REQUIRE(!BlocksizeStack().empty(), "Attempted to pop an empty blocksize stack");
    BlocksizeStack().pop_back();
}
void EmptyBlocksizeStack() { BlocksizeStack().clear(); }
void SetComputePanel(Int kc) { ELX_REQUIRE(kc >= 0, "compute panel must be >= 0"); g_compute_panel = kc; }
Int ComputePanel() { return g_compute_panel; }
int LastGemmAlgorithm() { return g_last_alg; }
void SetStreamPoolSize(int n) {
    ELX_REQUIRE(n >= 0, "stream pool size must be >= 0 (0: H_STREAMPOOL_SIZE)");
    g_pool_size = n == 0 ? -1 : n;
}
int StreamPoolSize() {
    if (g_pool_size > 0) return g_pool_size;
    const char* e = getenv("H_STREAMPOOL_SIZE");
    return e && atoi(e) > 0 ? atoi(e) : 1;
}

void SetProfiling(bool on) {
    if (Runtime::Get().GPUInitialized()) ELX_CHECK_HIP(hipDeviceSynchronize());
    Prof().Clear();
    Prof().on = on;
    CommProf().Clear();
    CommProf().on = on;
}

void CommProfileStats(double& transfer_ms, int64_t& bytes, int64_t& transfers) {
    transfer_ms = 0;
    bytes = transfers = 0;
    if (!Runtime::Get().GPUInitialized()) return;
    CommProf().Stats(transfer_ms, bytes, transfers);
}

// Compute-stream idle time between consecutive panel updates of one SummaC
// call: the time the MFMA stream waited for a panel gather the pipeline did not
// hide (0 when every transfer overlapped the previous update).
void PipelineStats(double& gap_ms, int64_t& gaps) {
    gap_ms = 0;
    gaps = 0;
    if (!Runtime::Get().GPUInitialized()) return;
    ELX_CHECK_HIP(hipDeviceSynchronize());
    const auto& g = Prof().gemm;
    for (size_t i = 1; i < g.size(); ++i) {
        if (g[i].call < 0 || g[i].call != g[i - 1].call) continue;
        float ms = 0;
        ELX_CHECK_HIP(hipEventElapsedTime(&ms, g[i - 1].b, g[i].a));
        gap_ms += ms > 0 ? ms : 0;
        ++gaps;
    }
}

void ProfileStats(double& gemm_ms, int64_t& launches, double& flops, double& comm_ms, int64_t& bytes) {
    gemm_ms = comm_ms = flops = 0;
    launches = bytes = 0;
    if (!Runtime::Get().GPUInitialized()) return;
    ELX_CHECK_HIP(hipDeviceSynchronize());
    for (auto& r : Prof().gemm) {
        float ms = 0;
        ELX_CHECK_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        gemm_ms += ms;
        flops += r.work;
        ++launches;
    }
    for (auto& r : Prof().comm) {
        float ms = 0;
        ELX_CHECK_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        comm_ms += ms;
        bytes += static_cast<int64_t>(r.work);
    }
}

void LocalGemm(int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, double beta, DistMatrix& C) {
    ELX_TRACE("El::LocalGemm");
    ELX_REQUIRE(A.Type() == B.Type() && A.Type() == C.Type(), "LocalGemm: mixed types");
    ELX_REQUIRE(A.Dev() == B.Dev() && A.Dev() == C.Dev(), "LocalGemm: mixed devices");
    // the reference's conformance checks (src/blas_like/level3/Gemm.cpp:326-423)
    const Dist aR = IsN(oA) ? A.ColDist() : A.RowDist(), aK = IsN(oA) ? A.RowDist() : A.ColDist();
    const Dist bK = IsN(oB) ? B.ColDist() : B.RowDist(), bC = IsN(oB) ? B.RowDist() : B.ColDist();
    const int aRa = IsN(oA) ? A.ColAlign() : A.RowAlign(), aKa = IsN(oA) ? A.RowAlign() : A.ColAlign();
    const int bKa = IsN(oB) ? B.ColAlign() : B.RowAlign(), bCa = IsN(oB) ? B.RowAlign() : B.ColAlign();
    const Int am = IsN(oA) ? A.Height() : A.Width(), ak = IsN(oA) ? A.Width() : A.Height();
    const Int bk = IsN(oB) ? B.Height() : B.Width(), bn = IsN(oB) ? B.Width() : B.Height();
    Check(aR == C.ColDist() && aK == bK && bC == C.RowDist(), "A, B and C do not have compatible distributions");
    Check(aRa == C.ColAlign() && aKa == bKa && bCa == C.RowAlign(), "A, B and C are not aligned");
    Check(am == C.Height() && ak == bk && bn == C.Width(), "nonconformal");
    const Int m = C.LocalHeight(), n = C.LocalWidth();
    const Int k = IsN(oA) ? A.LocalWidth() : A.LocalHeight();
    if (m == 0 || n == 0) return;
    if (k == 0) {  // Gemm.cpp:240-248
        Scale(beta, C);
        return;
    }
    const bool prof = C.Dev() == Device::GPU && Prof().on;
    Profiler::Rec rec{};
    MultiSync sync(C.Stream(), {A.Stream(), B.Stream()});
    if (prof) rec = Prof().Begin(C.Stream());
    exec::Gemm(C.Dev(), C.Type(), !IsN(oA), !IsN(oB), m, n, k, alpha, A.Buffer(), A.LDim(), B.Buffer(), B.LDim(),
               beta, C.Buffer(), C.LDim(), C.Stream());
    if (prof) Prof().End(rec, C.Stream(), 2.0 * m * n * k, Prof().gemm);
}

void LocalGemmResize(int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, DistMatrix& C) {
    const Int m = IsN(oA) ? A.Height() : A.Width();
    const Int n = IsN(oB) ? B.Width() : B.Height();
    const int ca = IsN(oA) ? A.ColAlign() : A.RowAlign();
    const int ra = IsN(oB) ? B.RowAlign() : B.ColAlign();
    if (!C.Viewing()) {
        if (!C.ColConstrained() || C.ColAlign() != ca) C.AlignCols(ca % C.ColStride(), false);
        if (!C.RowConstrained() || C.RowAlign() != ra) C.AlignRows(ra % C.RowStride(), false);
    }
    C.Resize(m, n);
    LocalGemm(oA, oB, alpha, A, B, 0.0, C);
}

void ScaleTrapezoid(double alpha, int uplo, DistMatrix& A, Int offset) {
    ELX_REQUIRE(uplo == ELX_LOWER || uplo == ELX_UPPER, "ScaleTrapezoid: bad UpperOrLower ", uplo);
    if (alpha == 1.0) return;  // ScaleTrapezoid.hpp:52-53
    exec::Trapezoid(A.Dev(), A.Type(), uplo == ELX_LOWER, A.LocalHeight(), A.LocalWidth(), 0.0, nullptr, 0, alpha,
                    A.Buffer(), A.LDim(), A.ColShift(), A.ColStride(), A.RowShift(), A.RowStride(), offset,
                    A.Stream());
}

// Syrk / Herk on DistMatrices (src/blas_like/level3/Syrk.cpp:196-211): the
// trapezoid of C is scaled by beta, then LN/LT/UN/UT run as the C-stationary
// pipeline with the triangular local update (Syrk/LN.hpp:13-48 and siblings:
// A1[MC,*] and A1^T[*,MR] per panel, LocalTrrk).  Real types only, so the
// conjugate flag (Herk) changes nothing.  The reference switches to its Dot
// variant when width > 10 height (LN.hpp:156); here the panel pipeline serves
// every shape (same sums, summation order within the normwise tolerance).
void Syrk(int uplo, int orient, double alpha, const DistMatrix& A, double beta, DistMatrix& C) {
    ELX_TRACE("El::Syrk");
    ELX_REQUIRE(uplo == ELX_LOWER || uplo == ELX_UPPER, "Syrk: bad UpperOrLower ", uplo);
    ELX_REQUIRE(orient >= ELX_NORMAL && orient <= ELX_ADJOINT, "Syrk: bad orientation");
    ELX_REQUIRE(&A.G() == &C.G(), "Syrk: matrices on different grids");
    ELX_REQUIRE(A.Type() == C.Type(), "Syrk: mixed types");
    const bool N = orient == ELX_NORMAL;
    const Int n = N ? A.Height() : A.Width();
    if (C.Height() != n || C.Width() != n) throw LogicError("Nonconformal Syrk");
    ScaleTrapezoid(beta, uplo, C, 0);
    if (N) SummaC(ELX_NORMAL, ELX_TRANSPOSE, alpha, A, A, 1.0, C, uplo);
    else SummaC(ELX_TRANSPOSE, ELX_NORMAL, alpha, A, A, 1.0, C, uplo);
}

// Trrk on DistMatrices (src/blas_like/level3/Trrk.cpp:100-117): C := alpha op(A)
// op(B) + beta C on C's uplo triangle; TrrkNN/NT/TN/TT are the same C-stationary
// pipeline with the triangular local update.
void Trrk(int uplo, int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, double beta,
          DistMatrix& C) {
    ELX_REQUIRE(uplo == ELX_LOWER || uplo == ELX_UPPER, "Trrk: bad UpperOrLower ", uplo);
    ELX_REQUIRE(&A.G() == &B.G() && &A.G() == &C.G(), "Trrk: matrices on different grids");
    ELX_REQUIRE(A.Type() == B.Type() && A.Type() == C.Type(), "Trrk: mixed types");
    if (oA == ELX_ADJOINT) oA = ELX_TRANSPOSE;
    if (oB == ELX_ADJOINT) oB = ELX_TRANSPOSE;
    const Int m = IsN(oA) ? A.Height() : A.Width(), k = IsN(oA) ? A.Width() : A.Height();
    const Int kb = IsN(oB) ? B.Height() : B.Width(), n = IsN(oB) ? B.Width() : B.Height();
    if (m != C.Height() || n != C.Width() || k != kb || m != n) throw LogicError("Nonconformal Trrk");
    ScaleTrapezoid(beta, uplo, C, 0);
    SummaC(oA, oB, alpha, A, B, 1.0, C, uplo);
}

// Syr2k / Her2k (src/blas_like/level3/Syr2k.cpp:78-93, Syr2k/LN.hpp): C := alpha
// (op(A) op(B)^T + op(B) op(A)^T) + beta C on C's uplo triangle.  The reference
// gathers both panels and runs two LocalTrrks per panel; here each term is one
// pass of the triangular pipeline.  Real types: conj(alpha) = alpha.
void Syr2k(int uplo, int orient, double alpha, const DistMatrix& A, const DistMatrix& B, double beta,
           DistMatrix& C) {
    ELX_REQUIRE(uplo == ELX_LOWER || uplo == ELX_UPPER, "Syr2k: bad UpperOrLower ", uplo);
    ELX_REQUIRE(orient >= ELX_NORMAL && orient <= ELX_ADJOINT, "Syr2k: bad orientation");
    ELX_REQUIRE(&A.G() == &B.G() && &A.G() == &C.G(), "Syr2k: matrices on different grids");
    ELX_REQUIRE(A.Type() == B.Type() && A.Type() == C.Type(), "Syr2k: mixed types");
    const bool N = orient == ELX_NORMAL;
    const Int n = N ? A.Height() : A.Width();
    if (A.Height() != B.Height() || A.Width() != B.Width() || C.Height() != n || C.Width() != n)
        throw LogicError("Nonconformal Syr2k");
    ScaleTrapezoid(beta, uplo, C, 0);
    const int oA = N ? ELX_NORMAL : ELX_TRANSPOSE, oB = N ? ELX_TRANSPOSE : ELX_NORMAL;
    SummaC(oA, oB, alpha, A, B, 1.0, C, uplo);
    SummaC(oA, oB, alpha, B, A, 1.0, C, uplo);
}

// Trsm on DistMatrices (src/blas_like/level3/Trsm.cpp:129-420): B := alpha
// op(A)^-1 B (LEFT) or alpha B op(A)^-1 (RIGHT).  LEFT follows Trsm/LLN.hpp:40-70
// (and LUN/LLT/LUT with the block order reversed where op(A) is upper):
//   A11[*,*] <- A11;  X1[*,VR] <- X1;  X1[*,VR] := op(A11)^-1 X1 (trsm_kernel);
//   X1 <- X1[*,VR];   X_rest -= op(A)_rest,1 X1 (the C-stationary SUMMA on views:
//   op(A) panel gathered [MC,*] / [*,MC], X1 as [*,MR], MFMA update).
// RIGHT solves the transposed LEFT problem (X op(A) = B <=> op(A)^T X^T = B^T)
// through two distributed transposes.  f64/f32 (the reference's GPU Trsm types).
// ELX_TRSM_FLAT=1: the reference's flat nb-step sweep (every update k = nb over
// all remaining rows) instead of the recursive split (tests, ablation)
bool TrsmFlat() {
    static const bool v = [] { const char* e = getenv("ELX_TRSM_FLAT"); return e && atoi(e) > 0; }();
    return v;
}

void TrsmLeft(int uplo, int orient, bool unit, const DistMatrix& APre, DistMatrix& XPre) {
    ELX_TRACE("El::Trsm");
    MultiSync sync(XPre.Stream(), {APre.Stream()});
    auto Ap = ReadProxy(APre, XPre, Dist::MC, Dist::MR);
    const DistMatrix& A = *Ap;
    RWProxy Xp(XPre);
    DistMatrix& X = Xp.Get();
    const Int m = X.Height(), n = X.Width();
    Int nb = std::max<Int>(1, Blocksize());
    const bool trans = orient != ELX_NORMAL, lower = uplo == ELX_LOWER;
    const bool forward = lower != trans;  // op(A) lower: blocks top to bottom
    auto A11s = A.Like(Dist::STAR, Dist::STAR);
    auto X1v = X.Like(Dist::STAR, Dist::VR);
    // X_rest -= op(A)(r0:r1, k0:k1) X(k0:k1, :) through the SUMMA pipeline on views
    // (solved rows are read from `src`: X itself, or Y on the batched path)
    const DistMatrix* src = &X;
    bool local = false;  // set on the batched path: every operand's local block is the whole matrix
    auto update = [&](Int r0, Int r1, Int k0, Int k1) {
        if (r1 <= r0 || k1 <= k0 || n == 0) return;
        if (local) {  // one MFMA GEMM on the local blocks: no views, proxies or pipeline on the host
            const size_t es = DTypeSize(X.Type());
            const char* a = static_cast<const char*>(A.Buffer()) +
                            ((trans ? k0 + r0 * A.LDim() : r0 + k0 * A.LDim()) * es);
            const char* y = static_cast<const char*>(src->Buffer()) + k0 * es;
            char* x = static_cast<char*>(X.Buffer()) + r0 * es;
            exec::Gemm(X.Dev(), X.Type(), trans, false, r1 - r0, n, k1 - k0, -1.0, a, A.LDim(), y, src->LDim(), 1.0, x,
                       X.LDim(), X.Stream());
            return;
        }
        auto Ar = trans ? DistMatrix::View(A, k0, k1, r0, r1) : DistMatrix::View(A, r0, r1, k0, k1);
        auto Xk = DistMatrix::View(*src, k0, k1, 0, n);
        auto Xr = DistMatrix::View(X, r0, r1, 0, n);
        SummaC(trans ? ELX_TRANSPOSE : ELX_NORMAL, ELX_NORMAL, -1.0, *Ar, *Xk, 1.0, *Xr);
    };
    // A whose local block is the whole matrix (1x1 grid): every diagonal block's
    // inverse comes from ONE batched launch up front (the per-block inversions
    // are independent), applied per block as an MFMA GEMM whose output goes
    // straight into a second buffer Y (no write-back per block; every later
    // update reads solved rows from Y, copied into X once at the end);
    // elsewhere each block is solved where it lands (exec::Trsm)
    const size_t es = DTypeSize(X.Type());
    Buffer winv;
    auto batch_ok = [&](Int b) {
        return X.Dev() == Device::GPU && SameLocalLayout(A, Dist::STAR, Dist::STAR, 0, 0) &&
               b * 65 * (Int)es <= kern::kTriInverseLdsMax && (m + b - 1) / b <= 65535 &&
               kern::tri_inverse_lds_ok(static_cast<int>(X.Type()), b) &&
               SameLocalLayout(X, Dist::STAR, Dist::VR, 0, X.RowAlign()) && X.LocalWidth() >= 4 * b;
    };
    // Batched path with the default Blocksize (128) and a large system: 256-row
    // diagonal blocks, so every leaf (inverse applied as a GEMM) and the lowest
    // updates are 256 x n MFMA launches (256 output tiles, the whole machine)
    // instead of 128 x n ones (half of it); ELX_TRSM_NB256=0 keeps 128.
    static const bool nb256 = [] { const char* e = getenv("ELX_TRSM_NB256"); return !e || atoi(e) != 0; }();
    if (nb256 && nb == 128 && m >= 8 * 256 && batch_ok(256)) nb = 256;
    const bool batched = batch_ok(nb);
    std::shared_ptr<DistMatrix> Y;
    if (batched) {
        FenceStreams(A.Stream(), X.Stream());
        winv.Reset(Device::GPU, static_cast<size_t>((m + nb - 1) / nb) * nb * nb * es, X.Stream());
        exec::TriInverseBatched(X.Type(), lower, trans, unit, nb, m, A.Buffer(), A.LDim(), winv.data(), X.Stream());
        Y = X.Like(Dist::MC, Dist::MR);
        Y->Align(X.ColAlign(), X.RowAlign(), true);
        Y->Resize(m, n);
        src = Y.get();
        local = X.LocalHeight() == m && X.LocalWidth() == n && Y->LDim() > 0 && !getenv("ELX_TRSM_SUMMA");
    }
    // X(k0:k1, :) := op(A11)^-1 X(k0:k1, :), one nb block (Trsm/LLN.hpp:49-60)
    auto leaf = [&](Int k0, Int k1) {
        auto X1 = DistMatrix::View(X, k0, k1, 0, n);
        if (batched) {
            auto Y1 = DistMatrix::View(*Y, k0, k1, 0, n);
            exec::Gemm(X.Dev(), X.Type(), false, false, k1 - k0, X1->LocalWidth(), k1 - k0, 1.0,
                       static_cast<const char*>(winv.data()) + (k0 / nb) * nb * nb * es, nb, X1->Buffer(),
                       X1->LDim(), 0.0, Y1->Buffer(), Y1->LDim(), X1->Stream());
            return;
        }
        // a block whose local storage already IS the [*,*] / [*,VR] layout (a
        // 1x1 grid) is used in place: no redistribution temporaries
        auto A11 = DistMatrix::View(A, k0, k1, k0, k1);
        std::shared_ptr<const DistMatrix> a11 = A11;
        if (!SameLocalLayout(*A11, Dist::STAR, Dist::STAR, 0, 0)) {
            Copy(*A11, *A11s);                               // A11[*,*] <- A11[MC,MR]
            a11 = A11s;
        }
        const bool inplace = SameLocalLayout(*X1, Dist::STAR, Dist::VR, 0, X1->RowAlign());
        DistMatrix* x1 = X1.get();
        if (!inplace) {
            X1v->AlignRows(X.RowAlign(), true);
            Copy(*X1, *X1v);                                 // X1[*,VR] <- X1[MC,MR]
            x1 = X1v.get();
        }
        if (X.Dev() == Device::GPU) FenceStreams(a11->Stream(), x1->Stream());
        exec::Trsm(X.Dev(), X.Type(), lower, trans, unit, k1 - k0, x1->LocalWidth(), a11->Buffer(), a11->LDim(),
                   x1->Buffer(), x1->LDim(), x1->Stream());
        if (!inplace) Copy(*X1v, *X1);                       // X1[MC,MR] <- X1[*,VR]
    };
    const Int nblk = (m + nb - 1) / nb;
    if (TrsmFlat()) {
        // the reference's order (Trsm/LLN.hpp:40-70): solve block b, then update
        // every remaining row with k = nb
        for (Int bi = 0; bi < nblk; ++bi) {
            const Int b = forward ? bi : nblk - 1 - bi;
            const Int k0 = b * nb, k1 = std::min(m, k0 + nb);
            leaf(k0, k1);
            if (forward) update(k1, m, k0, k1);
            else update(0, k0, k0, k1);
        }
    } else {
        // Recursive split at a block boundary: solve the half op(A) reaches first,
        // eliminate it from the other half with ONE GEMM (k = that half's height),
        // solve the other half.  The same eliminations as the nb-step sweep, but
        // half of all update FLOPs go to a k = m/2 GEMM, a quarter to two k = m/4
        // ones, ...: deep, full-machine MFMA launches instead of m/nb k = nb ones.
        std::function<void(Int, Int)> solve = [&](Int K0, Int K1) {
            const Int nbk = (K1 - K0 + nb - 1) / nb;
            if (nbk <= 1) return leaf(K0, K1);
            const Int mid = K0 + (nbk / 2) * nb;
            if (forward) {
                solve(K0, mid);
                update(mid, K1, K0, mid);
                solve(mid, K1);
            } else {
                solve(mid, K1);
                update(K0, mid, mid, K1);
                solve(K0, mid);
            }
        };
        if (m > 0) solve(0, m);
    }
    if (Y) Copy(*Y, X);
    Xp.Finish();
}

void Trsm(int side, int uplo, int orient, int diag, double alpha, const DistMatrix& A, DistMatrix& B,
          bool checkIfSingular) {
    ELX_REQUIRE(side == ELX_LEFT || side == ELX_RIGHT, "Trsm: bad LeftOrRight ", side);
    ELX_REQUIRE(uplo == ELX_LOWER || uplo == ELX_UPPER, "Trsm: bad UpperOrLower ", uplo);
    ELX_REQUIRE(orient >= ELX_NORMAL && orient <= ELX_ADJOINT, "Trsm: bad orientation");
    ELX_REQUIRE(diag == ELX_NON_UNIT || diag == ELX_UNIT, "Trsm: bad UnitOrNonUnit ", diag);
    ELX_REQUIRE(&A.G() == &B.G(), "Trsm: matrices on different grids");
    ELX_REQUIRE(A.Type() == B.Type(), "Trsm: mixed types");
    if (A.Type() != DType::F64 && A.Type() != DType::F32) throw LogicError("Trsm: only float and double are supported");
    if (A.Height() != A.Width()) throw LogicError("A must be square");  // Trsm.cpp:142-143
    if ((side == ELX_LEFT ? B.Height() : B.Width()) != A.Height()) throw LogicError("Nonconformal Trsm");
    if (checkIfSingular && diag != ELX_UNIT && DiagonalHasZero(A)) throw SingularMatrixError();
    Scale(alpha, B);  // Trsm.cpp:155 (B *= alpha)
    if (side == ELX_LEFT) return TrsmLeft(uplo, orient, diag == ELX_UNIT, A, B);
    auto Bt = B.Like(Dist::MC, Dist::MR);
    Transpose(B, *Bt);
    TrsmLeft(uplo, orient == ELX_NORMAL ? ELX_TRANSPOSE : ELX_NORMAL, diag == ELX_UNIT, A, *Bt);
    Transpose(*Bt, B);
}

// Symm / Hemm on DistMatrices (src/blas_like/level3/Symm.cpp:55-80): C := alpha
// A B + beta C (LEFT) or alpha B A + beta C (RIGHT), A symmetric with only its
// uplo triangle read.  The reference accumulates triangle-aware local products
// (Symm/LL.hpp LocalAccumulateLL); here A is completed once into a full [MC,MR]
// copy (one distributed transpose + a trapezoid copy of the mirrored strict
// triangle, O(n^2) HBM work) and the product runs through El::Gemm's pipeline.
void Symm(int side, int uplo, double alpha, const DistMatrix& A, const DistMatrix& B, double beta, DistMatrix& C) {
    ELX_REQUIRE(side == ELX_LEFT || side == ELX_RIGHT, "Symm: bad LeftOrRight ", side);
    ELX_REQUIRE(uplo == ELX_LOWER || uplo == ELX_UPPER, "Symm: bad UpperOrLower ", uplo);
    ELX_REQUIRE(&A.G() == &B.G() && &A.G() == &C.G(), "Symm: matrices on different grids");
    ELX_REQUIRE(A.Type() == B.Type() && A.Type() == C.Type(), "Symm: mixed types");
    if (A.Height() != A.Width()) throw LogicError("A must be square");
    const bool left = side == ELX_LEFT;
    if ((left ? B.Height() : B.Width()) != A.Height() || C.Height() != B.Height() || C.Width() != B.Width())
        throw LogicError("Nonconformal Symm");
    auto S = A.Like(Dist::MC, Dist::MR);
    Copy(A, *S);
    auto T = A.Like(Dist::MC, Dist::MR);
    T->AlignWith(*S, true);
    Transpose(*S, *T);
    // S's strictly-other triangle := T's (lower stored: strict upper is gi <= gj - 1)
    const bool other_lower = uplo == ELX_UPPER;
    if (S->Dev() == Device::GPU) FenceStreams(T->Stream(), S->Stream());
    exec::Trapezoid(S->Dev(), S->Type(), other_lower, S->LocalHeight(), S->LocalWidth(), 1.0, T->Buffer(), T->LDim(),
                    0.0, S->Buffer(), S->LDim(), S->ColShift(), S->ColStride(), S->RowShift(), S->RowStride(),
                    other_lower ? -1 : 1, S->Stream());
    if (left) Gemm(ELX_NORMAL, ELX_NORMAL, alpha, *S, B, beta, C, ELX_GEMM_DEFAULT);
    else Gemm(ELX_NORMAL, ELX_NORMAL, alpha, B, *S, beta, C, ELX_GEMM_DEFAULT);
}

void Gemm(int oA, int oB, double alpha, const DistMatrix& A, const DistMatrix& B, double beta, DistMatrix& C,
          int alg) {
    ELX_TRACE("El::Gemm");
    ELX_REQUIRE(oA >= ELX_NORMAL && oA <= ELX_ADJOINT && oB >= ELX_NORMAL && oB <= ELX_ADJOINT, "bad orientation");
    ELX_REQUIRE(&A.G() == &B.G() && &A.G() == &C.G(), "Gemm: matrices on different grids");
    ELX_REQUIRE(A.Type() == B.Type() && A.Type() == C.Type(), "Gemm: mixed types");
    // real types: ADJOINT == TRANSPOSE
    if (oA == ELX_ADJOINT) oA = ELX_TRANSPOSE;
    if (oB == ELX_ADJOINT) oB = ELX_TRANSPOSE;
    const Int m = IsN(oA) ? A.Height() : A.Width(), k = IsN(oA) ? A.Width() : A.Height();
    const Int kb = IsN(oB) ? B.Height() : B.Width(), n = IsN(oB) ? B.Width() : B.Height();
    ELX_REQUIRE(m == C.Height() && n == C.Width() && k == kb, "Gemm: nonconformal ", m, "x", k, " * ", kb, "x", n,
                " -> ", C.Height(), "x", C.Width());
    const bool tt = !IsN(oA) && !IsN(oB);
    // NN.hpp:583-600: with a GPU C and a stream pool larger than one, the
    // heuristic picks the multistream variants (TT has none, TT.hpp:410-433)
    const bool gpu_pool = C.Dev() == Device::GPU && TeamCount(C, 2) > 1 && !tt;
    if (alg == ELX_GEMM_DEFAULT) {
        alg = Heuristic(m, n, k);
        if (gpu_pool && alg == ELX_GEMM_SUMMA_A) alg = ELX_GEMM_SUMMA_A_MS;
        if (gpu_pool && alg == ELX_GEMM_SUMMA_B) alg = ELX_GEMM_SUMMA_B_MS;
        if (gpu_pool && alg == ELX_GEMM_SUMMA_C) alg = ELX_GEMM_SUMMA_C_MS;
    }
    const bool ms = alg == ELX_GEMM_SUMMA_A_MS || alg == ELX_GEMM_SUMMA_B_MS || alg == ELX_GEMM_SUMMA_C_MS;
    if (ms && tt) throw LogicError("Unsupported Gemm option");  // TT.hpp:433
    // a CPU C runs the plain variant (the reference warns "CPU doesn't support
    // multistream variants", TN.hpp:114-118); so does a pool of one
    const bool teams = ms && C.Dev() == Device::GPU && TeamCount(C, 2) > 1;
    const bool fused_beta = alg == ELX_GEMM_SUMMA_C || (alg == ELX_GEMM_SUMMA_C_MS && !teams);
    if (!fused_beta && !(alg == ELX_GEMM_SUMMA_C_MS && teams)) Scale(beta, C);  // Gemm.cpp:282
    switch (alg) {
    case ELX_GEMM_SUMMA_A_MS: case ELX_GEMM_SUMMA_A: SummaA(oA, oB, alpha, A, B, C, teams); break;
    case ELX_GEMM_SUMMA_B_MS: case ELX_GEMM_SUMMA_B: SummaB(oA, oB, alpha, A, B, C, teams); break;
    case ELX_GEMM_SUMMA_C_MS:
        if (teams) SummaCMultistream(oA, oB, alpha, A, B, beta, C);
        else SummaC(oA, oB, alpha, A, B, beta, C);
        break;
    case ELX_GEMM_SUMMA_C: SummaC(oA, oB, alpha, A, B, beta, C); break;
    case ELX_GEMM_SUMMA_DOT:
        SummaDot(oA, oB, alpha, A, B, C, C.Dev() == Device::GPU ? DotBlockGPU() : kDotBlock);
        break;
    case ELX_GEMM_CANNON:
        // Gemm.cpp:284-285: Cannon for NN; the other orientations' SUMMA switches
        // reject it (NT.hpp:526, TN.hpp:524, TT.hpp:435)
        if (oA != ELX_NORMAL || oB != ELX_NORMAL) throw LogicError("Unsupported Gemm option");
        Cannon(alpha, A, B, C);
        break;
    default: throw LogicError(Cat("Unsupported Gemm option ", alg));
    }
    g_last_alg = alg;
}

}  // namespace elx
