#include "distmatrix.hpp"
#include "exec.hpp"
#include <cmath>
#include <cstring>

namespace elx {

const char* DistName(Dist d) {
    switch (d) {
    case Dist::MC: return "MC";
    case Dist::MD: return "MD";
    case Dist::MR: return "MR";
    case Dist::VC: return "VC";
    case Dist::VR: return "VR";
    case Dist::STAR: return "STAR";
    case Dist::CIRC: return "CIRC";
    }
    return "?";
}

// ---------------------------------------------------------------- Grid ----

int Grid::DefaultHeight(int size) {  // src/core/Grid.cpp:58-64
    int h = static_cast<int>(std::sqrt(static_cast<double>(size)));
    if (h < 1) h = 1;
    while (size % h != 0) ++h;
    return h;
}

Grid::Grid(std::shared_ptr<Comm> world, int height, int order) : world_(std::move(world)), order_(order) {
    p_ = world_->Size();
    r_ = height > 0 ? height : DefaultHeight(p_);
    ELX_REQUIRE(p_ % r_ == 0, "grid height ", r_, " does not divide ", p_);
    c_ = p_ / r_;
    const int rank = world_->Rank();
    if (order == ELX_COLUMN_MAJOR) { mc_ = rank % r_; mr_ = rank / r_; }
    else { mr_ = rank % c_; mc_ = rank / c_; }
    // MatrixCol comm = same column of the grid (fixed mrRank), ordered by mcRank;
    // MatrixRow comm = same row (fixed mcRank), ordered by mrRank (Grid.cpp:133-148).
    mc_comm_ = world_->Split(mr_, mc_);
    mr_comm_ = world_->Split(mc_, mr_);
    vc_comm_ = world_->Split(0, VCRank());
    vr_comm_ = world_->Split(0, VRRank());
    ELX_REQUIRE(mc_comm_->Size() == r_ && mr_comm_->Size() == c_ && vc_comm_->Size() == p_,
                "grid communicator split produced inconsistent sizes");
    int a = r_, b = c_;
    while (b) { const int t = a % b; a = b; b = t; }
    gcd_ = a;
    md_rank_.assign(p_, 0);
    md_perp_.assign(p_, 0);
    for (int diag = 0; diag < gcd_; ++diag) {
        int row = 0, col = diag;
        for (int k = 0; k < LCM(); ++k) {
            const int vc = row + r_ * col;
            md_perp_[vc] = diag;
            md_rank_[vc] = k;
            row = (row + 1) % r_;
            col = (col + 1) % c_;
        }
    }
}

Device Grid::CommDevice() const {
    return world_->kind() == Comm::Kind::RCCL ? Device::GPU : Device::CPU;
}

int Grid::Stride(Dist d) const {
    switch (d) {
    case Dist::MC: return r_;
    case Dist::MR: return c_;
    case Dist::VC:
    case Dist::VR: return p_;
    case Dist::STAR:
    case Dist::CIRC: return 1;
    case Dist::MD: return LCM();
    }
    throw LogicError("unknown distribution");
}

int Grid::DistRankOf(Dist d, int vc) const {
    switch (d) {
    case Dist::MC: return MCOf(vc);
    case Dist::MR: return MROf(vc);
    case Dist::VC: return vc;
    case Dist::VR: return VROf(vc);
    case Dist::STAR:
    case Dist::CIRC: return 0;
    case Dist::MD: return MDRankOf(vc);
    }
    throw LogicError("unknown distribution");
}

Comm& Grid::DistComm(Dist d) const {
    switch (d) {
    case Dist::MC: return *mc_comm_;
    case Dist::MR: return *mr_comm_;
    case Dist::VC: return *vc_comm_;
    case Dist::VR: return *vr_comm_;
    default: break;
    }
    throw LogicError(Cat("no communicator for dist ", DistName(d)));
}

// ---------------------------------------------------------- DistMatrix ----

namespace {
bool ValidPair(Dist u, Dist v) {
    if (u == Dist::CIRC || v == Dist::CIRC) return u == Dist::CIRC && v == Dist::CIRC;
    if (u == Dist::MD || v == Dist::MD) return u == Dist::STAR || v == Dist::STAR;  // [MD,*], [*,MD]
    if (u == Dist::STAR || v == Dist::STAR) return true;
    return (u == Dist::MC && v == Dist::MR) || (u == Dist::MR && v == Dist::MC);
}
Dist Partial(Dist u) { return u == Dist::VC ? Dist::MC : (u == Dist::VR ? Dist::MR : u); }
Dist PartialUnionRow(Dist u, Dist v) { return u == Dist::VC ? Dist::MR : (u == Dist::VR ? Dist::MC : v); }
Dist PartialUnionCol(Dist u, Dist v) { return PartialUnionRow(v, u); }
Dist Collect(Dist u) { return u == Dist::CIRC ? Dist::CIRC : Dist::STAR; }
}  // namespace

DistMatrix::DistMatrix(std::shared_ptr<Grid> g, DType t, Dist colDist, Dist rowDist, Device dev, int root)
    : grid_(std::move(g)), dtype_(t), cdist_(colDist), rdist_(rowDist), dev_(dev), root_(root) {
    if (!ValidPair(colDist, rowDist))
        throw LogicError(Cat("invalid distribution [", DistName(colDist), ",", DistName(rowDist), "]"));
    ELX_REQUIRE(root >= 0 && root < CrossSize(), "Invalid root ", root);
    if (dev == Device::GPU) stream_ = Runtime::Get().ComputeStream();
    SetLocalSizes();
}

DistMatrix::~DistMatrix() {
    if (dev_ != Device::GPU || !buf_ || !buf_->data()) return;
    const hipStream_t home = buf_->stream();
    if (!home || !stream_ || home == stream_) return;
    try { StreamFence(stream_, home); } catch (...) {}
}

int DistMatrix::ColStride() const { return G().Stride(cdist_); }
int DistMatrix::RowStride() const { return G().Stride(rdist_); }

// The ranks that can hold data: CIRC's root, the root diagonal for [MD,*] /
// [*,MD] (CrossComm = MDPerp, MD_STAR.cpp:166-167), everyone otherwise.
int DistMatrix::CrossSize() const {
    if (cdist_ == Dist::CIRC) return G().Size();
    if (cdist_ == Dist::MD || rdist_ == Dist::MD) return G().GCD();
    return 1;
}
bool DistMatrix::CrossOf(int vc) const {
    if (cdist_ == Dist::CIRC) return vc == root_;
    if (cdist_ == Dist::MD || rdist_ == Dist::MD) return G().MDPerpOf(vc) == root_;
    return true;
}
int DistMatrix::ColRankOf(int vc) const {
    if (!CrossOf(vc)) return -1;
    return cdist_ == Dist::CIRC ? 0 : G().DistRankOf(cdist_, vc);
}
int DistMatrix::RowRankOf(int vc) const {
    if (!CrossOf(vc)) return -1;
    return rdist_ == Dist::CIRC ? 0 : G().DistRankOf(rdist_, vc);
}
Int DistMatrix::LocalHeightOf(int vc) const {
    if (!ParticipatingOf(vc)) return 0;
    return Length(h_, Shift(ColRankOf(vc), calign_, ColStride()), ColStride());
}
Int DistMatrix::LocalWidthOf(int vc) const {
    if (!ParticipatingOf(vc)) return 0;
    return Length(w_, Shift(RowRankOf(vc), ralign_, RowStride()), RowStride());
}

void DistMatrix::SetLocalSizes() {
    lh_ = LocalHeightOf(G().VCRank());
    lw_ = LocalWidthOf(G().VCRank());
}

void* DistMatrix::Buffer() const {
    if (!buf_ || !buf_->data()) return nullptr;
    return static_cast<char*>(buf_->data()) + offset_ * static_cast<Int>(ElemSize());
}

void DistMatrix::Allocate() {
    const Int need_ld = lh_ > 0 ? lh_ : 1;
    const size_t need = static_cast<size_t>(need_ld) * static_cast<size_t>(lw_) * ElemSize();
    if (buf_ && buf_->bytes() >= need && ld_ == need_ld) return;
    ld_ = need_ld;
    offset_ = 0;
    buf_ = std::make_shared<elx::Buffer>(dev_, need, stream_);
}

void DistMatrix::Resize(Int height, Int width) {
    ELX_REQUIRE(height >= 0 && width >= 0, "negative dimensions");
    if (viewing_) {
        ELX_REQUIRE(height == h_ && width == w_, "cannot resize a view");
        return;
    }
    h_ = height;
    w_ = width;
    SetLocalSizes();
    Allocate();
}

void DistMatrix::Empty() {
    ELX_REQUIRE(!viewing_, "cannot empty a view");
    h_ = w_ = 0;
    SetLocalSizes();
    buf_.reset();
    ld_ = 1;
    offset_ = 0;
}

// ElementalMatrix::Attach (src/core/DistMatrix/ElementMatrix.cpp:368-409): view
// caller storage as this rank's local block; alignments become constrained.
void DistMatrix::Attach(Int height, Int width, int colAlign, int rowAlign, void* buffer, Int ldim, int root) {
    ELX_REQUIRE(height >= 0 && width >= 0, "negative dimensions");
    ELX_REQUIRE(root >= 0 && root < CrossSize(), "Invalid root ", root);
    const int cs = ColStride(), rs = RowStride();
    ELX_REQUIRE(colAlign >= 0 && colAlign < cs, "invalid col alignment ", colAlign);
    ELX_REQUIRE(rowAlign >= 0 && rowAlign < rs, "invalid row alignment ", rowAlign);
    viewing_ = false;
    Empty();
    root_ = root;
    h_ = height;
    w_ = width;
    calign_ = colAlign;
    ralign_ = rowAlign;
    cconstr_ = rconstr_ = true;
    SetLocalSizes();
    ELX_REQUIRE(ldim >= (lh_ > 0 ? lh_ : 1), "Leading dimension must be no less than height (", ldim, " < ",
                lh_, ")");
    ELX_REQUIRE(buffer != nullptr || lh_ * lw_ == 0, "null buffer for a nonempty local block");
    ld_ = ldim;
    offset_ = 0;
    buf_ = std::make_shared<elx::Buffer>();
    if (lh_ * lw_ > 0) buf_->Wrap(dev_, buffer, static_cast<size_t>(ldim * (lw_ - 1) + lh_) * ElemSize());
    viewing_ = true;
}

void DistMatrix::AlignCols(int colAlign, bool constrain) {
    ELX_REQUIRE(colAlign >= 0 && colAlign < ColStride(), "invalid col alignment ", colAlign);
    ELX_REQUIRE(!(viewing_ && colAlign != calign_), "Tried to realign a view");
    if (colAlign != calign_) {  // data is invalidated (ElementMatrix.cpp:199-213)
        h_ = w_ = 0;
        buf_.reset();
        ld_ = 1;
    }
    calign_ = colAlign;
    if (constrain) cconstr_ = true;
    SetLocalSizes();
}
void DistMatrix::AlignRows(int rowAlign, bool constrain) {
    ELX_REQUIRE(rowAlign >= 0 && rowAlign < RowStride(), "invalid row alignment ", rowAlign);
    ELX_REQUIRE(!(viewing_ && rowAlign != ralign_), "Tried to realign a view");
    if (rowAlign != ralign_) {
        h_ = w_ = 0;
        buf_.reset();
        ld_ = 1;
    }
    ralign_ = rowAlign;
    if (constrain) rconstr_ = true;
    SetLocalSizes();
}
void DistMatrix::Align(int colAlign, int rowAlign, bool constrain) {
    AlignCols(colAlign, constrain);
    AlignRows(rowAlign, constrain);
}

// ElementalMatrix::AlignColsWith / AlignRowsWith (src/core/DistMatrix/ElementMatrix.cpp:243-296)
void DistMatrix::AlignWith(const DistMatrix& o, bool constrain) {
    const Dist U = cdist_, V = rdist_;
    {
        const Dist pc = Partial(U), puc = PartialUnionCol(U, V);
        if (o.cdist_ == U || o.cdist_ == pc) AlignCols(o.calign_ % ColStride(), constrain);
        else if (o.rdist_ == U || o.rdist_ == pc) AlignCols(o.ralign_ % ColStride(), constrain);
        else if (o.cdist_ == puc) AlignCols(o.calign_ % ColStride(), constrain);
        else if (o.rdist_ == puc) AlignCols(o.ralign_ % ColStride(), constrain);
        else if (U != Collect(U) && o.cdist_ != Collect(U) && o.rdist_ != Collect(U))
            throw LogicError("Nonsensical alignment");
    }
    {
        const Dist pr = Partial(V), pur = PartialUnionRow(U, V);
        if (o.cdist_ == V || o.cdist_ == pr) AlignRows(o.calign_ % RowStride(), constrain);
        else if (o.rdist_ == V || o.rdist_ == pr) AlignRows(o.ralign_ % RowStride(), constrain);
        else if (o.cdist_ == pur) AlignRows(o.calign_ % RowStride(), constrain);
        else if (o.rdist_ == pur) AlignRows(o.ralign_ % RowStride(), constrain);
        else if (V != Collect(V) && o.cdist_ != Collect(V) && o.rdist_ != Collect(V))
            throw LogicError("Nonsensical alignment");
    }
}

std::shared_ptr<DistMatrix> DistMatrix::View(const DistMatrix& A, Int i0, Int i1, Int j0, Int j1) {
    ELX_REQUIRE(0 <= i0 && i0 <= i1 && i1 <= A.h_ && 0 <= j0 && j0 <= j1 && j1 <= A.w_,
                "view [", i0, ",", i1, ")x[", j0, ",", j1, ") out of range for ", A.h_, "x", A.w_);
    auto V = std::make_shared<DistMatrix>(A.grid_, A.dtype_, A.cdist_, A.rdist_, A.dev_, A.root_);
    V->stream_ = A.stream_;
    V->h_ = i1 - i0;
    V->w_ = j1 - j0;
    V->calign_ = static_cast<int>((A.calign_ + i0) % A.ColStride());
    V->ralign_ = static_cast<int>((A.ralign_ + j0) % A.RowStride());
    V->cconstr_ = V->rconstr_ = true;
    V->viewing_ = true;
    V->SetLocalSizes();
    V->buf_ = A.buf_;
    V->ld_ = A.ld_;
    if (A.Participating()) {
        const Int rowOff = Length(i0, A.ColShift(), A.ColStride());  // LocalRowOffset
        const Int colOff = Length(j0, A.RowShift(), A.RowStride());
        V->offset_ = A.offset_ + rowOff + colOff * A.ld_;
    } else {
        V->offset_ = A.offset_;
    }
    return V;
}

std::shared_ptr<DistMatrix> DistMatrix::ViewOn(const DistMatrix& A, std::shared_ptr<Grid> g) {
    ELX_REQUIRE(g && g->Height() == A.G().Height() && g->Width() == A.G().Width() &&
                    g->VCRank() == A.G().VCRank() && g->Order() == A.G().Order(),
                "ViewOn: grids differ in shape or rank");
    auto V = View(A, 0, A.h_, 0, A.w_);
    V->grid_ = std::move(g);
    return V;
}

void DistMatrix::SetStream(hipStream_t s) {
    if (dev_ != Device::GPU || s == stream_) return;
    if (buf_ && buf_->data()) {
        StreamFence(stream_, s);
        if (!viewing_ && buf_->stream() == stream_) buf_->Rebind(s);
    }
    stream_ = s;
}

std::shared_ptr<DistMatrix> DistMatrix::Like(Dist cd, Dist rd) const {
    // the root carries over only within the same distribution (a CIRC root or a
    // diagonal index means nothing to another pair)
    auto B = std::make_shared<DistMatrix>(grid_, dtype_, cd, rd, dev_, cd == cdist_ && rd == rdist_ ? root_ : 0);
    B->stream_ = stream_;
    return B;
}

std::shared_ptr<DistMatrix> DistMatrix::LikeOn(Dist cd, Dist rd, Device dev) const {
    if (dev == dev_) return Like(cd, rd);
    return std::make_shared<DistMatrix>(grid_, dtype_, cd, rd, dev, cd == cdist_ && rd == rdist_ ? root_ : 0);
}

void DistMatrix::SetLocal(const void* host, Int ld) {
    if (lh_ == 0 || lw_ == 0) return;
    ELX_REQUIRE(ld >= lh_, "leading dimension ", ld, " < local height ", lh_);
    const size_t es = ElemSize();
    if (dev_ == Device::GPU) {
        ELX_CHECK_HIP(hipMemcpy2DAsync(Buffer(), ld_ * es, host, ld * es, lh_ * es, lw_, hipMemcpyHostToDevice,
                                       stream_));
        ELX_CHECK_HIP(hipStreamSynchronize(stream_));
    } else {
        for (Int j = 0; j < lw_; ++j)
            std::memcpy(static_cast<char*>(Buffer()) + j * ld_ * es, static_cast<const char*>(host) + j * ld * es,
                        lh_ * es);
    }
}

void DistMatrix::GetLocal(void* host, Int ld) const {
    if (lh_ == 0 || lw_ == 0) return;
    ELX_REQUIRE(ld >= lh_, "leading dimension ", ld, " < local height ", lh_);
    const size_t es = ElemSize();
    if (dev_ == Device::GPU) {
        ELX_CHECK_HIP(hipMemcpy2DAsync(host, ld * es, Buffer(), ld_ * es, lh_ * es, lw_, hipMemcpyDeviceToHost,
                                       stream_));
        ELX_CHECK_HIP(hipStreamSynchronize(stream_));
    } else {
        for (Int j = 0; j < lw_; ++j)
            std::memcpy(static_cast<char*>(host) + j * ld * es,
                        static_cast<const char*>(Buffer()) + j * ld_ * es, lh_ * es);
    }
}

void DistMatrix::FillHash(uint64_t seed, double center, double radius) {
    if (lh_ == 0 || lw_ == 0) return;
    exec::FillHash(dev_, dtype_, lh_, lw_, Buffer(), ld_, ColShift(), ColStride(), RowShift(), RowStride(), seed,
                   center, radius, stream_);
}

void DistMatrix::Synchronize() const {
    if (dev_ == Device::GPU) ELX_CHECK_HIP(hipStreamSynchronize(stream_));
}

}  // namespace elx
