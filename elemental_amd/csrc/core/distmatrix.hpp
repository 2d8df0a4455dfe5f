// El::Grid and the element-wise El::DistMatrix<T,U,V,ELEMENT,D> (type-erased:
// dtype, distributions and device are runtime fields so one C-ABI handle covers
// every instantiation the reference compiles).
//
// Layout conventions follow the reference exactly (bit-exact redistributions):
//   * global (i,j) lives on column-rank (i + colAlign) mod colStride and
//     row-rank (j + rowAlign) mod rowStride (src/core/DistMatrix/ElementMatrix.cpp:604-618);
//   * local storage is column-major, local row iLoc <-> global colShift + iLoc*colStride
//     with Shift(rank, align, stride) = (rank - align) mod stride and
//     Length(n, shift, stride) = n > shift ? (n - shift - 1)/stride + 1 : 0
//     (include/El/core/indexing/impl.hpp:33-36,244-245);
//   * grid ranks are column-major: vcRank = mcRank + r*mrRank,
//     vrRank = mrRank + c*mcRank (src/core/Grid.cpp:147-148).
#pragma once
#include "../common.hpp"
#include "../runtime/runtime.hpp"
#include "../comm/comm.hpp"
#include <memory>
#include <vector>

namespace elx {

enum class Dist : int { MC = ELX_MC, MD = ELX_MD, MR = ELX_MR, VC = ELX_VC, VR = ELX_VR, STAR = ELX_STAR, CIRC = ELX_CIRC };
const char* DistName(Dist d);

inline Int Mod(Int a, Int b) { Int r = a % b; return r < 0 ? r + b : r; }
inline Int Shift(Int rank, Int align, Int stride) { return Mod(rank - align, stride); }
inline Int Length(Int n, Int shift, Int stride) { return n > shift ? (n - shift - 1) / stride + 1 : 0; }
inline Int MaxLength(Int n, Int stride) { return n > 0 ? (n - 1) / stride + 1 : 0; }

class Grid {
public:
    Grid(std::shared_ptr<Comm> world, int height, int order);
    static int DefaultHeight(int size);

    int Height() const { return r_; }
    int Width() const { return c_; }
    int Size() const { return p_; }
    int MCRank() const { return mc_; }
    int MRRank() const { return mr_; }
    int VCRank() const { return mc_ + r_ * mr_; }
    int VRRank() const { return mr_ + c_ * mc_; }
    int Rank() const { return VCRank(); }
    // grid coordinates of the rank with VC rank q
    int MCOf(int vc) const { return vc % r_; }
    int MROf(int vc) const { return vc / r_; }
    int VROf(int vc) const { return MROf(vc) + c_ * MCOf(vc); }
    // diagonals (Grid.cpp:105-107,157-185): gcd(r,c) diagonals of lcm(r,c)
    // ranks each; rank (mc,mr) lies on diagonal mod(mr - mc, gcd) at the
    // position reached walking (0, diag) -> (+1, +1) mod (r, c)
    int GCD() const { return gcd_; }
    int LCM() const { return p_ / gcd_; }
    int MDRankOf(int vc) const { return md_rank_[vc]; }
    int MDPerpOf(int vc) const { return md_perp_[vc]; }
    int MDRank() const { return MDRankOf(VCRank()); }
    int MDPerpRank() const { return MDPerpOf(VCRank()); }

    Comm& MC() const { return *mc_comm_; }
    Comm& MR() const { return *mr_comm_; }
    Comm& VC() const { return *vc_comm_; }
    Comm& VR() const { return *vr_comm_; }
    Comm& World() const { return *world_; }
    std::shared_ptr<Comm> WorldPtr() const { return world_; }
    Device CommDevice() const;  // where the comms expect buffers (GPU for RCCL)
    int Order() const { return order_; }

    // stride / this rank's coordinate / comm of a distribution
    int Stride(Dist d) const;
    int DistRank(Dist d) const { return DistRankOf(d, VCRank()); }
    int DistRankOf(Dist d, int vc) const;
    Comm& DistComm(Dist d) const;

private:
    std::shared_ptr<Comm> world_, mc_comm_, mr_comm_, vc_comm_, vr_comm_;
    int r_ = 1, c_ = 1, p_ = 1, mc_ = 0, mr_ = 0, order_ = ELX_COLUMN_MAJOR, gcd_ = 1;
    std::vector<int> md_rank_, md_perp_;
};

class DistMatrix {
public:
    DistMatrix(std::shared_ptr<Grid> g, DType t, Dist colDist, Dist rowDist, Device dev, int root = 0);
    // A matrix whose stream differs from the one its pool storage is returned
    // on (a view queued on another stream) orders that stream after its own
    // work before letting go of the storage, so the free's event covers it.
    ~DistMatrix();
    DistMatrix(const DistMatrix&) = delete;
    DistMatrix& operator=(const DistMatrix&) = delete;

    // ---- distribution metadata ----
    const Grid& G() const { return *grid_; }
    std::shared_ptr<Grid> GridPtr() const { return grid_; }
    DType Type() const { return dtype_; }
    Dist ColDist() const { return cdist_; }
    Dist RowDist() const { return rdist_; }
    Device Dev() const { return dev_; }
    int Root() const { return root_; }
    Int Height() const { return h_; }
    Int Width() const { return w_; }
    int ColAlign() const { return calign_; }
    int RowAlign() const { return ralign_; }
    bool ColConstrained() const { return cconstr_; }
    bool RowConstrained() const { return rconstr_; }
    int ColStride() const;
    int RowStride() const;
    int ColRank() const { return ColRankOf(G().VCRank()); }
    int RowRank() const { return RowRankOf(G().VCRank()); }
    int CrossSize() const;         // number of roots a matrix of this distribution can have
    bool CrossOf(int vc) const;    // does rank vc lie in the root slice (CIRC root / root diagonal)?
    int ColRankOf(int vc) const;   // -1 when that rank holds nothing (CIRC non-root, off-root diagonal)
    int RowRankOf(int vc) const;
    int ColShift() const { return (int)Shift(ColRank(), calign_, ColStride()); }
    int RowShift() const { return (int)Shift(RowRank(), ralign_, RowStride()); }
    bool Participating() const { return ColRank() >= 0 && RowRank() >= 0; }
    bool ParticipatingOf(int vc) const { return ColRankOf(vc) >= 0 && RowRankOf(vc) >= 0; }
    Int LocalHeight() const { return lh_; }
    Int LocalWidth() const { return lw_; }
    Int LocalHeightOf(int vc) const;
    Int LocalWidthOf(int vc) const;
    Int LDim() const { return ld_; }
    bool Viewing() const { return viewing_; }

    // ---- storage ----
    void* Buffer() const;
    hipStream_t Stream() const { return stream_; }
    // Move the matrix to stream s (SetSyncInfo): with allocated storage, s is
    // first ordered after the old stream's queued work, and pool storage this
    // matrix owns is returned on s from then on.  (The reference refuses the
    // move once CUB memory is allocated, Memory/impl.hpp:305-316; here it is
    // fenced instead.)  A view moves alone: its storage stays with its owner,
    // and ~DistMatrix orders the owner's stream after the view's work.
    void SetStream(hipStream_t s);
    size_t ElemSize() const { return DTypeSize(dtype_); }

    // ---- realignment / resize (ElementMatrix.cpp:170-370 semantics) ----
    void Align(int colAlign, int rowAlign, bool constrain);
    void AlignCols(int colAlign, bool constrain);
    void AlignRows(int rowAlign, bool constrain);
    void AlignWith(const DistMatrix& other, bool constrain);
    void Resize(Int height, Int width);
    void Empty();

    // view caller storage (ElementalMatrix::Attach); the caller keeps ownership
    void Attach(Int height, Int width, int colAlign, int rowAlign, void* buffer, Int ldim, int root);
    // V := A(i0:i1, j0:j1), sharing A's storage
    static std::shared_ptr<DistMatrix> View(const DistMatrix& A, Int i0, Int i1, Int j0, Int j1);
    // all of A, sharing A's storage, on another Grid object of the same shape and
    // rank (a multistream team's grid, whose communicators are duplicates)
    static std::shared_ptr<DistMatrix> ViewOn(const DistMatrix& A, std::shared_ptr<Grid> g);
    // fresh matrix with the same grid/type/device
    std::shared_ptr<DistMatrix> Like(Dist cd, Dist rd) const;
    // same grid/type on device `dev` (this matrix's stream when the device matches)
    std::shared_ptr<DistMatrix> LikeOn(Dist cd, Dist rd, Device dev) const;

    // host <-> local block
    void SetLocal(const void* host, Int ld);
    void GetLocal(void* host, Int ld) const;
    void FillHash(uint64_t seed, double center, double radius);
    void Synchronize() const;

private:
    void SetLocalSizes();
    void Allocate();
    std::shared_ptr<Grid> grid_;
    DType dtype_;
    Dist cdist_, rdist_;
    Device dev_;
    int root_ = 0;
    Int h_ = 0, w_ = 0;
    int calign_ = 0, ralign_ = 0;
    bool cconstr_ = false, rconstr_ = false;
    Int lh_ = 0, lw_ = 0, ld_ = 1;
    std::shared_ptr<elx::Buffer> buf_;
    Int offset_ = 0;  // element offset into buf_ (views)
    bool viewing_ = false;
    hipStream_t stream_ = nullptr;
};

using DM = DistMatrix;
using DMPtr = std::shared_ptr<DistMatrix>;

}  // namespace elx
