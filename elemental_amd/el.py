"""Thin Python mirror of the El:: objects on the GEMM path, over the C-ABI.

Names and argument meaning follow the reference's C++ API (El::Grid,
El::DistMatrix<T,U,V,ELEMENT,D>, El::Gemm, El::Axpy, ...), so parity tests
read like the reference's own tests (tests/blas_like/Gemm.cpp,
tests/core/DistMatrix.cpp).  All work happens in libelemental_amd.so; this
module only moves handles and host arrays.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_double, c_int, c_int64, c_size_t, c_ubyte, c_void_p

import numpy as np

from . import _lib as L
from ._lib import (ADJOINT, BF16, CIRC, COLUMN_MAJOR, CPU, F16, F32, F64, GEMM_CANNON, GEMM_DEFAULT,
                   GEMM_SUMMA_A, GEMM_SUMMA_A_MS, GEMM_SUMMA_B, GEMM_SUMMA_B_MS, GEMM_SUMMA_C,
                   GEMM_SUMMA_C_MS, GEMM_SUMMA_DOT, GPU, MC, MD, MR, NORMAL, ROW_MAJOR, STAR, TRANSPOSE,
                   FILE_AUTO, FILE_BINARY, FILE_BINARY_FLAT, LOWER, UPPER, LEFT, RIGHT, NON_UNIT, UNIT,
                   VC, VR, call, lib)

__all__ = [
    "Comm", "Grid", "DistMatrix", "Gemm", "LocalGemm", "Axpy", "Scale", "Zero", "Fill", "Hadamard",
    "EntrywiseMap", "Combine", "AxpyContract", "InitializeRandom", "Uniform", "Transpose", "SetBlocksize",
    "Blocksize", "PushBlocksizeStack", "PopBlocksizeStack", "EmptyBlocksizeStack", "Initialize", "Finalize",
    "SetComputePanel", "FrobeniusNorm", "Syrk", "Herk", "Syr2k", "Her2k", "Trrk", "Trsm", "Symm", "Hemm", "ScaleTrapezoid", "LEFT", "RIGHT", "NON_UNIT", "UNIT", "LOWER", "UPPER",
    "NORMAL", "TRANSPOSE", "ADJOINT", "MC", "MD", "MR", "VC", "VR", "STAR", "CIRC", "CPU", "GPU",
    "F32", "F64", "F16", "BF16", "GEMM_DEFAULT", "GEMM_SUMMA_A", "GEMM_SUMMA_A_MS", "GEMM_SUMMA_B",
    "GEMM_SUMMA_B_MS", "GEMM_SUMMA_C", "GEMM_SUMMA_C_MS", "GEMM_SUMMA_DOT", "GEMM_CANNON",
    "ROW_MAJOR", "COLUMN_MAJOR", "FILE_AUTO", "FILE_BINARY", "FILE_BINARY_FLAT", "Write", "Read", "DIST_NAMES", "VALID_DISTS", "cross_size", "np_dtype",
]

DIST_NAMES = {MC: "MC", MD: "MD", MR: "MR", VC: "VC", VR: "VR", STAR: "STAR", CIRC: "CIRC"}
# the 14 element-wise distributions of the reference (ElementMatrix/*.cpp)
VALID_DISTS = [(MC, MR), (MC, STAR), (MR, MC), (MR, STAR), (STAR, MC), (STAR, MR), (STAR, STAR),
               (STAR, VC), (STAR, VR), (VC, STAR), (VR, STAR), (CIRC, CIRC), (MD, STAR), (STAR, MD)]


def cross_size(U: int, V: int, r: int, c: int) -> int:
    """How many roots a [U,V] matrix can have: CIRC -> any rank, MD -> the gcd(r,c)
    diagonals (CrossComm = MDPerp), otherwise 1 (AbstractDistMatrix::SetRoot)."""
    from math import gcd
    if U == CIRC:
        return r * c
    if MD in (U, V):
        return gcd(r, c)
    return 1


def np_dtype(t: int):
    """Host storage dtype (bf16 travels as uint16 bit patterns)."""
    return {F32: np.float32, F64: np.float64, F16: np.float16, BF16: np.uint16}[t]


# --------------------------------------------------------------------- comm
class Comm:
    """World communicator: RCCL (device buffers), host bridge, or self."""

    def __init__(self, handle, keepalive=None):
        self.h = handle
        self._keep = keepalive

    @classmethod
    def self_comm(cls) -> "Comm":
        h = c_void_p()
        call("elx_comm_init_host", byref(h), 0, 1, L.HOST_COLL_FN(), L.HOST_SPLIT_FN(), None)
        return cls(h)

    @staticmethod
    def unique_id() -> bytes:
        buf = (c_ubyte * 128)()
        call("elx_comm_unique_id", buf)
        return bytes(buf)

    @classmethod
    def rccl(cls, rank: int, size: int, uid: bytes) -> "Comm":
        h = c_void_p()
        buf = (c_ubyte * 128).from_buffer_copy(uid)
        call("elx_comm_init_rccl", byref(h), rank, size, buf)
        return cls(h)

    @classmethod
    def world(cls) -> "Comm":
        """El::mpi::COMM_WORLD: the library's world communicator (borrowed)."""
        h = c_void_p()
        call("elx_comm_world", byref(h))
        return cls(h)

    def install_as_world(self):
        """Make this communicator the one COMM_WORLD names."""
        call("elx_comm_set_world", self.h)

    @classmethod
    def host(cls, bridge) -> "Comm":
        """`bridge` implements the collectives (see torch_bridge.GlooBridge)."""
        h = c_void_p()
        call("elx_comm_init_host", byref(h), bridge.rank, bridge.size, bridge.coll_fn, bridge.split_fn, None)
        return cls(h, keepalive=bridge)

    @property
    def rank(self) -> int:
        r = c_int()
        call("elx_comm_rank", self.h, byref(r))
        return r.value

    @property
    def size(self) -> int:
        s = c_int()
        call("elx_comm_size", self.h, byref(s))
        return s.value

    def barrier(self):
        call("elx_comm_barrier", self.h)

    # typed collectives on host (numpy) buffers for host comms, device pointers
    # (ints) for RCCL comms; counts in elements (El::mpi::*, src/core/imports/mpi)
    def split(self, color: int, key: int) -> "Comm":
        h = c_void_p()
        call("elx_comm_split", self.h, color, key, byref(h))
        return Comm(h, keepalive=self)

    def allgather(self, dtype: int, send, recv, count: int, stream=None):
        call("elx_comm_allgather", self.h, dtype, _ptr(send), _ptr(recv), count, stream)

    def reduce_scatter(self, dtype: int, send, recv, count: int, stream=None):
        call("elx_comm_reduce_scatter", self.h, dtype, _ptr(send), _ptr(recv), count, stream)

    def allreduce(self, dtype: int, send, recv, count: int, stream=None):
        call("elx_comm_allreduce", self.h, dtype, _ptr(send), _ptr(recv), count, stream)

    def bcast(self, dtype: int, buf, count: int, root: int, stream=None):
        call("elx_comm_bcast", self.h, dtype, _ptr(buf), count, root, stream)

    def alltoall(self, dtype: int, send, recv, count: int, stream=None):
        call("elx_comm_alltoall", self.h, dtype, _ptr(send), _ptr(recv), count, stream)

    def sendrecv(self, dtype: int, send, dest: int, recv, src: int, count: int, stream=None):
        call("elx_comm_sendrecv", self.h, dtype, _ptr(send), dest, _ptr(recv), src, count, stream)


def _ptr(x):
    """numpy array -> its data pointer; int / None -> as is (device pointers)."""
    if isinstance(x, np.ndarray):
        return x.ctypes.data_as(c_void_p)
    return x


# --------------------------------------------------------------------- grid
class Grid:
    """El::Grid(comm, height, order); height 0 -> Grid::DefaultHeight."""

    def __init__(self, comm: Comm | None = None, height: int = 0, order: int = COLUMN_MAJOR):
        self.comm = comm or Comm.self_comm()
        h = c_void_p()
        call("elx_grid_create", byref(h), self.comm.h, height, order)
        self.h = h
        info = (c_int * 8)()
        call("elx_grid_info", self.h, info)
        (self.height, self.width, self.size, self.rank, self.mc_rank, self.mr_rank, self.vc_rank,
         self.vr_rank) = list(info)

    @staticmethod
    def default_height(size: int) -> int:
        return lib().elx_grid_default_height(size)

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().elx_grid_destroy(self.h)
                self.h = None
        except Exception:
            pass


# --------------------------------------------------------------- distmatrix
class DistMatrix:
    """El::DistMatrix<T,U,V,ELEMENT,D>(grid, root)."""

    def __init__(self, grid: Grid, dtype: int = F64, U: int = MC, V: int = MR, device: int = GPU,
                 root: int = 0, height: int = 0, width: int = 0, _handle=None, _parent=None):
        self.grid, self.dtype, self.U, self.V, self.device, self.root = grid, dtype, U, V, device, root
        self._parent = _parent  # keep the viewed matrix alive
        if _handle is None:
            h = c_void_p()
            call("elx_dm_create", byref(h), grid.h, dtype, U, V, device, root)
            self.h = h
            if height or width:
                self.Resize(height, width)
        else:
            self.h = _handle

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().elx_dm_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # -- metadata
    def info(self) -> dict:
        v = (c_int64 * 13)()
        call("elx_dm_info", self.h, v)
        keys = ["height", "width", "local_height", "local_width", "ldim", "col_align", "row_align",
                "col_shift", "row_shift", "col_stride", "row_stride", "participating", "viewing"]
        return dict(zip(keys, list(v)))

    def Height(self): return self.info()["height"]
    def Width(self): return self.info()["width"]
    def LocalHeight(self): return self.info()["local_height"]
    def LocalWidth(self): return self.info()["local_width"]
    def ColAlign(self): return self.info()["col_align"]
    def RowAlign(self): return self.info()["row_align"]
    def ColShift(self): return self.info()["col_shift"]
    def RowShift(self): return self.info()["row_shift"]
    def LDim(self): return self.info()["ldim"]

    def Buffer(self) -> int:
        p = c_void_p()
        call("elx_dm_buffer", self.h, byref(p))
        return p.value or 0

    # -- shape / alignment
    def Align(self, col_align: int, row_align: int, constrain: bool = True):
        call("elx_dm_align", self.h, col_align, row_align, int(constrain))
        return self

    def AlignWith(self, other: "DistMatrix", constrain: bool = True):
        call("elx_dm_align_with", self.h, other.h, int(constrain))
        return self

    def Resize(self, height: int, width: int):
        call("elx_dm_resize", self.h, height, width)
        return self

    # -- data
    def set_local(self, arr: np.ndarray):
        arr = np.asfortranarray(arr, dtype=np_dtype(self.dtype))
        i = self.info()
        assert arr.shape == (i["local_height"], i["local_width"]), (arr.shape, i)
        call("elx_dm_set_local", self.h, arr.ctypes.data_as(c_void_p), max(arr.shape[0], 1))

    def get_local(self) -> np.ndarray:
        i = self.info()
        out = np.zeros((i["local_height"], i["local_width"]), dtype=np_dtype(self.dtype), order="F")
        call("elx_dm_get_local", self.h, out.ctypes.data_as(c_void_p), max(out.shape[0], 1))
        return out

    def fill_hash(self, seed: int, center: float = 0.0, radius: float = 1.0):
        """Grid-independent synthetic fill: A(i,j) = center + radius*u(seed,i,j)."""
        call("elx_dm_fill_hash", self.h, seed, center, radius)
        return self

    def synchronize(self):
        call("elx_dm_synchronize", self.h)

    def set_stream(self, stream: int | None):
        """El::SetSyncInfo: queue this matrix's work on `stream` (a hipStream_t
        handle, e.g. torch.cuda.Stream().cuda_stream; None = the library's)."""
        call("elx_dm_set_stream", self.h, stream)

    def stream(self) -> int | None:
        """El::SyncInfoFromMatrix: the hipStream_t this matrix's work runs on."""
        s = ctypes.c_void_p()
        call("elx_dm_stream", self.h, ctypes.byref(s))
        return s.value

    def __call__(self, rows, cols) -> "DistMatrix":
        """A(IR(i0,i1), IR(j0,j1)) view; rows/cols are (start, stop) or slice(None)."""
        i = self.info()
        r0, r1 = (0, i["height"]) if rows is None or rows == slice(None) else rows
        c0, c1 = (0, i["width"]) if cols is None or cols == slice(None) else cols
        h = c_void_p()
        call("elx_dm_view", byref(h), self.h, r0, r1, c0, c1)
        return DistMatrix(self.grid, self.dtype, self.U, self.V, self.device, self.root, _handle=h, _parent=self)

    def attach(self, height: int, width: int, col_align: int, row_align: int, ptr: int, ldim: int,
               root: int = 0) -> "DistMatrix":
        """View caller storage at address `ptr` (device pointer for GPU matrices)
        as the local block (ElementalMatrix::Attach); the caller keeps it alive."""
        call("elx_dm_attach", self.h, height, width, col_align, row_align, ptr, ldim, root)
        self.root = root
        return self

    def assign(self, other: "DistMatrix") -> "DistMatrix":
        """self = other  (DistMatrix::operator=, any distribution pair)."""
        call("elx_dm_copy", self.h, other.h)
        return self

    def Get(self, i: int, j: int) -> float:
        """A.Get(i, j): collective; every rank returns the entry (setup.hpp:463-490)."""
        v = c_double()
        call("elx_dm_get", self.h, i, j, byref(v))
        return v.value

    def Set(self, i: int, j: int, value: float):
        """A.Set(i, j, value): ranks holding (i, j) write it; not collective."""
        call("elx_dm_set", self.h, i, j, float(value))

    def Update(self, i: int, j: int, value: float):
        """A.Update(i, j, value): A(i,j) += value on the ranks holding it."""
        call("elx_dm_update", self.h, i, j, float(value))

    def like(self, U=None, V=None, device=None) -> "DistMatrix":
        U = self.U if U is None else U
        V = self.V if V is None else V
        same = (U, V) == (self.U, self.V)  # a root means nothing to another distribution
        return DistMatrix(self.grid, self.dtype, U, V, self.device if device is None else device,
                          self.root if same else 0)


# ------------------------------------------------------------ front doors
def Gemm(orientA, orientB, alpha, A: DistMatrix, B: DistMatrix, beta, C: DistMatrix,
         alg: int = GEMM_DEFAULT) -> int:
    """El::Gemm(orientA, orientB, alpha, A, B, beta, C, alg); returns the algorithm run."""
    call("elx_gemm", orientA, orientB, float(alpha), A.h, B.h, float(beta), C.h, alg)
    return lib().elx_last_gemm_algorithm()


def LocalGemm(orientA, orientB, alpha, A, B, beta, C):
    call("elx_local_gemm", orientA, orientB, float(alpha), A.h, B.h, float(beta), C.h)


def Syrk(uplo, orientation, alpha, A: DistMatrix, beta, C: DistMatrix, conjugate: bool = False):
    """El::Syrk(uplo, orientation, alpha, A, beta, C, conjugate) (Syrk.cpp:196-211):
    C := alpha op(A) op(A)^T + beta C on C's uplo triangle; the other triangle is untouched."""
    call("elx_syrk", uplo, orientation, float(alpha), A.h, float(beta), C.h, int(bool(conjugate)))


def Herk(uplo, orientation, alpha, A: DistMatrix, beta, C: DistMatrix):
    """El::Herk (Herk.cpp): Syrk with conjugation, identical for the real types."""
    Syrk(uplo, orientation, alpha, A, beta, C, conjugate=True)


def Trrk(uplo, orientA, orientB, alpha, A: DistMatrix, B: DistMatrix, beta, C: DistMatrix):
    """El::Trrk(uplo, orientA, orientB, alpha, A, B, beta, C) (Trrk.cpp:100-117)."""
    call("elx_trrk", uplo, orientA, orientB, float(alpha), A.h, B.h, float(beta), C.h)


def Syr2k(uplo, orientation, alpha, A: DistMatrix, B: DistMatrix, beta, C: DistMatrix, conjugate: bool = False):
    """El::Syr2k (Syr2k.cpp:78-93): C := alpha (op(A) op(B)^T + op(B) op(A)^T) + beta C on uplo."""
    call("elx_syr2k", uplo, orientation, float(alpha), A.h, B.h, float(beta), C.h, int(bool(conjugate)))


def Her2k(uplo, orientation, alpha, A: DistMatrix, B: DistMatrix, beta, C: DistMatrix):
    """El::Her2k: Syr2k with conjugation, identical for the real types."""
    Syr2k(uplo, orientation, alpha, A, B, beta, C, conjugate=True)


def Trsm(side, uplo, orientation, diag, alpha, A: DistMatrix, B: DistMatrix, checkIfSingular: bool = False):
    """El::Trsm(side, uplo, orientation, diag, alpha, A, B, checkIfSingular) (Trsm.cpp:129-420):
    B is overwritten with alpha op(A)^-1 B (LEFT) or alpha B op(A)^-1 (RIGHT);
    checkIfSingular raises SingularMatrixError on an exact zero NON_UNIT diagonal."""
    call("elx_trsm", side, uplo, orientation, diag, float(alpha), A.h, B.h, int(bool(checkIfSingular)))


def Symm(side, uplo, alpha, A: DistMatrix, B: DistMatrix, beta, C: DistMatrix, conjugate: bool = False):
    """El::Symm(side, uplo, alpha, A, B, beta, C) (Symm.cpp:55-80): A symmetric, uplo stored."""
    call("elx_symm", side, uplo, float(alpha), A.h, B.h, float(beta), C.h, int(bool(conjugate)))


def Hemm(side, uplo, alpha, A: DistMatrix, B: DistMatrix, beta, C: DistMatrix):
    """El::Hemm: Symm with conjugation, identical for the real types."""
    Symm(side, uplo, alpha, A, B, beta, C, conjugate=True)


def ScaleTrapezoid(alpha, uplo, A: DistMatrix, offset: int = 0):
    """El::ScaleTrapezoid(alpha, uplo, A, offset) (ScaleTrapezoid.hpp:47-88)."""
    call("elx_dm_scale_trapezoid", float(alpha), uplo, A.h, int(offset))


def Axpy(alpha, X: DistMatrix, Y: DistMatrix):
    call("elx_dm_axpy", float(alpha), X.h, Y.h)


def Scale(alpha, A: DistMatrix):
    call("elx_dm_scale", float(alpha), A.h)


def Zero(A: DistMatrix):
    call("elx_dm_zero", A.h)


def Fill(A: DistMatrix, alpha):
    """El::Fill(A, alpha) (include/El/blas_like/level1/Fill.hpp:66-70)."""
    call("elx_dm_fill", A.h, float(alpha))


def Hadamard(A, B, C):
    call("elx_dm_hadamard", A.h, B.h, C.h)


def EntrywiseMap(fn: int, A, B):
    call("elx_dm_entrywise_map", fn, A.h, B.h)


def InitializeRandom(deterministic: bool = True, world_rank: int = 0):
    """El::InitializeRandom: seed (21 << 16) | rank when deterministic (random.cpp:24-35)."""
    call("elx_initialize_random", int(deterministic), world_rank)


def Uniform(A, height: int, width: int, center: float = 0.0, radius: float = 1.0):
    """El::Uniform: the reference's mt19937 draws on RedundantRank 0, broadcast."""
    call("elx_dm_uniform", A.h, height, width, center, radius)
    return A


def Write(A, basename: str = "matrix", fmt: int = L.FILE_BINARY, int_bytes: int = 4):
    """El::Write in the reference's BINARY (basename.bin: Int h, Int w, column-major
    data) or BINARY_FLAT (basename.dat) format; int_bytes = sizeof(El::Int)."""
    call("elx_dm_write", A.h, basename.encode(), fmt, int_bytes)


def Read(A, filename: str, fmt: int = L.FILE_AUTO, int_bytes: int = 4):
    """El::Read of a BINARY / BINARY_FLAT file into A's distribution and device."""
    call("elx_dm_read", A.h, filename.encode(), fmt, int_bytes)
    return A


def Combine(fn: int, A, B):
    """B := f(A, B) entrywise on matching local blocks (ELX_COMBINE_* functors)."""
    call("elx_dm_combine", fn, A.h, B.h)


def AxpyContract(alpha, A, B):
    call("elx_dm_axpy_contract", float(alpha), A.h, B.h)


def Copy(A: DistMatrix, B: DistMatrix):
    """B := A (El::Copy): any distribution pair; different element types convert
    with one rounding (CopyDistMatrix.hpp:28-57)."""
    call("elx_dm_copy", B.h, A.h)


def Transpose(A, B):
    call("elx_dm_transpose", A.h, B.h)


def SetBlocksize(nb: int):
    call("elx_set_blocksize", nb)


def Blocksize() -> int:
    nb = lib().elx_blocksize()
    if nb < 0:
        raise L.LogicError(L.ERR_LOGIC, lib().elx_last_error().decode(errors="replace"))
    return nb


def PushBlocksizeStack(nb: int):
    call("elx_push_blocksize", nb)


def PopBlocksizeStack():
    call("elx_pop_blocksize")


def EmptyBlocksizeStack():
    call("elx_empty_blocksize_stack")


def Initialize():
    """El::Initialize: world communicator from RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_ADDR (RCCL; size 1 without them), blocksize stack {128}, RNG seeded."""
    call("elx_initialize")


def Finalize():
    call("elx_finalize")


def watchdog_stage(name: str, seconds: float = 0.0):
    """Arm the stage watchdog: past `seconds` (or on an asynchronous RCCL error)
    every owned RCCL communicator is aborted and the process exits with
    WATCHDOG_EXIT, naming the stage on stderr; seconds <= 0 disarms."""
    call("elx_watchdog_stage", name.encode(), float(seconds))


WATCHDOG_EXIT = 75


def watchdog_epitaph(text: str | None, exit_code: int = WATCHDOG_EXIT):
    """Text the watchdog prints to stdout before exiting, and its exit status then."""
    call("elx_watchdog_epitaph", (text or "").encode(), int(exit_code))


def rendezvous_bcast(data: bytes | None, nbytes: int, rank: int, size: int, addr: str, port: int,
                     timeout: float = 60.0) -> bytes:
    """Rank 0's `data` (nbytes) to every rank over TCP (rank 0 listens on port)."""
    buf = (c_ubyte * nbytes)()
    if rank == 0:
        ctypes.memmove(buf, data, nbytes)
    call("elx_rendezvous_bcast", buf, nbytes, rank, size, addr.encode(), port, float(timeout))
    return bytes(buf)


def FrobeniusNorm(A: DistMatrix) -> float:
    """El::FrobeniusNorm (collective over A's grid; scaled sum of squares)."""
    v = c_double()
    call("elx_dm_frobenius_norm", A.h, byref(v))
    return v.value


def SetComputePanel(kc: int):
    call("elx_set_compute_panel", kc)


def SetStreamPoolSize(n: int):
    """Size of the multistream pool (H_STREAMPOOL_SIZE; 0 = read the variable)."""
    call("elx_set_stream_pool_size", n)


def StreamPoolSize() -> int:
    return lib().elx_stream_pool_size()


def comm_stats() -> dict:
    b, s, c = c_int64(), c_double(), c_int64()
    call("elx_comm_stats", byref(b), byref(s), byref(c))
    return {"bytes": b.value, "seconds": s.value, "calls": c.value}


def comm_stats_reset():
    call("elx_comm_stats_reset")


def device_count() -> int:
    n = c_int()
    call("elx_device_count", byref(n))
    return n.value


def device_synchronize():
    call("elx_device_synchronize")


def pool_stats() -> tuple[int, int]:
    r, u = c_size_t(), c_size_t()
    call("elx_pool_stats", byref(r), byref(u))
    return r.value, u.value


def pool_backing_reserved() -> int:
    """Bytes the allocator holds from the driver (live + cached blocks)."""
    r = c_size_t()
    call("elx_pool_backing_reserved", byref(r))
    return r.value
