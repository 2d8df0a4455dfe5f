"""Python handle on the CPU oracle (oracle.c) — TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
always as the checker; the product (elemental_amd) never imports it.
Parity-pinning status: see the header of oracle.c and DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_char, c_double, c_float, c_int, c_int64, c_uint64, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

MC, MD, MR, VC, VR, STAR, CIRC = range(7)


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        i64, d = c_int64, c_double
        L.orc_shift.restype = i64
        L.orc_shift.argtypes = [i64, i64, i64]
        L.orc_length.restype = i64
        L.orc_length.argtypes = [i64, i64, i64]
        L.orc_max_length.restype = i64
        L.orc_max_length.argtypes = [i64, i64]
        L.orc_default_height.restype = c_int
        L.orc_default_height.argtypes = [c_int]
        L.orc_dist_stride.restype = c_int
        L.orc_dist_stride.argtypes = [c_int, c_int, c_int]
        L.orc_dist_rank.restype = c_int
        L.orc_dist_rank.argtypes = [c_int, c_int, c_int, c_int, c_int]
        L.orc_local_block.restype = None
        L.orc_local_block.argtypes = [c_void_p, i64, i64, i64, i64, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_int, c_int, c_void_p, i64, POINTER(i64), POINTER(i64)]
        L.orc_place_block.restype = None
        L.orc_place_block.argtypes = [c_void_p, i64, i64, i64, i64, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_int, c_int, c_void_p, i64]
        L.orc_hash_unit.restype = d
        L.orc_hash_unit.argtypes = [c_uint64, i64, i64]
        L.orc_hash_fill_f64.restype = None
        L.orc_hash_fill_f64.argtypes = [i64, i64, c_uint64, d, d, c_void_p, i64]
        L.orc_hash_fill_f32.restype = None
        L.orc_hash_fill_f32.argtypes = [i64, i64, c_uint64, d, d, c_void_p, i64]
        L.orc_gemm_f64.restype = None
        L.orc_gemm_f64.argtypes = [c_char, c_char, i64, i64, i64, d, c_void_p, i64, c_void_p, i64, d, c_void_p, i64]
        L.orc_gemm_f32.restype = None
        L.orc_gemm_f32.argtypes = [c_char, c_char, i64, i64, i64, c_float, c_void_p, i64, c_void_p, i64, c_float,
                                   c_void_p, i64]
        L.orc_summa_nnc_f64.restype = None
        L.orc_summa_nnc_f64.argtypes = [c_int, c_int, i64, i64, i64, i64, d, c_void_p, i64, c_void_p, i64, d,
                                        c_void_p, i64]
        L.orc_fro.restype = d
        L.orc_fro.argtypes = [i64, i64, c_void_p, i64]
        L.orc_cpu_gemm_f64.restype = None
        L.orc_cpu_gemm_f64.argtypes = [c_char, c_char, i64, i64, i64, d, c_void_p, i64, c_void_p, i64, d,
                                       c_void_p, i64]
        L.orc_cpu_threads.restype = c_int
        L.orc_cpu_threads.argtypes = []
        L.orc_cpu_set_threads.restype = None
        L.orc_cpu_set_threads.argtypes = [c_int]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(c_void_p)


# ------------------------------------------------------------------ layout
def shift(rank, align, stride):
    return lib().orc_shift(rank, align, stride)


def length(n, shift_, stride):
    return lib().orc_length(n, shift_, stride)


def local_block(G: np.ndarray, U: int, V: int, r: int, c: int, vc: int, col_align=0, row_align=0,
                root=0) -> np.ndarray:
    """Local block of global column-major G on VC rank vc for [U,V] (bit copy)."""
    G = np.asfortranarray(G)
    H, W = G.shape
    out = np.zeros((max(H, 1), max(W, 1)), dtype=G.dtype, order="F")
    lh, lw = c_int64(), c_int64()
    lib().orc_local_block(_p(G), G.itemsize, H, W, max(H, 1), U, V, r, c, vc, col_align, row_align, root,
                          _p(out), out.shape[0], ctypes.byref(lh), ctypes.byref(lw))
    return np.asfortranarray(out[:lh.value, :lw.value])


def place_block(G: np.ndarray, loc: np.ndarray, U, V, r, c, vc, col_align=0, row_align=0, root=0):
    H, W = G.shape
    loc = np.asfortranarray(loc, dtype=G.dtype)
    lib().orc_place_block(_p(G), G.itemsize, H, W, max(H, 1), U, V, r, c, vc, col_align, row_align, root,
                          _p(loc), max(loc.shape[0], 1))


# ------------------------------------------------------------------ inputs
def hash_matrix(H: int, W: int, seed: int, center=0.0, radius=1.0, dtype=np.float64) -> np.ndarray:
    """Global matrix identical to elx_fill_hash / DistMatrix.fill_hash."""
    G = np.zeros((H, W), dtype=np.float64, order="F")
    if H and W:
        lib().orc_hash_fill_f64(H, W, seed, center, radius, _p(G), H)
    if dtype == np.float64:
        return G
    if dtype == np.float32:
        return G.astype(np.float32)
    if dtype == np.float16:  # double -> float (RNE) -> half (RNE), as the device does
        return G.astype(np.float32).astype(np.float16)
    if dtype == "bf16":
        return f32_to_bf16_bits(G.astype(np.float32))
    raise ValueError(dtype)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(np.asarray(x, dtype=np.float32))
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return np.asfortranarray(r)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


# ------------------------------------------------------ type conversion
# Copy_GPU_impl<SrcT,DestT> (src/hydrogen/blas/gpu/Copy.cu:13-21: `dest = src`):
# the exact source value rounded once, to nearest-even, into the target format.
_FMT = {"f32": (24, -126, np.finfo(np.float32).max), "f16": (11, -14, 65504.0),
        "bf16": (8, -126, float.fromhex("0x1.fep127"))}


def round_to_format(d: np.ndarray, fmt: str) -> np.ndarray:
    """Round float64 values to the `fmt` grid (p significand bits, minimum normal
    exponent emin, largest finite maxv) by scaling to the quantum of each value's
    binade and numpy's round-half-even; results stay float64 (exact)."""
    p, emin, maxv = _FMT[fmt]
    d = np.asarray(d, dtype=np.float64)
    _, e = np.frexp(d)                                   # d = m 2^e, 0.5 <= |m| < 1
    q = np.ldexp(1.0, np.maximum(e, emin + 1) - p)       # quantum (subnormals: 2^(emin+1-p))
    with np.errstate(over="ignore", invalid="ignore"):
        r = np.round(d / q) * q
        r = np.where(np.abs(r) > maxv, np.copysign(np.inf, d), r)
    return np.where(np.isfinite(d), r, d)


def to_f64(x: np.ndarray, fmt: str) -> np.ndarray:
    """Storage array (bf16 as uint16 bit patterns) -> exact float64 values."""
    return bf16_bits_to_f32(x).astype(np.float64) if fmt == "bf16" else np.asarray(x).astype(np.float64)


def convert(x: np.ndarray, src: str, dst: str) -> np.ndarray:
    """Type-converting copy of a storage array: src/dst in {f64, f32, f16, bf16}."""
    d = to_f64(x, src)
    if dst == "f64":
        out = d
    elif dst == "bf16":
        out = f32_to_bf16_bits(round_to_format(d, "bf16").astype(np.float32))  # exact -> bits
    else:
        out = round_to_format(d, dst).astype(np.float32 if dst == "f32" else np.float16)
    return np.asfortranarray(out)


# -------------------------------------------------------------------- gemm
def gemm(ta: str, tb: str, alpha, A: np.ndarray, B: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """C := alpha op(A) op(B) + beta C with the reference's loop nest (f64/f32)."""
    C = np.array(C, order="F", copy=True)
    A = np.asfortranarray(A)
    B = np.asfortranarray(B)
    m, n = C.shape
    k = A.shape[1] if ta == "N" else A.shape[0]
    f = lib().orc_gemm_f64 if C.dtype == np.float64 else lib().orc_gemm_f32
    f(ta.encode(), tb.encode(), m, n, k, alpha, _p(A), max(A.shape[0], 1), _p(B), max(B.shape[0], 1), beta,
      _p(C), max(m, 1))
    return C


def syrk(uplo: str, trans: str, alpha, A: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """C := alpha op(A) op(A)^T + beta C on C's uplo ('L'/'U') triangle only, the
    rest of C untouched: BLAS xSYRK semantics, which the reference's CPU path calls
    (Syrk.cpp:20-41 -> blas::Syrk) and its distributed Syrk reproduces
    (Syrk.cpp:196-211: ScaleTrapezoid(beta) then LocalTrrk per panel).  The full
    product comes from the reference GEMM loop nest above."""
    full = gemm(trans, "T" if trans == "N" else "N", alpha, A, A, beta, C)
    n = C.shape[0]
    i, j = np.indices((n, n))
    mask = (i >= j) if uplo == "L" else (i <= j)
    out = np.array(C, order="F", copy=True)
    out[mask] = full[mask]
    return out


def _tri_mask(n: int, uplo: str) -> np.ndarray:
    i, j = np.indices((n, n))
    return (i >= j) if uplo == "L" else (i <= j)


def trrk(uplo: str, ta: str, tb: str, alpha, A: np.ndarray, B: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """El::Trrk (Trrk.cpp:100-117, Trrk/Local.hpp): the GEMM update applied to C's
    uplo triangle only (ScaleTrapezoid(beta) + LocalTrrk per panel)."""
    full = gemm(ta, tb, alpha, A, B, beta, C)
    out = np.array(C, order="F", copy=True)
    mask = _tri_mask(C.shape[0], uplo)
    out[mask] = full[mask]
    return out


def syr2k(uplo: str, trans: str, alpha, A: np.ndarray, B: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """BLAS xSYR2K semantics (Syr2k.cpp:20-40 -> blas::Syr2k; distributed
    Syr2k.cpp:78-93): alpha (op(A) op(B)^T + op(B) op(A)^T) + beta C on uplo."""
    tb = "T" if trans == "N" else "N"
    full = gemm(trans, tb, alpha, B, A, 1.0, gemm(trans, tb, alpha, A, B, beta, C))
    out = np.array(C, order="F", copy=True)
    mask = _tri_mask(C.shape[0], uplo)
    out[mask] = full[mask]
    return out


def trsm(side: str, uplo: str, trans: str, diag: str, alpha, A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """BLAS xTRSM semantics (the reference's CPU path: Trsm.cpp -> blas::Trsm;
    distributed Trsm.cpp:129-420): X = alpha op(A)^-1 B (side 'L') or
    alpha B op(A)^-1 ('R'); only A's uplo triangle is read, its diagonal only when
    diag == 'N'.  Column-oriented substitution in float64."""
    A = np.asarray(A, dtype=np.float64)
    X = alpha * np.array(B, dtype=np.float64)
    m = A.shape[0]
    i, j = np.indices((m, m))
    T = np.where((i >= j) if uplo == "L" else (i <= j), A, 0.0)  # the other triangle is never read
    if diag == "U":
        np.fill_diagonal(T, 1.0)
    op = T.T if trans != "N" else T
    if side == "R":  # X op(A) = B  <=>  op(A)^T X^T = B^T
        op, X = op.T, X.T
    lower = bool(np.allclose(op, np.tril(op)))
    order = range(m) if lower else range(m - 1, -1, -1)
    for i in order:
        X[i] /= op[i, i]
        rest = slice(i + 1, m) if lower else slice(0, i)
        X[rest] -= np.outer(op[rest, i], X[i])
    return X.T.copy() if side == "R" else X


def symm(side: str, uplo: str, alpha, A: np.ndarray, B: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """BLAS xSYMM semantics (Symm.cpp:55-80 -> blas::Symm): A symmetric with only
    its uplo triangle read; the full A is mirrored, then the GEMM loop nest."""
    m = A.shape[0]
    i, j = np.indices((m, m))
    keep = (i >= j) if uplo == "L" else (i <= j)
    T = np.where(keep, A, 0.0)
    S = np.where(keep, A, T.T).astype(A.dtype)
    return gemm("N", "N", alpha, S, B, beta, C) if side == "L" else gemm("N", "N", alpha, B, S, beta, C)


def cpu_gemm(ta: str, tb: str, alpha, A: np.ndarray, B: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """bench.py's CPU baseline: blocked OpenMP f64 GEMM (cpu_gemm.c), BLAS semantics."""
    C = np.array(C, order="F", copy=True, dtype=np.float64)
    A = np.asfortranarray(A, dtype=np.float64)
    B = np.asfortranarray(B, dtype=np.float64)
    m, n = C.shape
    k = A.shape[1] if ta == "N" else A.shape[0]
    lib().orc_cpu_gemm_f64(ta.encode(), tb.encode(), m, n, k, alpha, _p(A), max(A.shape[0], 1), _p(B),
                           max(B.shape[0], 1), beta, _p(C), max(m, 1))
    return C


def cpu_threads() -> int:
    return int(lib().orc_cpu_threads())


def mt_uniform(seed: int, count: int, lo: float, hi: float, kind: str = "f64") -> np.ndarray:
    """The reference's SampleUniform / SampleBall (include/El/core/random/impl.hpp:113-139,
    230-231): libstdc++ std::uniform_real_distribution over std::mt19937, restated
    with numpy's MT19937 (same init_genrand seeding, same 32-bit outputs) and
    libstdc++'s generate_canonical (two draws for double, one for float; a
    result of 1 becomes the largest value below 1).  kind: f64 | f32 | f16 | bf16
    (f16 draws in float and rounds to half, as cpu_half_type does)."""
    rs = np.random.RandomState(seed & 0xFFFFFFFF)
    if kind == "f64":
        u = rs.randint(0, 2 ** 32, size=2 * count, dtype=np.uint32).astype(np.float64)
        r = (u[0::2] + u[1::2] * 4294967296.0) / 18446744073709551616.0
        r = np.where(r >= 1.0, np.nextafter(1.0, 0.0), r)
        return r * (hi - lo) + lo
    u = rs.randint(0, 2 ** 32, size=count, dtype=np.uint32).astype(np.float32)
    r = u / np.float32(4294967296.0)
    r = np.where(r >= 1, np.nextafter(np.float32(1), np.float32(0)), r).astype(np.float32)
    a, b = np.float32(lo), np.float32(hi)
    x = (r * (b - a) + a).astype(np.float32)
    if kind == "f16":
        return x.astype(np.float16)
    if kind == "bf16":
        return f32_to_bf16_bits(x)
    return x


def gemm_half(ta: str, tb: str, alpha, A: np.ndarray, B: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """The reference's CPU half path: the naive loops of
    src/core/imports/blas/Gemm.hpp:47-260 with every operation rounded to half
    (half_float semantics), vectorised over i."""
    h = np.float16
    A = A.astype(h)
    B = B.astype(h)
    C = np.array(C, dtype=h, order="F", copy=True)
    m, n = C.shape
    k = A.shape[1] if ta == "N" else A.shape[0]
    al, be = h(alpha), h(beta)
    if be == h(0):
        C[:] = h(0)
    elif be != h(1):
        C *= be
    opB = (lambda l, j: B[l, j]) if tb == "N" else (lambda l, j: B[j, l])
    for j in range(n):
        if ta == "N":
            for l in range(k):
                gamma = h(al * opB(l, j))
                C[:, j] = (C[:, j] + (A[:, l] * gamma).astype(h)).astype(h)
        else:
            for i in range(m):
                g = h(0)
                for l in range(k):
                    g = h(g + h(A[l, i] * opB(l, j)))
                C[i, j] = h(C[i, j] + h(g * al))
    return C


def summa_nnc(r: int, c: int, nb: int, alpha, A: np.ndarray, B: np.ndarray, beta, C: np.ndarray) -> np.ndarray:
    """SUMMA_NNC_impl simulated over an r x c grid (oracle.c:orc_summa_nnc_f64)."""
    C = np.array(C, dtype=np.float64, order="F", copy=True)
    A = np.asfortranarray(A, dtype=np.float64)
    B = np.asfortranarray(B, dtype=np.float64)
    m, n = C.shape
    k = A.shape[1]
    lib().orc_summa_nnc_f64(r, c, m, n, k, nb, alpha, _p(A), max(m, 1), _p(B), max(k, 1), beta, _p(C), max(m, 1))
    return C


def parity_ratio(C: np.ndarray, Cref: np.ndarray, A: np.ndarray, B: np.ndarray, k: int, eps: float) -> float:
    """north_star metric ||C - Cref||_F / (||A||_F ||B||_F k eps)."""
    num = np.linalg.norm((np.asarray(C, np.float64) - np.asarray(Cref, np.float64)).ravel())
    den = np.linalg.norm(np.asarray(A, np.float64).ravel()) * np.linalg.norm(np.asarray(B, np.float64).ravel())
    den *= max(k, 1) * eps
    return float(num / den) if den > 0 else float(num)
