"""gfx950 kernel parity through the C-ABI (local GEMM, BLAS-1, hash fill)."""
import ctypes

import numpy as np
import pytest

import oracle
from elemental_amd import _lib as L
from elemental_amd import el

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dev(a: np.ndarray) -> "torch.Tensor":
    """Column-major host array -> device tensor holding the same bytes."""
    a = np.asfortranarray(a)
    flat = np.ravel(a, order="F")
    if flat.dtype == np.uint16:
        flat = flat.view(np.int16)
    return torch.from_numpy(flat.copy()).cuda()


def host(t, shape, dtype):
    torch.cuda.synchronize()
    a = t.cpu().numpy()
    if dtype == np.uint16:
        a = a.view(np.uint16)
    return np.asfortranarray(a.reshape(shape, order="F"))


def sync():
    L.call("elx_device_synchronize")
    torch.cuda.synchronize()


OPS = {"N": L.NORMAL, "T": L.TRANSPOSE}
SHAPES = [(1, 1, 1), (67, 53, 41), (128, 128, 16), (255, 257, 130), (300, 200, 517), (16, 700, 3),
          # few output tiles, long k: split-k chunks + ordered reduce (even and odd k)
          (96, 80, 9000), (67, 53, 4099)]
# >= 512 128x128 tiles: the fp64 LDS-DMA kernel (ragged edges, k tail of 4)
BIG = [(3000, 2900, 100)]


@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("ta", ["N", "T"])
@pytest.mark.parametrize("tb", ["N", "T"])
def test_local_gemm_f64_f32(dt, ta, tb):
    npdt = np.float64 if dt == "f64" else np.float32
    eps = np.finfo(npdt).eps
    fn = L.lib().elx_gemm_f64 if dt == "f64" else L.lib().elx_gemm_f32
    for (m, n, k) in SHAPES + BIG:
        for beta in (0.0, -0.5):
            A = oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, 11, 0, 1, npdt)
            B = oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, 12, 0, 1, npdt)
            C = oracle.hash_matrix(m, n, 13, 0, 1, npdt)
            if beta == 0.0:
                C[:] = np.nan  # beta == 0 must never read C
            ref = oracle.gemm(ta, tb, 0.5, A, B, beta, np.nan_to_num(C))
            dA, dB, dC = dev(A), dev(B), dev(C)
            torch.cuda.synchronize()
            L.check(fn(OPS[ta], OPS[tb], m, n, k, 0.5, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0],
                       beta, dC.data_ptr(), m, None))
            sync()
            got = host(dC, (m, n), npdt)
            assert np.isfinite(got).all()
            r = oracle.parity_ratio(got, ref, A, B, k, eps)
            assert r <= 10, f"{dt} {ta}{tb} {m}x{n}x{k} beta={beta}: ratio {r}"


@pytest.mark.parametrize("k", [300, 8192])
def test_local_gemm_known_answer_exact(k):
    """Integer-valued operands: every partial sum is exact in fp64, so the
    product must match bit for bit whatever the summation order (k = 8192
    takes the split-k path)."""
    rng = np.random.default_rng(0)
    m, n = 130, 70
    A = np.asfortranarray(rng.integers(-8, 8, (m, k)).astype(np.float64))
    B = np.asfortranarray(rng.integers(-8, 8, (k, n)).astype(np.float64))
    C = np.asfortranarray(rng.integers(-8, 8, (m, n)).astype(np.float64))
    dA, dB, dC = dev(A), dev(B), dev(C)
    torch.cuda.synchronize()
    L.call("elx_gemm_f64", 0, 0, m, n, k, 2.0, dA.data_ptr(), m, dB.data_ptr(), k, -1.0, dC.data_ptr(), m, None)
    sync()
    assert np.array_equal(host(dC, (m, n), np.float64), 2.0 * A @ B - C)


_SMALL_TILE_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from elemental_amd import _lib as L
dt = np.float64 if sys.argv[2] == "f64" else np.float32
OPS = {"N": 0, "T": 1}
bad = []
for (m, n, k) in [(2048, 2048, 2072), (2000, 1990, 1056), (64, 128, 48), (190, 130, 4104), (132, 68, 32),
                  (68, 132, 64)]:
    for ta in "NT":
        for tb in "NT":
            rng = np.random.default_rng(k + m)
            A = np.asfortranarray(rng.integers(-4, 4, (m, k) if ta == "N" else (k, m)).astype(dt))
            B = np.asfortranarray(rng.integers(-4, 4, (k, n) if tb == "N" else (n, k)).astype(dt))
            C = np.asfortranarray(rng.integers(-4, 4, (m, n)).astype(dt))
            dv = lambda X: torch.from_numpy(np.ascontiguousarray(X.T)).cuda()
            dA, dB, dC = dv(A), dv(B), dv(C)
            torch.cuda.synchronize()
            L.call("elx_gemm_" + sys.argv[2], OPS[ta], OPS[tb], m, n, k, 2.0, dA.data_ptr(), A.shape[0],
                   dB.data_ptr(), B.shape[0], -1.0, dC.data_ptr(), m, None)
            L.call("elx_device_synchronize")
            got = dC.cpu().numpy().T
            want = 2.0 * (A if ta == "N" else A.T) @ (B if tb == "N" else B.T) - C
            if not np.array_equal(got, want):
                bad.append((m, n, k, ta, tb))
print("BAD", bad if bad else "none")
"""


@pytest.mark.parametrize("dtype,knob", [("f64", "ELX_F64G_T64"), ("f32", "ELX_F32G_T64")])
def test_local_gemm_64x64_tiles_exact(dtype, knob):
    """The LDS-DMA kernels' 64 x 64 tiles forced on every shape (ELX_F64G_T64=2 /
    ELX_F32G_T64=2: RC images of 512-B (fp64) / 256-B (fp32) k-rows, several per
    DMA instruction, for A and B), every orientation, edges, split-k and the k
    tail: exact on small-integer operands (products and sums stay exact in fp32
    too), run in a child since the knob is read once."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _SMALL_TILE_SCRIPT, root, dtype], capture_output=True, text=True,
                       timeout=110, env=dict(os.environ, **{knob: "2"}))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert "BAD none" in p.stdout, p.stdout[-2000:]


@pytest.mark.parametrize("ta", ["N", "T"])
@pytest.mark.parametrize("tb", ["N", "T"])
@pytest.mark.parametrize("shape", [(2048, 2048, 2072), (2000, 1990, 1056), (1024, 1024, 288)])
def test_local_gemm_f64_one_workgroup_per_cu_exact(ta, tb, shape):
    """Grids of at most one workgroup per CU (the eight-wave 32 x 64 split of the
    fp64 LDS-DMA kernel) and the k % 16 tail through the general kernel
    (2072 = 2048 + 16 + 8): integer operands, so every orientation must match
    exactly."""
    m, n, k = shape
    rng = np.random.default_rng(k)
    A = np.asfortranarray(rng.integers(-4, 4, (m, k) if ta == "N" else (k, m)).astype(np.float64))
    B = np.asfortranarray(rng.integers(-4, 4, (k, n) if tb == "N" else (n, k)).astype(np.float64))
    C = np.asfortranarray(rng.integers(-4, 4, (m, n)).astype(np.float64))
    dA, dB, dC = dev(A), dev(B), dev(C)
    torch.cuda.synchronize()
    L.call("elx_gemm_f64", OPS[ta], OPS[tb], m, n, k, 2.0, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0],
           -1.0, dC.data_ptr(), m, None)
    sync()
    opA = A if ta == "N" else A.T
    opB = B if tb == "N" else B.T
    assert np.array_equal(host(dC, (m, n), np.float64), 2.0 * (opA @ opB) - C)


_F64_RING_CASES = [(r, sh, b) for r in ("1", "0") for sh, b in [
    ((4096, 4096, 640), -1.0), ((4000, 4040, 1056), 0.0), ((2048, 4096, 2072), -1.0), ((4096, 2048, 32), 0.5)]] + [
    ("2", (1536, 2048, 640), -1.0), ("2", (1000, 1016, 1056), 0.0), ("2", (1536, 2048, 2072), -1.0),
    ("2", (1024, 512, 16), 0.5), ("2", (512, 512, 2048), -1.0), ("2", (520, 600, 3000), 0.0)]


def _with_stages(cases):
    """Each ring case in both DMA forms; the slab kernels (ring "0") only in the
    buffer-descriptor form: they read their *_STAGE knob once per process, so a
    per-test setting could never reach them."""
    return [(r, sh, b, st) for r, sh, b in cases for st in ("buf", "global") if not (r == "0" and st == "global")]


@pytest.mark.parametrize("ta", ["N", "T"])
@pytest.mark.parametrize("tb", ["N", "T"])
@pytest.mark.parametrize("ring,shape,beta,stage", _with_stages(_F64_RING_CASES))
def test_local_gemm_f64_ring_exact(ta, tb, shape, beta, ring, stage, monkeypatch):
    """The fp64 ring kernel (gemm_f64r_kernel: four waves, a 5-slot LDS ring of
    32-deep K-tiles; ELX_F64G_RING=1) on 128-tile grids: many wraps of the ring
    (k = 640: 20 K-tiles), ragged edge tiles with beta = 0 (C holds NaN and must
    not be read), the k % 32 tail through the general kernel (2072 = 64 x 32 +
    24), and a single K-tile (k = 32: prologue and clamped restaging only).
    Integer operands: exact in every orientation.  ring = "0": the same cases
    through the two-stage slab kernel it replaced as the default; ring = "2":
    the 64 x 64 ring (16-deep K-tiles, four workgroups per CU) on grids of
    64-tiles, likewise with a ragged grid, a k tail (2072 = 129 x 16 + 8), a
    single K-tile, and grids of 64 / 90 tiles that split k into chunks
    (partials through splitk_reduce)."""
    monkeypatch.setenv("ELX_F64G_RING", ring)
    if stage == "global":  # the 64-bit-address DMA form (operands too long for 31-bit offsets)
        monkeypatch.setenv("ELX_F64G_STAGE", "g")
    m, n, k = shape
    rng = np.random.default_rng(m + k)
    A = np.asfortranarray(rng.integers(-4, 4, (m, k) if ta == "N" else (k, m)).astype(np.float64))
    B = np.asfortranarray(rng.integers(-4, 4, (k, n) if tb == "N" else (n, k)).astype(np.float64))
    C = np.asfortranarray(rng.integers(-4, 4, (m, n)).astype(np.float64))
    C0 = C.copy()
    if beta == 0.0:
        C0[:] = np.nan
    dA, dB, dC = dev(A), dev(B), dev(C0)
    torch.cuda.synchronize()
    L.call("elx_gemm_f64", OPS[ta], OPS[tb], m, n, k, 2.0, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0],
           beta, dC.data_ptr(), m, None)
    sync()
    opA = A if ta == "N" else A.T
    opB = B if tb == "N" else B.T
    want = 2.0 * (opA @ opB) + (beta * C if beta != 0.0 else 0.0)
    got = host(dC, (m, n), np.float64)
    assert np.array_equal(got, want), f"{int(np.count_nonzero(got != want))} mismatches"


@pytest.mark.parametrize("ta", ["N", "T"])
@pytest.mark.parametrize("tb", ["N", "T"])
@pytest.mark.parametrize("ring,shape,beta,stage", _with_stages([
    ("1", (2048, 2048, 640), -1.0), ("1", (4000, 4040, 1088), 0.0), ("1", (2048, 4096, 2072), -1.0),
    ("1", (4096, 2048, 64), 0.5),
    ("2", (1024, 1024, 2048), -1.0), ("2", (1000, 1016, 1152), 0.0), ("2", (1536, 2048, 2100), -1.0),
    ("2", (1024, 512, 128), 0.5),
    ("4", (1536, 2048, 640), -1.0), ("4", (1000, 1016, 1056), 0.0), ("4", (1536, 2048, 2100), -1.0),
    ("4", (1024, 512, 32), 0.5), ("4", (512, 512, 4096), -1.0), ("4", (520, 600, 3000), 0.0),
    ("0", (4000, 4040, 1088), 0.0), ("0", (1000, 1016, 1152), 0.0)]))
def test_local_gemm_f32_ring_exact(ta, tb, ring, shape, beta, stage, monkeypatch):
    """The fp32 ring kernel (gemm_f32r_kernel; ELX_F32G_RING bit 0: 128 x 128
    tiles with 64-deep K-tiles on grids of 128-tiles, bit 1: 64 x 64 tiles with
    128-deep K-tiles on grids of 64-tiles): many wraps of the 5-slot ring, ragged
    edge tiles with beta = 0 (C holds NaN and must not be read), the k tail
    through the general kernel (2072 = 32 x 64 + 24, 2100 = 16 x 128 + 52), a
    single K-tile (prologue and clamped restaging only), and the k-permuted
    MFMA steps in every orientation.  ring = "4": the 64 x 64 ring with 32-deep
    K-tiles and four workgroups per CU, likewise (2100 = 65 x 32 + 20), and on
    grids small enough to split k into chunks.  ring =
    "0": the slab kernels on the ragged cases.  Integer operands: exact."""
    monkeypatch.setenv("ELX_F32G_RING", ring)
    if stage == "global":  # the 64-bit-address DMA form (operands too long for 31-bit offsets)
        monkeypatch.setenv("ELX_F32G_STAGE", "g")
    m, n, k = shape
    rng = np.random.default_rng(m + k + 1)
    A = np.asfortranarray(rng.integers(-4, 4, (m, k) if ta == "N" else (k, m)).astype(np.float32))
    B = np.asfortranarray(rng.integers(-4, 4, (k, n) if tb == "N" else (n, k)).astype(np.float32))
    C = np.asfortranarray(rng.integers(-4, 4, (m, n)).astype(np.float32))
    C0 = C.copy()
    if beta == 0.0:
        C0[:] = np.nan
    dA, dB, dC = dev(A), dev(B), dev(C0)
    torch.cuda.synchronize()
    L.call("elx_gemm_f32", OPS[ta], OPS[tb], m, n, k, 2.0, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0],
           beta, dC.data_ptr(), m, None)
    sync()
    opA = (A if ta == "N" else A.T).astype(np.float64)
    opB = (B if tb == "N" else B.T).astype(np.float64)
    want = (2.0 * (opA @ opB) + (beta * C if beta != 0.0 else 0.0)).astype(np.float32)
    got = host(dC, (m, n), np.float32)
    assert np.array_equal(got, want), f"{int(np.count_nonzero(got != want))} mismatches"


@pytest.mark.parametrize("kind", ["f16", "bf16"])
@pytest.mark.parametrize("ta", ["N", "T"])
@pytest.mark.parametrize("tb", ["N", "T"])
@pytest.mark.parametrize("shape", [(131, 77, 95), (2000, 2056, 200), (2048, 2312, 520)])
def test_local_gemm_16bit(kind, ta, tb, shape):
    """(131, 77, 95): the 128x128 kernel; (2000, 2056, 200): the 256x256
    glds/transposed-read kernel with ragged edge tiles plus the k-tail pass;
    (2048, 2312, 520): 8 K-tiles through its pipeline."""
    m, n, k = shape
    if kind == "f16":
        A = oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, 21, 0, 1, np.float16)
        B = oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, 22, 0, 1, np.float16)
        C = oracle.hash_matrix(m, n, 23, 0, 1, np.float16)
        Af, Bf, Cf = A.astype(np.float64), B.astype(np.float64), C.astype(np.float64)
        fn, eps, hostdt = L.lib().elx_gemm_f16, 2.0 ** -11, np.float16
    else:
        A = oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, 21, 0, 1, "bf16")
        B = oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, 22, 0, 1, "bf16")
        C = oracle.hash_matrix(m, n, 23, 0, 1, "bf16")
        Af, Bf, Cf = (oracle.bf16_bits_to_f32(x).astype(np.float64) for x in (A, B, C))
        fn, eps, hostdt = L.lib().elx_gemm_bf16, 2.0 ** -8, np.uint16
    exact = oracle.gemm(ta, tb, 0.5, Af, Bf, -0.5, Cf)
    dA, dB, dC = dev(A), dev(B), dev(C)
    torch.cuda.synchronize()
    L.check(fn(OPS[ta], OPS[tb], m, n, k, 0.5, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0], -0.5,
               dC.data_ptr(), m, None))
    sync()
    got = host(dC, (m, n), hostdt)
    gotf = got.astype(np.float64) if kind == "f16" else oracle.bf16_bits_to_f32(got).astype(np.float64)
    r = oracle.parity_ratio(gotf, exact, Af, Bf, k, eps)
    assert r <= 10, f"{kind} {ta}{tb}: ratio {r}"
    if kind == "f16" and m * n * k < 2e6:  # (the half-path oracle is a Python loop nest)
        # never worse than the reference's own CPU half path (half accumulation)
        refh = oracle.gemm_half(ta, tb, 0.5, A, B, -0.5, C).astype(np.float64)
        assert np.linalg.norm(gotf - exact) <= np.linalg.norm(refh - exact) + 1e-3


@pytest.mark.parametrize("kind", ["f16", "bf16"])
@pytest.mark.parametrize("alpha,beta", [(0.5, 0.0), (-1.0, 0.25)])
def test_local_gemm_16bit_split_alpha_beta_exact(kind, alpha, beta):
    """The 16-bit split-k reduce applies alpha and beta (including beta = 0, where
    C is not read: it holds NaN here) once, after summing the f32 partials:
    integer operands keep every partial and the scaled sum exact, so the result
    is numpy's single rounding of the exact value, bit for bit."""
    m, n, k = 1024, 1024, 8192
    rng = np.random.default_rng(7)
    A = rng.integers(-2, 3, (m, k)).astype(np.float32)
    B = rng.integers(-2, 3, (k, n)).astype(np.float32)
    C = rng.integers(-64, 65, (m, n)).astype(np.float32)
    if beta == 0.0:
        C[:] = np.nan
    exact = alpha * (A.astype(np.float64) @ B.astype(np.float64)) + (beta * C.astype(np.float64) if beta else 0.0)
    if kind == "f16":
        enc = lambda x: np.asfortranarray(x.astype(np.float16))
        fn, want = L.lib().elx_gemm_f16, exact.astype(np.float16).view(np.uint16)
    else:
        enc = lambda x: np.asfortranarray(oracle.f32_to_bf16_bits(x))
        fn, want = L.lib().elx_gemm_bf16, oracle.f32_to_bf16_bits(exact.astype(np.float32))
    dA, dB, dC = dev(enc(A)), dev(enc(B)), dev(enc(C))
    torch.cuda.synchronize()
    L.check(fn(0, 0, m, n, k, alpha, dA.data_ptr(), m, dB.data_ptr(), k, beta, dC.data_ptr(), m, None))
    sync()
    got = host(dC, (m, n), np.uint16)
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"{kind} alpha={alpha} beta={beta}: {len(bad)} mismatches, first at {bad[:4].tolist()}"


@pytest.mark.parametrize("tile", ["", "64", "128", "160", "192", "224", "256", "g"])
@pytest.mark.parametrize("kind", ["f16", "bf16"])
@pytest.mark.parametrize("ta", ["N", "T"])
@pytest.mark.parametrize("tb", ["N", "T"])
@pytest.mark.parametrize("shape", [(2048, 2312, 2112), (4096, 2048, 640), (2304, 2048, 64), (1024, 1024, 8192),
                                   (1002, 1032, 4096), (2048, 2048, 2112), (1536, 2312, 704), (4096, 4096, 192),
                                   (3072, 3072, 192), (2560, 2560, 192), (3584, 3584, 128), (2048, 2312, 2088),
                                   (1536, 2312, 712)])
def test_local_gemm_16bit_exact(kind, ta, tb, shape, tile, monkeypatch):
    """Integer operands in [-2, 2]: every partial sum is exact in the f32
    accumulators, so alpha op(A) op(B) + beta C is exact before the one rounding
    to 16 bits, and the result must equal numpy's rounding of the exact value bit
    for bit.  k = 2112: 66 slabs of 32 (the 16-bit kernels' main loop over many
    wraps of their LDS ring); 2312 columns: ragged edge tiles; k = 64: a single
    K-tile (the ring's prologue and clamped restaging only).  Grids of at most
    64 tiles split k (f32 partials, one reduce that rounds once), e.g. with
    256-tiles (2048, 2048, 2112) 2 chunks, (1536, 2312, 704) 2 with ragged edge
    tiles, (1024, 1024, 8192) 16, (1002, 1032, 4096) 13 with m % 4 != 0 (the
    partials' scalar stores; TN / TT only, the others take the simple kernel).
    `tile`: the four-wave kernel's tile as the plan picks it (""), or forced to
    64 / 128 / 160 / 192 / 224 / 256 (ELX_H16_TILE), so every instantiation sees
    every shape (rows-contiguous images in 128-column blocks plus a 64- and / or
    a 32-column block: 192 = 128 + 64, 160 = 128 + 32, 224 = 128 + 64 + 32).
    (4096, 4096, 192) / (3072, 3072, 192) / (2560, 2560, 192) / (3584, 3584,
    128): 16 x 16 grids of 256- / 192- / 160- / 224-tiles (the 256-tiles' in the
    super-block tile order, tile_of_sb).  (2048, 2312, 2088) / (1536, 2312, 712):
    a k tail of 40 / 8 past the last whole K-tile, added inside the kernel
    before the one rounding.  tile = "g": the plan's
    tile with the DMA in its 64-bit-address form (ELX_H16_STAGE=g; operands too
    long for 31-bit buffer offsets take it)."""
    if tile == "g":
        monkeypatch.setenv("ELX_H16_STAGE", "g")
    elif tile:
        monkeypatch.setenv("ELX_H16_TILE", tile)
    m, n, k = shape
    rng = np.random.default_rng(m + n + k)
    A = rng.integers(-2, 3, (m, k) if ta == "N" else (k, m)).astype(np.float32)
    B = rng.integers(-2, 3, (k, n) if tb == "N" else (n, k)).astype(np.float32)
    C = rng.integers(-64, 65, (m, n)).astype(np.float32)
    opA = A if ta == "N" else A.T
    opB = B if tb == "N" else B.T
    exact = 1.0 * (opA.astype(np.float64) @ opB.astype(np.float64)) - 2.0 * C
    if kind == "f16":
        enc = lambda x: np.asfortranarray(x.astype(np.float16))
        fn, want = L.lib().elx_gemm_f16, exact.astype(np.float16).view(np.uint16)
    else:
        enc = lambda x: np.asfortranarray(oracle.f32_to_bf16_bits(x))
        fn, want = L.lib().elx_gemm_bf16, oracle.f32_to_bf16_bits(exact.astype(np.float32))
    dA, dB, dC = dev(enc(A)), dev(enc(B)), dev(enc(C))
    torch.cuda.synchronize()
    L.check(fn(OPS[ta], OPS[tb], m, n, k, 1.0, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0], -2.0,
               dC.data_ptr(), m, None))
    sync()
    got = host(dC, (m, n), np.uint16)
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"{kind} {ta}{tb}: {len(bad)} mismatches, first at {bad[:4].tolist()}"


@pytest.mark.parametrize("kind", ["f16", "bf16"])
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("k", [2088, 4104, 1091, 2047])
def test_local_gemm_16bit_ktail_rounding(kind, ta, tb, k):
    """k not a multiple of 64.  With both operands rows-contiguous (NT) the tail
    is always added inside the kernel, so C is rounded once: bit-exact.  With a
    k-contiguous operand that needs k % 8 == 0 (whole 16-B chunks); otherwise
    (1091, 2047) the tail is a second pass over the rounded C: bf16 within one
    ulp of the exact rounding (f16 holds these integers exactly).  2088 / 4104:
    tails of 40 / 8 with k % 8 == 0, in the kernel in every orientation."""
    m, n = 2048, 2312
    rng = np.random.default_rng(m + n + k)
    A = rng.integers(-2, 3, (m, k) if ta == "N" else (k, m)).astype(np.float32)
    B = rng.integers(-2, 3, (k, n) if tb == "N" else (n, k)).astype(np.float32)
    C = rng.integers(-64, 65, (m, n)).astype(np.float32)
    opA = A if ta == "N" else A.T
    opB = B if tb == "N" else B.T
    exact = 1.0 * (opA.astype(np.float64) @ opB.astype(np.float64)) - 2.0 * C
    if kind == "f16":
        enc = lambda x: np.asfortranarray(x.astype(np.float16))  # noqa: E731
        fn, want = L.lib().elx_gemm_f16, exact.astype(np.float16).view(np.uint16)
    else:
        enc = lambda x: np.asfortranarray(oracle.f32_to_bf16_bits(x))  # noqa: E731
        fn, want = L.lib().elx_gemm_bf16, oracle.f32_to_bf16_bits(exact.astype(np.float32))
    dA, dB, dC = dev(enc(A)), dev(enc(B)), dev(enc(C))
    torch.cuda.synchronize()
    L.check(fn(OPS[ta], OPS[tb], m, n, k, 1.0, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0], -2.0,
               dC.data_ptr(), m, None))
    sync()
    got = host(dC, (m, n), np.uint16)
    in_kernel = (ta == "N" and tb == "T") or k % 8 == 0
    if in_kernel or kind == "f16":
        bad = np.argwhere(got != want)
        assert bad.size == 0, f"{kind} {ta}{tb} k={k}: {len(bad)} mismatches, first at {bad[:4].tolist()}"
    else:  # two roundings: at most one bf16 ulp from the exact rounding (same sign, adjacent codes)
        d = np.abs(got.astype(np.int32) - want.astype(np.int32))
        assert d.max() <= 1, (kind, ta, tb, k, int(d.max()))


@pytest.mark.parametrize("tail", ["1", "0"])
@pytest.mark.parametrize("kind", ["f16", "bf16"])
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("shape,tile", [((4096, 4352, 1024), "256"), ((3072, 3072, 1024), "128"),
                                        ((3072, 2816, 1024), "128"), ((7168, 1280, 1088), "256"),
                                        ((4608, 4608, 1024), "256"), ((4608, 4608, 1064), "256")])
def test_local_gemm_16bit_tail_split_exact(kind, ta, tb, shape, tile, tail, monkeypatch):
    """The four-wave kernel's data-parallel rounds + tail (gemm_mfma_h): the
    last, partly filled round of tiles is a rectangle of C (the last group's
    last columns) computed as its own GEMM, the full rounds by one launch over
    the first tiles of the order.  (6144, 4096): 384 256-tiles, the whole last
    group (8 x 16) the tail; (3072, 3072) in 128-tiles: 576 = 512 + 64, an
    8 x 8 tail; (3072, 2816): 24 x 22 = 528, 16 tiles rounded up to two group
    columns; (7168, 1280, 1088): 28 x 5 = 140 256-tiles in one round (no tail),
    the control; (4608, 4608): 324 = 256 + 68 256-tiles, a tail between a
    quarter and a third of a round, run as split-k over the same tiles (the
    group height shrinks to 6 so the last group holds it; z = 3 chunks of k,
    and with k = 1064 the last chunk also takes the 40-deep k tail; TN keeps
    the smaller-tile form: no split-k tail there).  Exact integer products, tail
    on and off (ELX_H16_TAIL), bit for bit the same."""
    monkeypatch.setenv("ELX_H16_TILE", tile)
    monkeypatch.setenv("ELX_H16_TAIL", tail)
    m, n, k = shape
    rng = np.random.default_rng(m + n + k + 7)
    A = rng.integers(-2, 3, (m, k) if ta == "N" else (k, m)).astype(np.float32)
    B = rng.integers(-2, 3, (k, n) if tb == "N" else (n, k)).astype(np.float32)
    C = rng.integers(-64, 65, (m, n)).astype(np.float32)
    opA = A if ta == "N" else A.T
    opB = B if tb == "N" else B.T
    exact = 1.0 * (opA.astype(np.float64) @ opB.astype(np.float64)) - 2.0 * C
    if kind == "f16":
        enc = lambda x: np.asfortranarray(x.astype(np.float16))  # noqa: E731
        fn, want = L.lib().elx_gemm_f16, exact.astype(np.float16).view(np.uint16)
    else:
        enc = lambda x: np.asfortranarray(oracle.f32_to_bf16_bits(x))  # noqa: E731
        fn, want = L.lib().elx_gemm_bf16, oracle.f32_to_bf16_bits(exact.astype(np.float32))
    dA, dB, dC = dev(enc(A)), dev(enc(B)), dev(enc(C))
    torch.cuda.synchronize()
    L.check(fn(OPS[ta], OPS[tb], m, n, k, 1.0, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0], -2.0,
               dC.data_ptr(), m, None))
    sync()
    got = host(dC, (m, n), np.uint16)
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"{kind} {ta}{tb}: {len(bad)} mismatches, first at {bad[:4].tolist()}"


@pytest.mark.parametrize("dt", ["f64", "f32", "bf16", "f16"])
@pytest.mark.parametrize("ta,tb", [("N", "N"), ("T", "N"), ("N", "T")])
def test_local_gemm_matches_vendor_blas(dt, ta, tb):
    """The same column-major product through the vendor GPU BLAS (torch.matmul ->
    hipBLASLt, the library family of the reference's rocblas_{d,s,h}gemm calls,
    src/hydrogen/device/rocBLAS_API.cpp:151-170): both within the north_star
    bound of the exact product and of each other.  For bf16 this is the only
    anchor besides the exact-integer test (the reference's CPU path has no bf16)."""
    m, n, k = 2304, 2056, 1088  # the large-tile kernels, ragged in n
    tdt = {"f64": torch.float64, "f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[dt]
    eps = {"f64": 2.0 ** -53, "f32": 2.0 ** -24, "bf16": 2.0 ** -8, "f16": 2.0 ** -11}[dt]
    g = torch.Generator(device="cuda").manual_seed(7)
    Ash = (m, k) if ta == "N" else (k, m)
    Bsh = (k, n) if tb == "N" else (n, k)
    # column-major storage = the transpose of a row-major torch tensor
    At = (torch.rand(Ash[1], Ash[0], device="cuda", generator=g, dtype=torch.float64) - 0.5).to(tdt)
    Bt = (torch.rand(Bsh[1], Bsh[0], device="cuda", generator=g, dtype=torch.float64) - 0.5).to(tdt)
    C = torch.zeros(n, m, device="cuda", dtype=tdt)  # C^T row-major = C column-major
    fn = {"f64": L.lib().elx_gemm_f64, "f32": L.lib().elx_gemm_f32, "bf16": L.lib().elx_gemm_bf16,
          "f16": L.lib().elx_gemm_f16}[dt]
    torch.cuda.synchronize()
    L.check(fn(OPS[ta], OPS[tb], m, n, k, 1.0, At.data_ptr(), Ash[0], Bt.data_ptr(), Bsh[0], 0.0, C.data_ptr(), m,
               None))
    sync()
    opA = At.t() if ta == "N" else At   # op(A), m x k
    opB = Bt.t() if tb == "N" else Bt   # op(B), k x n
    vend = torch.matmul(opA, opB)
    exact = opA.double() @ opB.double()
    ours = C.t().double()
    Ah, Bh = opA.double().cpu().numpy(), opB.double().cpu().numpy()
    r_ours = oracle.parity_ratio(ours.cpu().numpy(), exact.cpu().numpy(), Ah, Bh, k, eps)
    r_vend = oracle.parity_ratio(vend.double().cpu().numpy(), exact.cpu().numpy(), Ah, Bh, k, eps)
    r_pair = oracle.parity_ratio(ours.cpu().numpy(), vend.double().cpu().numpy(), Ah, Bh, k, eps)
    assert r_ours <= 10 and r_pair <= 10, f"{dt} {ta}{tb}: ours {r_ours:.3g} vendor {r_vend:.3g} pair {r_pair:.3g}"


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k,beta", [(2994, 2900, 32837, 0.0), (1000, 1030, 524325, -2.0)])
def test_local_gemm_f32_tn_long_k_exact(m, n, k, beta):
    """f32 TN with a long k per tile takes the 64 x 64 wave tiles (C4's shape,
    gemm_f32g.hip launch_fb): the first case as one launch over 552 tiles, the
    second split-k into 16 chunks of 32768 plus the k tail, with beta != 0.
    Integer operands in [-2, 2] keep every partial sum below 2^24, so the f32
    result is exact and must equal the f64 product bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(11)
    At = torch.randint(-2, 3, (m, k), device="cuda", generator=g).float()  # column-major k x m = op(A)^T
    Bt = torch.randint(-2, 3, (n, k), device="cuda", generator=g).float()  # column-major k x n
    C0 = torch.randint(-3, 4, (n, m), device="cuda", generator=g).float()  # C^T row-major = C column-major
    C = C0.clone()
    torch.cuda.synchronize()
    L.check(L.lib().elx_gemm_f32(OPS["T"], OPS["N"], m, n, k, 1.0, At.data_ptr(), k, Bt.data_ptr(), k, beta, C.data_ptr(), m,
                                 None))
    sync()
    want = (Bt.double() @ At.double().t() + beta * C0.double()).float()  # (A^T B)^T = B^T A, n x m
    assert torch.equal(C, want), f"max err {(C - want).abs().max().item()}"


def test_local_gemm_16bit_group_knob_clamped(monkeypatch):
    """ELX_H16_GROUP (the tile-order group height, read per call) of 0 or garbage
    must not reach the kernel's tile mapping, which divides by it: a zero height
    once sent workgroups to tiles far outside the operands (an illegal-address
    fault).  The library clamps it to >= 1; the product is unchanged."""
    m, n, k = 2048, 2048, 256  # 64 tiles of 256 x 256: the large-tile kernels
    rng = np.random.default_rng(5)
    A = rng.integers(-2, 3, (m, k)).astype(np.float32)
    B = rng.integers(-2, 3, (k, n)).astype(np.float32)
    want = oracle.f32_to_bf16_bits((A.astype(np.float64) @ B).astype(np.float32))
    for g in ("0", "", "-3", "1"):
        monkeypatch.setenv("ELX_H16_GROUP", g)
        dA, dB = dev(np.asfortranarray(oracle.f32_to_bf16_bits(A))), dev(np.asfortranarray(oracle.f32_to_bf16_bits(B)))
        dC = dev(np.zeros((m, n), np.uint16))
        torch.cuda.synchronize()
        L.check(L.lib().elx_gemm_bf16(0, 0, m, n, k, 1.0, dA.data_ptr(), m, dB.data_ptr(), k, 0.0, dC.data_ptr(), m,
                                      None))
        sync()
        assert np.array_equal(host(dC, (m, n), np.uint16), want), g


DTYPES = [(L.F64, np.float64), (L.F32, np.float32), (L.F16, np.float16), (L.BF16, "bf16")]


def _mat(m, n, seed, npdt):
    return oracle.hash_matrix(m, n, seed, 0.0, 2.0, npdt)


def _as_f64(x, npdt):
    return oracle.bf16_bits_to_f32(x).astype(np.float64) if npdt == "bf16" else x.astype(np.float64)


def _round(x, npdt):
    if npdt == "bf16":
        return oracle.f32_to_bf16_bits(x.astype(np.float32))
    return x.astype(npdt)


def test_local_gemm_matches_mkl():
    """elx_gemm_{f64,f32} (the MFMA kernels LocalGemm runs) against one MKL
    dgemm_/sgemm_ call each (tests/golden/mkl_local.npz: the reference CPU
    path's own BLAS at Gemm_impl<CPU>'s call site), all orientations, odd shapes."""
    import os
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mkl_local.npz"))
    keys = [k for k in d.files if k != "_mkl" and not k.endswith("_seed")]
    assert len(keys) == 32
    for key in keys:
        tag, orient, shape = key.split("_")
        dt = np.float64 if tag == "f64" else np.float32
        ta, tb = orient[0], orient[1]
        m, n, k = map(int, shape.split("x"))
        s = [int(x) for x in d[key + "_seed"]]
        A = oracle.hash_matrix(m if ta == "N" else k, k if ta == "N" else m, s[0], 0.0, 0.1, dt)
        B = oracle.hash_matrix(k if tb == "N" else n, n if tb == "N" else k, s[1], 0.0, 0.1, dt)
        C = oracle.hash_matrix(m, n, s[2], 0.0, 0.1, dt)
        dA, dB, dC = dev(A), dev(B), dev(C)
        torch.cuda.synchronize()
        fn = "elx_gemm_f64" if tag == "f64" else "elx_gemm_f32"
        L.call(fn, OPS[ta], OPS[tb], m, n, k, 0.5, dA.data_ptr(), A.shape[0], dB.data_ptr(), B.shape[0], -0.5,
               dC.data_ptr(), m, None)
        sync()
        got = host(dC, (m, n), dt)
        r = oracle.parity_ratio(got, d[key], A, B, k, np.finfo(dt).eps)
        assert r <= 10, (key, r)


@pytest.mark.parametrize("t,npdt", DTYPES)
@pytest.mark.parametrize("m,n,lda,ldb", [(200, 136, 208, 144), (64, 64, 64, 64), (512, 8, 520, 16), (256, 384, 264, 392)])
def test_transpose_vectorized(t, npdt, m, n, lda, ldb):
    """Transposing moves whose unit-stride runs are 16-B aligned on both sides
    (transpose_vec_kernel: N x N register blocks, 8N x 8N wave tiles): whole and
    ragged wave tiles, ld > height on both sides; copy (Transpose_GPU_impl) and
    the transposed Axpy form (Axpy.cu:119-189), bit-exact."""
    hostdt = np.uint16 if npdt == "bf16" else npdt
    X = _mat(lda, n, 41, npdt)        # m x n view with ld = lda
    B0 = _mat(ldb, m, 42, npdt)       # n x m view with ld = ldb
    dX, dB = dev(X), dev(B0)
    torch.cuda.synchronize()
    L.call("elx_transpose", t, m, n, dX.data_ptr(), lda, dB.data_ptr(), ldb, None)
    sync()
    got = host(dB, (ldb, m), hostdt)
    want = B0.copy()
    want[:n, :] = X[:m, :].T
    assert np.array_equal(got, want)
    # W (n x m, ld ldb) += -2 X^T
    W = _mat(ldb, m, 43, npdt)
    dW = dev(W)
    torch.cuda.synchronize()
    L.call("elx_axpy2d", t, n, m, -2.0, dX.data_ptr(), lda, 1, dW.data_ptr(), 1, ldb, None)
    sync()
    cdt = np.float64 if t == L.F64 else np.float32
    Wf, Xf = _as_f64(W, npdt), _as_f64(X, npdt)
    wantW = W.copy()
    wantW[:n, :] = _round(Wf[:n, :].astype(cdt) + cdt(-2.0) * Xf[:m, :].T.astype(cdt), npdt)
    assert np.array_equal(host(dW, (ldb, m), hostdt), wantW)


@pytest.mark.parametrize("t,npdt", DTYPES)
def test_blas1_kernels(t, npdt):
    hostdt = np.uint16 if npdt == "bf16" else npdt
    m, n = 77, 45
    X = _mat(m, n, 31, npdt)
    Y = _mat(m, n, 32, npdt)
    Xf, Yf = _as_f64(X, npdt), _as_f64(Y, npdt)
    # copy2d with a transposing stride pattern: B (n x m) = X^T
    dX, dB = dev(X), dev(np.zeros((n, m), dtype=hostdt))
    torch.cuda.synchronize()
    L.call("elx_transpose", t, m, n, dX.data_ptr(), m, dB.data_ptr(), n, None)
    sync()
    assert np.array_equal(host(dB, (n, m), hostdt), np.asfortranarray(X.T))
    # strided copy: every other row/column
    dC = dev(np.zeros(((m + 1) // 2, (n + 1) // 2), dtype=hostdt))
    torch.cuda.synchronize()
    L.call("elx_copy2d", t, (m + 1) // 2, (n + 1) // 2, dX.data_ptr(), 2, 2 * m, dC.data_ptr(), 1, (m + 1) // 2, None)
    sync()
    assert np.array_equal(host(dC, ((m + 1) // 2, (n + 1) // 2), hostdt), np.asfortranarray(X[::2, ::2]))
    # axpy2d Y += 0.5 X and the transposed form
    dY = dev(Y)
    torch.cuda.synchronize()
    L.call("elx_axpy2d", t, m, n, 0.5, dX.data_ptr(), 1, m, dY.data_ptr(), 1, m, None)
    sync()
    got = _as_f64(host(dY, (m, n), hostdt), npdt)
    want = _as_f64(_round((Yf + 0.5 * Xf) if t in (L.F64,) else (Yf.astype(np.float32) + np.float32(0.5) * Xf.astype(np.float32)), npdt), npdt)
    assert np.array_equal(got, want)
    # transposed form (Axpy_GPU_impl with X's strides swapped, Axpy.cu:119-189):
    # W (n x m) += -2 X^T (a power-of-two alpha: the product is exact, so a fused
    # multiply-add and the numpy restatement round identically)
    W = _mat(n, m, 33, npdt)
    Wf = _as_f64(W, npdt)
    dW = dev(W)
    torch.cuda.synchronize()
    L.call("elx_axpy2d", t, n, m, -2.0, dX.data_ptr(), m, 1, dW.data_ptr(), 1, n, None)
    sync()
    cdt = np.float64 if t == L.F64 else np.float32
    wantT = _as_f64(_round(Wf.astype(cdt) + cdt(-2.0) * Xf.T.astype(cdt), npdt), npdt)
    assert np.array_equal(_as_f64(host(dW, (n, m), hostdt), npdt), wantT)
    # scale, fill, hadamard, entrywise map
    dS = dev(X)
    torch.cuda.synchronize()
    L.call("elx_scale2d", t, m, n, -2.0, dS.data_ptr(), m, None)
    sync()
    assert np.array_equal(_as_f64(host(dS, (m, n), hostdt), npdt), -2.0 * Xf)
    L.call("elx_fill2d", t, m, n, 0.25, dS.data_ptr(), m, None)
    sync()
    assert (_as_f64(host(dS, (m, n), hostdt), npdt) == 0.25).all()
    dZ = dev(np.zeros((m, n), dtype=hostdt))
    dY = dev(Y)
    torch.cuda.synchronize()
    L.call("elx_hadamard2d", t, m, n, dX.data_ptr(), m, dY.data_ptr(), m, dZ.data_ptr(), m, None)
    sync()
    prod = (Xf * Yf) if t == L.F64 else (Xf.astype(np.float32) * Yf.astype(np.float32))
    assert np.array_equal(_as_f64(host(dZ, (m, n), hostdt), npdt), _as_f64(_round(prod, npdt), npdt))
    # in-place forms (Hadamard.cu:64-116): C aliasing A, and C aliasing both
    dA2 = dev(X)
    torch.cuda.synchronize()
    L.call("elx_hadamard2d", t, m, n, dA2.data_ptr(), m, dY.data_ptr(), m, dA2.data_ptr(), m, None)
    sync()
    assert np.array_equal(_as_f64(host(dA2, (m, n), hostdt), npdt), _as_f64(_round(prod, npdt), npdt))
    dA3 = dev(X)
    torch.cuda.synchronize()
    L.call("elx_hadamard2d", t, m, n, dA3.data_ptr(), m, dA3.data_ptr(), m, dA3.data_ptr(), m, None)
    sync()
    sq = (Xf * Xf) if t == L.F64 else (Xf.astype(np.float32) * Xf.astype(np.float32))
    assert np.array_equal(_as_f64(host(dA3, (m, n), hostdt), npdt), _as_f64(_round(sq, npdt), npdt))
    L.call("elx_entrywise_map", t, L.MAP_ABS, m, n, dX.data_ptr(), m, dZ.data_ptr(), m, None)
    sync()
    assert np.array_equal(_as_f64(host(dZ, (m, n), hostdt), npdt), np.abs(Xf))
    # combine: B := f(A, B) (CombineImpl.hpp), every functor, in the compute type
    cdt = np.float64 if t == L.F64 else np.float32
    a, b = Xf.astype(cdt), Yf.astype(cdt)
    funcs = {L.COMBINE_ADD: a + b, L.COMBINE_SUB: b - a, L.COMBINE_MUL: a * b, L.COMBINE_DIV: b / a,
             L.COMBINE_MAX: np.maximum(a, b), L.COMBINE_MIN: np.minimum(a, b),
             L.COMBINE_RELU_GRAD: np.where(a > 0, b, 0).astype(cdt)}
    for fn, ref in funcs.items():
        dB = dev(Y)
        torch.cuda.synchronize()
        L.call("elx_combine", t, fn, m, n, dX.data_ptr(), m, dB.data_ptr(), m, None)
        sync()
        got, want = _as_f64(host(dB, (m, n), hostdt), npdt), _as_f64(_round(ref, npdt), npdt)
        if fn == L.COMBINE_DIV:
            assert np.allclose(got, want, rtol=4 * np.finfo(cdt).eps if npdt in (np.float64, np.float32) else 1e-2)
        else:
            assert np.array_equal(got, want), fn


@pytest.mark.parametrize("t,npdt", DTYPES)
def test_fill_hash_bit_exact(t, npdt):
    hostdt = np.uint16 if npdt == "bf16" else npdt
    m, n = 300, 129
    d = dev(np.zeros((m, n), dtype=hostdt))
    torch.cuda.synchronize()
    L.call("elx_fill_hash", t, m, n, d.data_ptr(), m, 0, 1, 0, 1, 77, -0.1, 0.1, None)
    sync()
    want = oracle.hash_matrix(m, n, 77, -0.1, 0.1, npdt)
    got = host(d, (m, n), hostdt)
    assert got.tobytes(order="F") == np.asarray(want, dtype=hostdt).tobytes(order="F")


def test_pool_alloc_free():
    """The caching allocator that replaces hipCUB's CachingDeviceAllocator
    (src/core/imports/cub.cpp; contract in csrc/runtime/runtime.hpp):
    stream-ordered alloc/free, blocks freed on one stream and reallocated on
    another, in-use back to zero, and the steady-state rule: after one warm-up
    pass a repeated pattern reserves nothing new, whichever streams it uses.
    Reserved bytes are the allocator's own bin accounting (live + cached), so
    the check does not depend on the driver's pool."""
    el.device_synchronize()
    _, u0 = el.pool_stats()
    s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
    L.call("elx_stream_create", ctypes.byref(s1))
    L.call("elx_stream_create", ctypes.byref(s2))
    sizes = [1 << 20, 3 << 20, 64 << 20, 5000]
    try:
        def round_trip(alloc_stream, free_stream):
            ptrs = []
            for b in sizes:
                p = ctypes.c_void_p()
                L.call("elx_pool_alloc", ctypes.byref(p), b, alloc_stream)
                assert p.value and p.value % 256 == 0
                ptrs.append(p)
            _, u = el.pool_stats()
            assert u - u0 == sum(sizes)
            # the blocks are distinct and writable
            for p, b in zip(ptrs, sizes):
                L.call("elx_fill2d", L.F32, b // 4, 1, 1.0, p, max(b // 4, 1), alloc_stream)
            for p in ptrs:
                L.call("elx_pool_free", p, free_stream)
            _, u = el.pool_stats()
            assert u == u0

        round_trip(s1, s1)
        r1, _ = el.pool_stats()
        for _ in range(4):  # freed on one stream, reallocated on the other: served from the cache
            round_trip(s2, s1)
            round_trip(s1, s2)
            round_trip(None, s2)
        r2, _ = el.pool_stats()
        assert r2 == r1, (r1, r2)
        L.call("elx_stream_synchronize", s1)
        L.call("elx_stream_synchronize", s2)
        L.call("elx_pool_trim", 0)
        r3, u3 = el.pool_stats()
        assert r3 <= r2 and r3 - u3 <= r2 - u0
        with pytest.raises(L.LogicError, match="not from this pool"):
            L.call("elx_pool_free", ctypes.c_void_p(0x1000), None)
    finally:
        el.device_synchronize()
        L.call("elx_stream_destroy", s1)
        L.call("elx_stream_destroy", s2)


def test_pool_bins_and_cap():
    """Bins (powers of two to 1 MiB, then 8 per octave) and the
    H_CUB_MAX_CACHED_SIZE cap (cub.cpp:37-43): a free past the cap returns the
    block to the driver instead of caching it (CUB's cudaFree), so
    reserved - in_use never exceeds the cap, and the bytes held from the driver
    are exactly the live and cached blocks."""
    lib = L.lib()
    assert lib.elx_pool_bin_bytes(1) == 512
    assert lib.elx_pool_bin_bytes(5000) == 8192
    assert lib.elx_pool_bin_bytes(1 << 20) == 1 << 20
    assert lib.elx_pool_bin_bytes((1 << 20) + 1) == (1 << 20) + (128 << 10)
    assert lib.elx_pool_bin_bytes(3 << 20) == 3 << 20
    for b in [(1 << 20) + 1, 5 << 20, (1 << 30) + 1, 5 << 30, (1 << 33) + 12345, 32 << 30]:
        bb = lib.elx_pool_bin_bytes(b)
        assert b <= bb <= b * 1.125
    el.device_synchronize()
    old = ctypes.c_size_t()
    L.call("elx_pool_max_cached", ctypes.byref(old))
    try:
        cap = 8 << 20
        L.call("elx_pool_set_max_cached", cap)
        r, u = el.pool_stats()
        assert r - u <= cap
        base = el.pool_backing_reserved()
        ptrs = []
        for _ in range(6):
            p = ctypes.c_void_p()
            L.call("elx_pool_alloc", ctypes.byref(p), 3 << 20, None)
            ptrs.append(p)
        held = el.pool_backing_reserved()
        assert held >= base + 6 * (3 << 20) - cap, (base, held)
        for p in ptrs:
            L.call("elx_pool_free", p, None)
        r, u = el.pool_stats()
        assert r - u <= cap, (r, u)
        # what left the cache left the process
        assert el.pool_backing_reserved() == r, (el.pool_backing_reserved(), r, u)
    finally:
        L.call("elx_pool_set_max_cached", old.value)
        el.device_synchronize()


def _pool_worker(case, **env):
    import os
    import subprocess
    import sys
    e = dict(os.environ)
    e.update(env)
    here = os.path.dirname(os.path.abspath(__file__))
    return subprocess.run([sys.executable, os.path.join(here, "_pool_workers.py"), case], env=e,
                          capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("cache", ["1", "0"])
def test_pool_delayed_reader_regression(cache):
    """Round 4's wrong GEMMs, as one deterministic regression test: a reader
    delayed ~0.2 s by a spin kernel on its own stream, the block freed behind it
    (pool level; a DistMatrix view on another stream dropped before its owner;
    a matrix moved to another stream), and the same bin requested and
    overwritten at once on another stream.  With and without the cache
    (ELX_POOL_CACHE=0: every free returns its block to the driver, the setting
    under which the round-4 failures survived).  Before round 5 the view case
    failed deterministically (every entry overwritten)."""
    cases = ["pool_free_after_delayed_reader", "view_on_other_stream", "set_stream_owned"]
    for c in cases:
        r = _pool_worker(c, ELX_POOL_CACHE=cache)
        assert r.returncode == 0 and f"OK {c}" in r.stdout, (c, r.stdout[-2000:], r.stderr[-4000:])


def test_pool_release_path_off_the_host():
    """The over-cap release path (H_CUB_MAX_CACHED_SIZE=0, cub.cpp:37-43): a
    free behind a 0.2 s spin returns to the host in < 10 ms, a second thread's
    Alloc completes while the spin runs, and the memory is back with the driver
    once the device is idle (runtime.hpp's contract)."""
    r = _pool_worker("release_off_the_lock", H_CUB_MAX_CACHED_SIZE="0")
    assert r.returncode == 0 and "OK release_off_the_lock" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    print(r.stdout.strip().splitlines()[0])


def test_pool_debug_trace_lists_cross_stream_reuse():
    """H_CUB_DEBUG=1 (cub.cpp:45-50): the trace names each allocation, cache
    return and reuse with its streams and event; a block freed on one stream
    while its work still runs and requested on another is reported as a
    cross-stream reuse that makes the new stream wait on the free's event."""
    r = _pool_worker("debug_trace_cross_stream", H_CUB_DEBUG="1")
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [x for x in r.stderr.splitlines() if x.startswith("elx_pool[")]
    assert any("allocated new block" in x for x in lines), lines
    assert any("to the cache" in x for x in lines), lines
    reuse = [x for x in lines if "reused cached block" in x]
    assert reuse and "cross-stream reuse, the new stream waits on the event" in reuse[-1], lines


@pytest.mark.parametrize("s", [L.F64, L.F32, L.F16, L.BF16])
@pytest.mark.parametrize("t", [L.F64, L.F32, L.F16, L.BF16])
def test_copy2d_convert(s, t):
    """elx_copy2d_convert (Copy_GPU_impl<SrcT,DestT>): direct, strided and
    transposing moves, bit-exact vs the oracle's single-rounding restatement."""
    import _dist_workers as W
    fs, ft = W.FMT[s], W.FMT[t]
    hs = np.uint16 if fs == "bf16" else {"f64": np.float64, "f32": np.float32, "f16": np.float16}[fs]
    ht = np.uint16 if ft == "bf16" else {"f64": np.float64, "f32": np.float32, "f16": np.float16}[ft]
    m, n = 131, 70
    X = oracle.convert(W.convert_values(m, n, 3), "f64", fs)
    dX = dev(X)
    want = oracle.convert(X, fs, ft)
    dY = dev(np.zeros((m, n), dtype=ht))
    L.call("elx_copy2d_convert", s, t, m, n, dX.data_ptr(), 1, m, dY.data_ptr(), 1, m, None)
    sync()
    same = lambda a, b: np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))
    assert same(host(dY, (m, n), ht), want)
    # transposing: Y (n x m) = convert(X^T)
    dT = dev(np.zeros((n, m), dtype=ht))
    L.call("elx_copy2d_convert", s, t, n, m, dX.data_ptr(), m, 1, dT.data_ptr(), 1, n, None)
    sync()
    assert same(host(dT, (n, m), ht), want.T)
    # strided: every other row and column
    mh, nh = (m + 1) // 2, (n + 1) // 2
    dS = dev(np.zeros((mh, nh), dtype=ht))
    L.call("elx_copy2d_convert", s, t, mh, nh, dX.data_ptr(), 2, 2 * m, dS.data_ptr(), 1, mh, None)
    sync()
    assert same(host(dS, (mh, nh), ht), want[::2, ::2])


@pytest.mark.parametrize("h,w,ca,cs,ra,rs", [(1000, 37, 3, 4, 1, 2), (129, 65, 0, 2, 0, 4), (7, 300, 1, 8, 0, 1)])
def test_gpu_pack_unpack_strided(h, w, ca, cs, ra, rs):
    """elx_pack_strided / elx_unpack_strided / elx_unpack_axpy_strided on device
    buffers (one batched launch each) against the numpy restatement of
    StridedPack / StridedUnpack (Copy/util.hpp:667-718)."""
    import torch
    import test_pack_cpu as P
    ld = h + 5
    A = P.padded(h, w, ld, 4)
    ps = -(-h // cs) * -(-w // rs) + 3
    want = np.full(cs * rs * ps, np.nan)
    for l in range(rs):
        rsh = P.shift(l, ra, rs)
        for k in range(cs):
            csh = P.shift(k, ca, cs)
            sub = A[csh:h:cs, rsh:w:rs]
            q = (k + l * cs) * ps
            want[q:q + sub.size] = sub.ravel(order="F")
    Ad = torch.from_numpy(np.ascontiguousarray(A.T)).cuda()  # column-major ld x w
    Pd = torch.full((cs * rs * ps,), float("nan"), dtype=torch.float64, device="cuda")
    Bd = torch.full_like(Ad, -7.0)
    torch.cuda.synchronize()
    L.call("elx_pack_strided", 1, el.F64, h, w, ca, cs, ra, rs, Ad.data_ptr(), ld, Pd.data_ptr(), ps, None)
    L.call("elx_unpack_strided", 1, el.F64, h, w, ca, cs, ra, rs, Pd.data_ptr(), ps, Bd.data_ptr(), ld, None)
    L.call("elx_device_synchronize")
    assert np.array_equal(Pd.cpu().numpy(), want, equal_nan=True)
    B = Bd.cpu().numpy().T
    assert np.array_equal(B[:h, :w], A[:h, :w]) and np.all(B[h:, :] == -7.0)
    L.call("elx_unpack_axpy_strided", 1, el.F64, h, w, -2.0, ca, cs, ra, rs, Pd.data_ptr(), ps, Bd.data_ptr(), ld,
           None)
    L.call("elx_device_synchronize")
    assert np.array_equal(Bd.cpu().numpy().T[:h, :w], -A[:h, :w])
