"""Multi-rank workers for the CPU (gloo) and GPU (host-staged) distributed tests.

Each worker builds El::Grid over a host-collective bridge (torch.distributed
gloo), runs the library's redistribution engine / SUMMA drivers on its local
blocks and checks ONLY its own local block against the oracle's extraction
of the same global result — exactly what the reference's own tests do
(tests/core/DistMatrix.cpp:12-78, tests/blas_like/Gemm.cpp:15-49), but
against an oracle instead of self-consistency.
"""
from __future__ import annotations

import os
import random
import traceback

import numpy as np

ORIENTS = {0: "N", 1: "T", 2: "T"}
W_FMT = {0: "f32", 1: "f64", 2: "f16", 3: "bf16"}  # ELX_F32, ELX_F64, ELX_F16, ELX_BF16


def init(rank: int, world: int, port: int):
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from elemental_amd import el
    if os.environ.get("ELX_TEST_BACKEND") == "rccl":
        # one GPU per rank, data over RCCL; gloo only carries the unique id
        from elemental_amd import _lib as L
        L.call("elx_set_device", rank)
        obj = [el.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return el, el.Comm.rccl(rank, world, obj[0])
    from elemental_amd.torch_bridge import GlooBridge
    bridge = GlooBridge()
    return el, el.Comm.host(bridge)


def finish():
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _bits(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a)
    return a.view({8: np.uint64, 4: np.uint32, 2: np.uint16}[a.itemsize])


def redist_worker(rank: int, world: int, port: int, height: int, device: int, dtype: int, m: int, n: int,
                  seed: int):
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        npdt = {el.F64: np.float64, el.F32: np.float32, el.F16: np.float16, el.BF16: "bf16"}[dtype]
        G = oracle.hash_matrix(m, n, seed, 0.0, 5.0, npdt)
        rng = random.Random(seed)  # same sequence on every rank
        pairs = el.VALID_DISTS
        for (U, V) in pairs:
            ca = rng.randrange(oracle.lib().orc_dist_stride(U, r, c))
            ra = rng.randrange(oracle.lib().orc_dist_stride(V, r, c))
            A = el.DistMatrix(g, dtype, U, V, device, root=el.cross_size(U, V, r, c) - 1)
            A.Align(ca, ra)
            A.Resize(m, n)
            A.set_local(oracle.local_block(G, U, V, r, c, g.vc_rank, ca, ra, A.root))
            for (X, Y) in pairs:
                xa = rng.randrange(oracle.lib().orc_dist_stride(X, r, c))
                ya = rng.randrange(oracle.lib().orc_dist_stride(Y, r, c))
                B = el.DistMatrix(g, dtype, X, Y, device, root=rng.randrange(el.cross_size(X, Y, r, c)))
                B.Align(xa, ya)
                B.assign(A)
                want = oracle.local_block(G, X, Y, r, c, g.vc_rank, xa, ya, B.root)
                got = B.get_local()
                tag = f"[{el.DIST_NAMES[X]},{el.DIST_NAMES[Y]}]({xa},{ya}) <- " \
                      f"[{el.DIST_NAMES[U]},{el.DIST_NAMES[V]}]({ca},{ra}) grid {r}x{c} rank {rank}"
                assert got.shape == want.shape, f"{tag}: shape {got.shape} vs {want.shape}"
                assert np.array_equal(_bits(got), _bits(want)), f"{tag}: data mismatch"
                # an unconstrained target adopts an alignment and still holds the matrix
                B2 = el.DistMatrix(g, dtype, X, Y, device)
                B2.assign(A)
                i = B2.info()
                want2 = oracle.local_block(G, X, Y, r, c, g.vc_rank, i["col_align"], i["row_align"], 0)
                assert np.array_equal(_bits(B2.get_local()), _bits(want2)), f"{tag}: unconstrained target"
        finish()
    except Exception:
        traceback.print_exc()
        raise


def _tol(dtype):
    """Unit roundoff the normwise bound uses: f32/f64 eps; for the 16-bit types
    the storage format's (2^-11 f16, 2^-8 bf16) against the exact product of the
    16-bit inputs, as test_local_gemm_16bit."""
    return {0: np.finfo(np.float32).eps, 1: np.finfo(np.float64).eps, 2: 2.0 ** -11, 3: 2.0 ** -8}[dtype]


def _host_dt(dtype):
    return {0: np.float32, 1: np.float64, 2: np.float16, 3: "bf16"}[dtype]


MS_ALGS = (1, 3, 5)  # GEMM_SUMMA_A_MS, GEMM_SUMMA_B_MS, GEMM_SUMMA_C_MS (level3.hpp:22-35)


def gemm_worker(rank: int, world: int, port: int, height: int, device: int, dtype: int, shapes, algs,
                nb: int, seed: int, kc: int = 0, pool: int = 0):
    """El::Gemm NN/NT/TN/TT x `algs` against the oracle (north_star normwise
    tolerance).  kc > 0 forces the C-stationary compute panel to kc columns, so
    k >= 2 kc runs several panels through the two-slot pipeline: on grids larger
    than 1x1 every slot is refilled (gathered) while the previous update may still
    read it (the write-after-read fence of NN.hpp:371-384's loop).  pool > 1
    sets the multistream pool (H_STREAMPOOL_SIZE): the _MS ids then run on that
    many streams (GPU), and GEMM_DEFAULT picks them (NN.hpp:583-600); TT rejects
    the _MS ids (TT.hpp:410-433)."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        fmt = W_FMT[dtype]
        npdt = _host_dt(dtype)
        el.SetBlocksize(nb)
        el.SetComputePanel(kc)
        el.SetStreamPoolSize(pool)
        for (m, n, k) in shapes:
            for oA in (el.NORMAL, el.TRANSPOSE):
                for oB in (el.NORMAL, el.TRANSPOSE):
                    Ag = oracle.hash_matrix(m if oA == 0 else k, k if oA == 0 else m, seed + 1, -0.1, 0.1, npdt)
                    Bg = oracle.hash_matrix(k if oB == 0 else n, n if oB == 0 else k, seed + 2, -0.1, 0.1, npdt)
                    Cg = oracle.hash_matrix(m, n, seed + 3, -0.1, 0.1, npdt)
                    Af, Bf, Cf = (oracle.to_f64(x, fmt) for x in (Ag, Bg, Cg))
                    alpha, beta = 0.5, -0.5  # Gemm_Suite.cpp:158-172
                    # f64/f32: the reference's loop nest in the working precision;
                    # 16-bit: the exact product of the 16-bit inputs
                    ref = oracle.gemm(ORIENTS[oA], ORIENTS[oB], alpha, Ag, Bg, beta, Cg) if dtype in (0, 1) else \
                        oracle.gemm(ORIENTS[oA], ORIENTS[oB], alpha, Af, Bf, beta, Cf)
                    for alg in algs:
                        A = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=Ag.shape[0], width=Ag.shape[1])
                        B = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=Bg.shape[0], width=Bg.shape[1])
                        C = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=m, width=n)
                        A.set_local(oracle.local_block(Ag, el.MC, el.MR, r, c, g.vc_rank))
                        B.set_local(oracle.local_block(Bg, el.MC, el.MR, r, c, g.vc_rank))
                        C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank))
                        if alg in MS_ALGS and oA != el.NORMAL and oB != el.NORMAL:
                            try:
                                el.Gemm(oA, oB, alpha, A, B, beta, C, alg)
                                raise AssertionError("TT with a multistream id must raise")
                            except el.L.LogicError:
                                continue
                        ran = el.Gemm(oA, oB, alpha, A, B, beta, C, alg)
                        if pool > 1 and device == el.GPU and alg == el.GEMM_DEFAULT and \
                                not (oA != el.NORMAL and oB != el.NORMAL):
                            assert ran in MS_ALGS + (el.GEMM_SUMMA_DOT,), ran
                        got = oracle.to_f64(C.get_local(), fmt)
                        want = oracle.local_block(ref, el.MC, el.MR, r, c, g.vc_rank).astype(np.float64)
                        # north_star normwise bound, applied blockwise with the global norms
                        num = np.linalg.norm(got - want) if got.size else 0.0
                        den = np.linalg.norm(Af) * np.linalg.norm(Bf) * max(k, 1) * _tol(dtype)
                        assert np.isfinite(got).all() and num <= 10 * den, (
                            f"Gemm {fmt} {ORIENTS[oA]}{ORIENTS[oB]} alg {alg}->{ran} {m}x{n}x{k} kc {kc} "
                            f"grid {r}x{c} rank {rank}: {num / den:.3g}")
        el.SetComputePanel(0)
        el.SetStreamPoolSize(0)
        finish()
    except Exception:
        traceback.print_exc()
        raise


def syrk_worker(rank: int, world: int, port: int, height: int, device: int, dtype: int, shapes, nb: int,
                seed: int, kc: int = 0):
    """El::Syrk/Herk, Syr2k/Her2k and Trrk, LOWER/UPPER x NORMAL/TRANSPOSE
    (Syrk/*.hpp, Syr2k/*.hpp, Trrk/*.hpp): the uplo triangle against the oracle
    (north_star tolerance), the other triangle bit-identical to the input
    (including NaNs planted there)."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        npdt = np.float64 if dtype == el.F64 else np.float32
        el.SetBlocksize(nb)
        el.SetComputePanel(kc)  # kc > 0: several panels through the triangular pipeline
        for (n, k) in shapes:
            for uplo in (el.LOWER, el.UPPER):
                for orient in (el.NORMAL, el.TRANSPOSE):
                    Ag = oracle.hash_matrix(n if orient == 0 else k, k if orient == 0 else n, seed + 1, -0.1, 0.1,
                                            npdt)
                    Cg = oracle.hash_matrix(n, n, seed + 3, -0.1, 0.1, npdt)
                    i, j = np.indices((n, n))
                    outside = (i < j) if uplo == el.LOWER else (i > j)
                    Cg[outside & ((i + j) % 3 == 0)] = np.nan  # never read
                    alpha, beta = 0.5, -0.5
                    ref = oracle.syrk("L" if uplo == el.LOWER else "U", ORIENTS[orient], alpha, Ag, beta, Cg)
                    A = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=Ag.shape[0], width=Ag.shape[1])
                    C = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=n, width=n)
                    A.set_local(oracle.local_block(Ag, el.MC, el.MR, r, c, g.vc_rank))
                    C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank))
                    if (uplo + orient) % 2:
                        el.Herk(uplo, orient, alpha, A, beta, C)
                    else:
                        el.Syrk(uplo, orient, alpha, A, beta, C)
                    got = C.get_local()
                    want = oracle.local_block(ref, el.MC, el.MR, r, c, g.vc_rank)
                    out_loc = oracle.local_block(outside.astype(np.uint8), el.MC, el.MR, r, c, g.vc_rank).astype(bool)
                    assert np.array_equal(_bits(got[out_loc]), _bits(want[out_loc])), \
                        f"Syrk uplo {uplo} orient {orient} touched the other triangle (rank {rank})"
                    d = (got.astype(np.float64) - want.astype(np.float64))[~out_loc]
                    num = np.linalg.norm(d) if d.size else 0.0
                    den = np.linalg.norm(Ag.astype(np.float64)) ** 2 * max(k, 1) * _tol(dtype)
                    assert num <= 10 * den, (f"Syrk uplo {uplo} orient {orient} n={n} k={k} grid {r}x{c} "
                                             f"rank {rank}: {num / den:.3g}")

                    # Syr2k / Her2k with a second operand of A's shape
                    Bg = oracle.hash_matrix(*Ag.shape, seed + 2, -0.1, 0.1, npdt)
                    ref2 = oracle.syr2k("L" if uplo == el.LOWER else "U", ORIENTS[orient], alpha, Ag, Bg, beta, Cg)
                    B = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=Bg.shape[0], width=Bg.shape[1])
                    B.set_local(oracle.local_block(Bg, el.MC, el.MR, r, c, g.vc_rank))
                    C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank))
                    (el.Her2k if orient else el.Syr2k)(uplo, orient, alpha, A, B, beta, C)
                    got = C.get_local()
                    want = oracle.local_block(ref2, el.MC, el.MR, r, c, g.vc_rank)
                    assert np.array_equal(_bits(got[out_loc]), _bits(want[out_loc])), "Syr2k touched the other triangle"
                    d = (got.astype(np.float64) - want.astype(np.float64))[~out_loc]
                    num = np.linalg.norm(d) if d.size else 0.0
                    den = 2 * np.linalg.norm(Ag.astype(np.float64)) * np.linalg.norm(Bg.astype(np.float64)) \
                        * max(k, 1) * _tol(dtype)
                    assert num <= 10 * den, f"Syr2k uplo {uplo} orient {orient} rank {rank}: {num / den:.3g}"

                    # Trrk with mixed orientations: op(A) n x k, op(B) k x n
                    oB = (orient + uplo) % 2
                    Tg = oracle.hash_matrix(k if oB == 0 else n, n if oB == 0 else k, seed + 4, -0.1, 0.1, npdt)
                    ref3 = oracle.trrk("L" if uplo == el.LOWER else "U", ORIENTS[orient], ORIENTS[oB], alpha,
                                       Ag, Tg, beta, Cg)
                    T = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=Tg.shape[0], width=Tg.shape[1])
                    T.set_local(oracle.local_block(Tg, el.MC, el.MR, r, c, g.vc_rank))
                    C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank))
                    el.Trrk(uplo, orient, oB, alpha, A, T, beta, C)
                    got = C.get_local()
                    want = oracle.local_block(ref3, el.MC, el.MR, r, c, g.vc_rank)
                    assert np.array_equal(_bits(got[out_loc]), _bits(want[out_loc])), "Trrk touched the other triangle"
                    d = (got.astype(np.float64) - want.astype(np.float64))[~out_loc]
                    num = np.linalg.norm(d) if d.size else 0.0
                    den = np.linalg.norm(Ag.astype(np.float64)) * np.linalg.norm(Tg.astype(np.float64)) \
                        * max(k, 1) * _tol(dtype)
                    assert num <= 10 * den, f"Trrk uplo {uplo} oA {orient} oB {oB} rank {rank}: {num / den:.3g}"
        el.SetComputePanel(0)
        finish()
    except Exception:
        traceback.print_exc()
        raise


def trsm_worker(rank: int, world: int, port: int, height: int, device: int, dtype: int, m: int, n: int, nb: int,
                seed: int):
    """El::Trsm, every side x uplo x orientation x diag (Trsm/{LLN,...,RUT}.hpp),
    against oracle.trsm; the triangle (and unit diagonal) A must not read is NaN."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        npdt = np.float64 if dtype == el.F64 else np.float32
        el.SetBlocksize(nb)
        for side in (el.LEFT, el.RIGHT):
            for uplo in (el.LOWER, el.UPPER):
                for orient in (el.NORMAL, el.TRANSPOSE):
                    for diag in (el.NON_UNIT, el.UNIT):
                        k = m if side == el.LEFT else n
                        Ag = oracle.hash_matrix(k, k, seed + 1, 0.0, 0.3, npdt)
                        Ag[np.diag_indices(k)] += npdt(2.0)
                        i, j = np.indices((k, k))
                        Ag[(i < j) if uplo == el.LOWER else (i > j)] = np.nan
                        if diag == el.UNIT:
                            Ag[np.diag_indices(k)] = np.nan
                        Bg = oracle.hash_matrix(m, n, seed + 2, -1.0, 1.0, npdt)
                        alpha = 0.75
                        ref = oracle.trsm("LR"[side], "LU"[uplo], ORIENTS[orient], "NU"[diag], alpha, Ag, Bg)
                        A = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=k, width=k)
                        B = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=m, width=n)
                        A.set_local(oracle.local_block(Ag, el.MC, el.MR, r, c, g.vc_rank))
                        B.set_local(oracle.local_block(Bg, el.MC, el.MR, r, c, g.vc_rank))
                        el.Trsm(side, uplo, orient, diag, alpha, A, B)
                        got = B.get_local().astype(np.float64)
                        want = oracle.local_block(ref, el.MC, el.MR, r, c, g.vc_rank)
                        num = np.linalg.norm(got - want) if got.size else 0.0
                        den = np.linalg.norm(ref) * k * _tol(dtype)
                        assert np.isfinite(got).all() and num <= 10 * den, \
                            (f"Trsm side {side} uplo {uplo} orient {orient} diag {diag} {m}x{n} nb {nb} "
                             f"grid {r}x{c} rank {rank}: {num / den:.3g}")
        finish()
    except Exception:
        traceback.print_exc()
        raise


def symm_worker(rank: int, world: int, port: int, height: int, device: int, dtype: int, m: int, n: int, seed: int):
    """El::Symm / El::Hemm LEFT/RIGHT x LOWER/UPPER (Symm/{LL,LU,RL,RU}.hpp) against
    oracle.symm; A's unread triangle is NaN."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        npdt = np.float64 if dtype == el.F64 else np.float32
        for side in (el.LEFT, el.RIGHT):
            for uplo in (el.LOWER, el.UPPER):
                k = m if side == el.LEFT else n
                Ag = oracle.hash_matrix(k, k, seed + 1, -0.1, 0.1, npdt)
                i, j = np.indices((k, k))
                Ag[(i < j) if uplo == el.LOWER else (i > j)] = np.nan
                Bg = oracle.hash_matrix(m, n, seed + 2, -0.1, 0.1, npdt)
                Cg = oracle.hash_matrix(m, n, seed + 3, -0.1, 0.1, npdt)
                ref = oracle.symm("LR"[side], "LU"[uplo], 0.5, Ag, Bg, -0.5, Cg)
                A = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=k, width=k)
                B = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=m, width=n)
                C = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=m, width=n)
                A.set_local(oracle.local_block(Ag, el.MC, el.MR, r, c, g.vc_rank))
                B.set_local(oracle.local_block(Bg, el.MC, el.MR, r, c, g.vc_rank))
                C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank))
                (el.Hemm if uplo else el.Symm)(side, uplo, 0.5, A, B, -0.5, C)
                got = C.get_local().astype(np.float64)
                want = oracle.local_block(ref, el.MC, el.MR, r, c, g.vc_rank)
                num = np.linalg.norm(got - want) if got.size else 0.0
                Af = np.where(np.isnan(Ag), 0.0, Ag).astype(np.float64)
                den = 2 * np.linalg.norm(Af) * np.linalg.norm(Bg.astype(np.float64)) * k * _tol(dtype)
                assert np.isfinite(got).all() and num <= 10 * den, \
                    f"Symm side {side} uplo {uplo} grid {r}x{c} rank {rank}: {num / den:.3g}"
        finish()
    except Exception:
        traceback.print_exc()
        raise


def cannon_worker(rank: int, world: int, port: int, height: int, device: int, dtype: int, shapes, seed: int):
    """Cannon_NN (src/blas_like/level3/Gemm/NN.hpp:21-104) on a square grid with
    misaligned A, B and C (exercises the initial skew shifts), against the
    oracle; plus the reference's error behaviour (non-NN orientation, width(A)
    not a multiple of sqrt(p), non-square grid)."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        npdt = np.float64 if dtype == el.F64 else np.float32
        from elemental_amd import _lib as L
        if r != c:
            A = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=4, width=4)
            B = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=4, width=4)
            C = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=4, width=4)
            try:
                el.Gemm(el.NORMAL, el.NORMAL, 1.0, A, B, 0.0, C, el.GEMM_CANNON)
                raise AssertionError("Cannon on a non-square grid must raise")
            except L.LogicError:
                pass
            finish()
            return
        rng = np.random.default_rng(seed)
        for (m, n, k) in shapes:
            Ag = oracle.hash_matrix(m, k, seed + 1, -0.1, 0.1, npdt)
            Bg = oracle.hash_matrix(k, n, seed + 2, -0.1, 0.1, npdt)
            Cg = oracle.hash_matrix(m, n, seed + 3, -0.1, 0.1, npdt)
            ref = oracle.gemm("N", "N", 0.5, Ag, Bg, -0.5, Cg)
            # the same random alignments on every rank
            al = [int(x) for x in rng.integers(0, r, 6)]
            A = el.DistMatrix(g, dtype, el.MC, el.MR, device).Align(al[0], al[1])
            B = el.DistMatrix(g, dtype, el.MC, el.MR, device).Align(al[2], al[3])
            C = el.DistMatrix(g, dtype, el.MC, el.MR, device).Align(al[4], al[5])
            A.Resize(m, k)
            B.Resize(k, n)
            C.Resize(m, n)
            A.set_local(oracle.local_block(Ag, el.MC, el.MR, r, c, g.vc_rank, al[0], al[1]))
            B.set_local(oracle.local_block(Bg, el.MC, el.MR, r, c, g.vc_rank, al[2], al[3]))
            C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank, al[4], al[5]))
            if k % r:
                try:
                    el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C, el.GEMM_CANNON)
                    raise AssertionError("Cannon with width(A) % sqrt(p) != 0 must raise")
                except L.LogicError:
                    continue
            el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C, el.GEMM_CANNON)
            got = C.get_local().astype(np.float64)
            want = oracle.local_block(ref, el.MC, el.MR, r, c, g.vc_rank, al[4], al[5]).astype(np.float64)
            num = np.linalg.norm(got - want) if got.size else 0.0
            den = np.linalg.norm(Ag.astype(np.float64)) * np.linalg.norm(Bg.astype(np.float64)) * k * _tol(dtype)
            assert num <= 10 * den, f"Cannon {m}x{n}x{k} grid {r}x{c} rank {rank}: {num / den:.3g}"
        try:  # the other orientations reject GEMM_CANNON (NT.hpp:526 etc.)
            A = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=4, width=4)
            C = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=4, width=4)
            el.Gemm(el.TRANSPOSE, el.NORMAL, 1.0, A, A, 0.0, C, el.GEMM_CANNON)
            raise AssertionError("Cannon TN must raise")
        except L.LogicError:
            pass
        finish()
    except Exception:
        traceback.print_exc()
        raise


def uniform_worker(rank: int, world: int, port: int, height: int, device: int):
    """El::Uniform on a multi-rank grid (Uniform.cpp:53-66): every rank seeds
    (21 << 16) | rank; RedundantRank 0 of each redundant group draws its local
    block in column-major order and broadcasts it to the group."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        m, n = 11, 9
        for (U, V) in ((el.MC, el.MR), (el.STAR, el.STAR), (el.MC, el.STAR), (el.STAR, el.MR), (el.VC, el.STAR),
                       (el.MD, el.STAR), (el.STAR, el.MD), (el.CIRC, el.CIRC)):
            el.InitializeRandom(True, rank)
            A = el.DistMatrix(g, el.F64, U, V, device)
            el.Uniform(A, m, n, 0.0, 1.0)
            lh, lw = A.LocalHeight(), A.LocalWidth()
            # the drawer: the rank of this group whose coordinate along the uncovered
            # grid dimension(s) is 0 (RedundantRank 0)
            # (MD and CIRC: RedundantComm is self, every holder draws its own block)
            covers = {el.MC: "c", el.MR: "r", el.VC: "cr", el.VR: "cr", el.STAR: "", el.MD: "cr", el.CIRC: "cr"}
            cov = covers[U] + covers[V]
            mc, mr = g.mc_rank, g.mr_rank
            d_mc = mc if "c" in cov else 0
            d_mr = mr if "r" in cov else 0
            drawer = d_mc + r * d_mr  # VC rank == world rank (column-major grid)
            want = oracle.mt_uniform((21 << 16) | drawer, lh * lw, -1.0, 1.0).reshape((lh, lw), order="F")
            assert np.array_equal(A.get_local(), want), (el.DIST_NAMES[U], el.DIST_NAMES[V], rank)
        finish()
    except Exception:
        traceback.print_exc()
        raise


def blas1_worker(rank: int, world: int, port: int, height: int, device: int, seed: int):
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        m, n = 23, 17
        Xg = oracle.hash_matrix(m, n, seed, 0.0, 1.0)
        Yg = oracle.hash_matrix(m, n, seed + 1, 0.0, 1.0)
        # Axpy across distributions: Y[MC,MR] += 2 X[VC,STAR]
        X = el.DistMatrix(g, el.F64, el.VC, el.STAR, device, height=m, width=n)
        X.set_local(oracle.local_block(Xg, el.VC, el.STAR, r, c, g.vc_rank))
        Y = el.DistMatrix(g, el.F64, el.MC, el.MR, device, height=m, width=n)
        Y.set_local(oracle.local_block(Yg, el.MC, el.MR, r, c, g.vc_rank))
        el.Axpy(2.0, X, Y)
        want = oracle.local_block(Yg + 2.0 * Xg, el.MC, el.MR, r, c, g.vc_rank)
        assert np.array_equal(Y.get_local(), want), "Axpy"
        # Hadamard on [MC,MR]
        Z = el.DistMatrix(g, el.F64, el.MC, el.MR, device)
        Yc = el.DistMatrix(g, el.F64, el.MC, el.MR, device, height=m, width=n)
        Yc.set_local(oracle.local_block(Yg, el.MC, el.MR, r, c, g.vc_rank))
        Xm = el.DistMatrix(g, el.F64, el.MC, el.MR, device, height=m, width=n)
        Xm.set_local(oracle.local_block(Xg, el.MC, el.MR, r, c, g.vc_rank))
        el.Hadamard(Xm, Yc, Z)
        assert np.array_equal(Z.get_local(), oracle.local_block(Xg * Yg, el.MC, el.MR, r, c, g.vc_rank)), "Hadamard"
        # AxpyContract: [MC,*] partial sums over MR -> [MC,MR]
        D = el.DistMatrix(g, el.F64, el.MC, el.STAR, device, height=m, width=n)
        D.set_local(oracle.local_block(Xg, el.MC, el.STAR, r, c, g.vc_rank) * (g.mr_rank + 1))
        E = el.DistMatrix(g, el.F64, el.MC, el.MR, device, height=m, width=n)
        E.set_local(oracle.local_block(Yg, el.MC, el.MR, r, c, g.vc_rank))
        el.AxpyContract(1.0, D, E)
        # bit-exact: the c contributions summed in rank order (AxpyContract.hpp:
        # 462-478), each addition rounded -- one fused pass over E on the GPU,
        # one axpy per source on the host, the same arithmetic
        want = Yg.copy()
        for q in range(c):
            want = want + Xg * (q + 1)
        want = oracle.local_block(want, el.MC, el.MR, r, c, g.vc_rank)
        assert np.array_equal(E.get_local(), want), "AxpyContract"
        # EntrywiseMap into another distribution
        F = el.DistMatrix(g, el.F64, el.STAR, el.VR, device)
        el.EntrywiseMap(el.L.MAP_SQUARE if hasattr(el, "L") else 3, Xm, F)
        want = oracle.local_block(Xg * Xg, el.STAR, el.VR, r, c, g.vc_rank, 0, F.RowAlign())
        assert np.array_equal(F.get_local(), want), "EntrywiseMap"
        # Combine on matching [MC,MR] blocks: Yc := relu'(Xm) * Yc, then Yc := Yc - Xm
        Yc.set_local(oracle.local_block(Yg - 0.5, el.MC, el.MR, r, c, g.vc_rank))
        el.Combine(el.L.COMBINE_RELU_GRAD, Yc, Xm)  # Xm := (Yc > 0) ? Xm : 0
        want = oracle.local_block(np.where(Yg - 0.5 > 0, Xg, 0.0), el.MC, el.MR, r, c, g.vc_rank)
        assert np.array_equal(Xm.get_local(), want), "Combine relu_grad"
        el.Combine(el.L.COMBINE_SUB, Xm, Yc)  # Yc := Yc - Xm
        want = oracle.local_block((Yg - 0.5) - np.where(Yg - 0.5 > 0, Xg, 0.0), el.MC, el.MR, r, c, g.vc_rank)
        assert np.array_equal(Yc.get_local(), want), "Combine sub"
        try:
            el.Combine(el.L.COMBINE_ADD, F, Yc)  # [STAR,VR] vs [MC,MR]: must refuse
            raise AssertionError("Combine across distributions must raise")
        except el.L.LogicError:
            pass
        # C5's entrywise half: 16-bit Axpy / Hadamard on [MC,MR] (every operation in
        # f32, rounded once to the storage format), plus the in-place Hadamard
        # forms (Z aliasing X or Y, Hadamard.cu:64-116), bit-exact
        for dt, fmt in ((el.F16, "f16"), (el.BF16, "bf16")):
            npdt = _host_dt(dt)
            X16 = oracle.hash_matrix(m, n, seed + 5, 0.0, 4.0, npdt)
            Y16 = oracle.hash_matrix(m, n, seed + 6, 0.0, 4.0, npdt)
            xf, yf = oracle.to_f64(X16, fmt), oracle.to_f64(Y16, fmt)

            def stored(v):  # f32 result -> the 16-bit storage array
                return oracle.convert(np.asarray(v, np.float32).astype(np.float64), "f64", fmt)

            Xd = el.DistMatrix(g, dt, el.MC, el.MR, device, height=m, width=n)
            Yd = el.DistMatrix(g, dt, el.MC, el.MR, device, height=m, width=n)
            Xd.set_local(oracle.local_block(X16, el.MC, el.MR, r, c, g.vc_rank))
            Yd.set_local(oracle.local_block(Y16, el.MC, el.MR, r, c, g.vc_rank))
            el.Axpy(2.0, Xd, Yd)
            want = stored(yf.astype(np.float32) + np.float32(2.0) * xf.astype(np.float32))
            assert np.array_equal(_bits(Yd.get_local()), _bits(oracle.local_block(want, el.MC, el.MR, r, c,
                                                                                  g.vc_rank))), f"Axpy {fmt}"
            Zd = el.DistMatrix(g, dt, el.MC, el.MR, device)
            el.Hadamard(Xd, Yd, Zd)
            y2 = oracle.to_f64(want, fmt)
            prod = stored(xf.astype(np.float32) * y2.astype(np.float32))
            assert np.array_equal(_bits(Zd.get_local()), _bits(oracle.local_block(prod, el.MC, el.MR, r, c,
                                                                                  g.vc_rank))), f"Hadamard {fmt}"
            el.Hadamard(Xd, Yd, Yd)  # Y := X .* Y in place (C aliases B)
            assert np.array_equal(_bits(Yd.get_local()), _bits(Zd.get_local())), f"in-place Hadamard (C = B) {fmt}"
            el.Hadamard(Xd, Xd, Xd)  # X := X .* X in place (C aliases A and B)
            sq = stored(xf.astype(np.float32) * xf.astype(np.float32))
            assert np.array_equal(_bits(Xd.get_local()), _bits(oracle.local_block(sq, el.MC, el.MR, r, c,
                                                                                  g.vc_rank))), f"X.*X in place {fmt}"
            # 16-bit AxpyContract over MR: rank-ordered, each sum in f32 rounded
            # to the storage format before the next source
            contrib = [stored(xf.astype(np.float32) * np.float32(q + 1)) for q in range(c)]
            Dd = el.DistMatrix(g, dt, el.MC, el.STAR, device, height=m, width=n)
            Dd.set_local(oracle.local_block(contrib[g.mr_rank], el.MC, el.STAR, r, c, g.vc_rank))
            Ed = el.DistMatrix(g, dt, el.MC, el.MR, device, height=m, width=n)
            Ed.set_local(oracle.local_block(Y16, el.MC, el.MR, r, c, g.vc_rank))
            el.AxpyContract(1.0, Dd, Ed)
            acc = Y16
            for q in range(c):
                acc = stored(oracle.to_f64(acc, fmt).astype(np.float32) + oracle.to_f64(contrib[q], fmt).astype(np.float32))
            assert np.array_equal(_bits(Ed.get_local()), _bits(oracle.local_block(acc, el.MC, el.MR, r, c,
                                                                                  g.vc_rank))), f"AxpyContract {fmt}"
        finish()
    except Exception:
        traceback.print_exc()
        raise


def io_worker(rank: int, world: int, port: int, height: int, device: int, tmpdir: str):
    """El::Write / El::Read in the reference's BINARY and BINARY_FLAT formats:
    file bytes = [Int h][Int w][column-major data] (Write/Binary.hpp), read back
    into other distributions bit-exactly (src/io/Read.cpp)."""
    import oracle
    import torch.distributed as dist
    from elemental_amd import _lib as L
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        m, n = 13, 11
        for dtype, npdt in ((el.F64, np.float64), (el.F32, np.float32), (el.F16, np.float16)):
            G = oracle.hash_matrix(m, n, 17, 0.0, 3.0, npdt)
            file_vals = G.astype(np.float32) if npdt == np.float16 else G  # half travels as float
            A = el.DistMatrix(g, dtype, el.MC, el.MR, device)
            A.Align(1 % r, 0)
            A.Resize(m, n)
            A.set_local(oracle.local_block(G, el.MC, el.MR, r, c, g.vc_rank, 1 % r, 0))
            for int_bytes in (4, 8):
                base = os.path.join(tmpdir, f"m{dtype}_{int_bytes}")
                el.Write(A, base, el.FILE_BINARY, int_bytes)
                dist.barrier()
                raw = open(base + ".bin", "rb").read()
                idt = np.int32 if int_bytes == 4 else np.int64
                assert np.frombuffer(raw[:2 * int_bytes], dtype=idt).tolist() == [m, n]
                body = np.frombuffer(raw[2 * int_bytes:], dtype=file_vals.dtype)
                assert np.array_equal(body, np.asfortranarray(file_vals).ravel(order="F"))
                for (U, V) in ((el.VC, el.STAR), (el.STAR, el.MR), (el.CIRC, el.CIRC), (el.MD, el.STAR)):
                    B = el.DistMatrix(g, dtype, U, V, device)
                    el.Read(B, base + ".bin", el.FILE_AUTO, int_bytes)
                    i = B.info()
                    assert (i["height"], i["width"]) == (m, n)
                    want = oracle.local_block(G, U, V, r, c, g.vc_rank, i["col_align"], i["row_align"], 0)
                    assert np.array_equal(B.get_local(), want), (dtype, el.DIST_NAMES[U], el.DIST_NAMES[V])
                dist.barrier()
            base = os.path.join(tmpdir, f"f{dtype}")
            el.Write(A, base, el.FILE_BINARY_FLAT)
            dist.barrier()
            assert np.array_equal(np.fromfile(base + ".dat", dtype=file_vals.dtype),
                                  np.asfortranarray(file_vals).ravel(order="F"))
            C = el.DistMatrix(g, dtype, el.STAR, el.VR, device, height=m, width=n)
            el.Read(C, base + ".dat")
            i = C.info()
            assert np.array_equal(C.get_local(), oracle.local_block(G, el.STAR, el.VR, r, c, g.vc_rank, 0,
                                                                    i["row_align"], 0))
            D = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=m + 1, width=n)
            try:
                el.Read(D, base + ".dat")
                raise AssertionError("a size mismatch must raise")
            except L.ElxError as e:
                assert "Expected file to be" in str(e)
            dist.barrier()
        try:
            el.Read(A, os.path.join(tmpdir, "missing.bin"))
            raise AssertionError("a missing file must raise")
        except L.ElxError as e:
            assert "Could not open" in str(e)
        finish()
    except Exception:
        traceback.print_exc()
        raise


FMT = {0: "f32", 1: "f64", 2: "f16", 3: "bf16"}  # ELX_F32, ELX_F64, ELX_F16, ELX_BF16


def convert_values(m: int, n: int, seed: int) -> np.ndarray:
    """float64 test matrix spanning many binades, with round-to-nearest-even ties
    of every target format, signed zeros and f16 overflow/underflow."""
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((m, n)) * np.ldexp(1.0, rng.integers(-30, 20, (m, n)))
    special = [1 + 2.0 ** -11, 1 + 3 * 2.0 ** -11, 1 + 2.0 ** -8, 1 + 3 * 2.0 ** -8, 1 + 2.0 ** -24,
               -(1 + 2.0 ** -8), 0.0, -0.0, 65520.0, 1e6, 2.0 ** -25, 3 * 2.0 ** -26, 1e-30]
    G.flat[: len(special)] = special
    return np.asfortranarray(G)


def convert_worker(rank: int, world: int, port: int, height: int, device: int, seed: int):
    """El::Copy(DistMatrix<S>, DistMatrix<T>) for every S != T over a few
    distribution pairs (same distribution: local conversion; otherwise
    redistribute in S, then convert), bit-exact against the oracle."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        m, n = 21, 17
        G = convert_values(m, n, seed)
        pairs = [((el.MC, el.MR), (el.MC, el.MR)), ((el.MC, el.MR), (el.STAR, el.VR)),
                 ((el.VC, el.STAR), (el.MC, el.MR)), ((el.CIRC, el.CIRC), (el.MR, el.STAR))]
        for S in FMT:
            GS = oracle.convert(G, "f64", FMT[S])
            for T in FMT:
                if S == T:
                    continue
                want_g = oracle.convert(GS, FMT[S], FMT[T])
                for (U, V), (X, Y) in pairs:
                    A = el.DistMatrix(g, S, U, V, device)
                    A.Resize(m, n)
                    A.set_local(oracle.local_block(GS, U, V, r, c, g.vc_rank, 0, 0, 0))
                    for xa in range(min(2, oracle.lib().orc_dist_stride(X, r, c))):
                        B = el.DistMatrix(g, T, X, Y, device)
                        B.Align(xa, 0)
                        el.Copy(A, B)
                        want = oracle.local_block(want_g, X, Y, r, c, g.vc_rank, xa, 0, 0)
                        got = B.get_local()
                        tag = f"{FMT[S]}->{FMT[T]} [{el.DIST_NAMES[X]},{el.DIST_NAMES[Y]}]({xa}) <- " \
                              f"[{el.DIST_NAMES[U]},{el.DIST_NAMES[V]}] grid {r}x{c} rank {rank}"
                        assert got.shape == want.shape, f"{tag}: shape {got.shape} vs {want.shape}"
                        assert np.array_equal(_bits(got), _bits(want)), f"{tag}: data mismatch"
        finish()
    except Exception:
        traceback.print_exc()
        raise


def xdevice_worker(rank: int, world: int, port: int, height: int, seed: int):
    """Cross-device DistMatrix copies (ElementMatrix/setup.hpp:80-160, the CPU<->GPU
    copy constructors BasicGemm.cpp:96-234 validates with), both directions, into
    other distributions and alignments, bit-exact; then Level-3 calls on
    mixed-device operands (A, B brought to C's / X's device like
    DistMatrixReadProxy, Gemm/NN.hpp:357-359) against the oracle."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        m, n = 17, 13
        G = oracle.hash_matrix(m, n, seed, 0.0, 3.0)
        pairs = [((el.MC, el.MR), (el.MC, el.MR)), ((el.MC, el.MR), (el.STAR, el.VR)),
                 ((el.VC, el.STAR), (el.MR, el.MC)), ((el.STAR, el.STAR), (el.MC, el.STAR)),
                 ((el.CIRC, el.CIRC), (el.VR, el.STAR))]
        for src_dev, dst_dev in ((el.CPU, el.GPU), (el.GPU, el.CPU)):
            for (U, V), (X, Y) in pairs:
                A = el.DistMatrix(g, el.F64, U, V, src_dev)
                A.Align(1 % oracle.lib().orc_dist_stride(U, r, c), 0)
                A.Resize(m, n)
                A.set_local(oracle.local_block(G, U, V, r, c, g.vc_rank, A.ColAlign(), A.RowAlign(), 0))
                for xa in range(min(2, oracle.lib().orc_dist_stride(X, r, c))):
                    B = el.DistMatrix(g, el.F64, X, Y, dst_dev).Align(xa, 0)
                    B.assign(A)
                    want = oracle.local_block(G, X, Y, r, c, g.vc_rank, xa, 0, 0)
                    assert np.array_equal(_bits(B.get_local()), _bits(want)), \
                        (src_dev, dst_dev, el.DIST_NAMES[U], el.DIST_NAMES[V], el.DIST_NAMES[X], el.DIST_NAMES[Y])
        # El::Gemm with A on one device and B, C on another (both ways)
        mm, nn, kk = 19, 11, 23
        Ag = oracle.hash_matrix(mm, kk, seed + 1, -0.1, 0.1)
        Bg = oracle.hash_matrix(kk, nn, seed + 2, -0.1, 0.1)
        Cg = oracle.hash_matrix(mm, nn, seed + 3, -0.1, 0.1)
        ref = oracle.gemm("N", "N", 0.5, Ag, Bg, -0.5, Cg)
        for a_dev, c_dev in ((el.CPU, el.GPU), (el.GPU, el.CPU)):
            for alg in (el.GEMM_SUMMA_C, el.GEMM_SUMMA_A, el.GEMM_SUMMA_DOT):
                A = el.DistMatrix(g, el.F64, el.MC, el.MR, a_dev, height=mm, width=kk)
                B = el.DistMatrix(g, el.F64, el.VC, el.STAR, c_dev, height=kk, width=nn)
                C = el.DistMatrix(g, el.F64, el.MC, el.MR, c_dev, height=mm, width=nn)
                A.set_local(oracle.local_block(Ag, el.MC, el.MR, r, c, g.vc_rank))
                B.set_local(oracle.local_block(Bg, el.VC, el.STAR, r, c, g.vc_rank))
                C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank))
                el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C, alg)
                got = C.get_local()
                want = oracle.local_block(ref, el.MC, el.MR, r, c, g.vc_rank)
                num = np.linalg.norm(got - want) if got.size else 0.0
                den = np.linalg.norm(Ag) * np.linalg.norm(Bg) * kk * _tol(1)
                assert num <= 10 * den, (a_dev, c_dev, alg, num / den)
        # El::Trsm with the triangle on the CPU and the right-hand sides on the GPU
        Tg = oracle.hash_matrix(kk, kk, seed + 4, 0.0, 0.3)
        Tg[np.diag_indices(kk)] += 2.0
        Rg = oracle.hash_matrix(kk, nn, seed + 5, -1.0, 1.0)
        T = el.DistMatrix(g, el.F64, el.MC, el.MR, el.CPU, height=kk, width=kk)
        R = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=kk, width=nn)
        T.set_local(oracle.local_block(Tg, el.MC, el.MR, r, c, g.vc_rank))
        R.set_local(oracle.local_block(Rg, el.MC, el.MR, r, c, g.vc_rank))
        el.Trsm(el.LEFT, el.LOWER, el.NORMAL, el.NON_UNIT, 1.0, T, R)
        ref = oracle.trsm("L", "L", "N", "N", 1.0, Tg, Rg)
        got = R.get_local()
        want = oracle.local_block(ref, el.MC, el.MR, r, c, g.vc_rank)
        assert np.linalg.norm(got - want) <= 10 * np.linalg.norm(ref) * kk * _tol(1)
        finish()
    except Exception:
        traceback.print_exc()
        raise


def half_sum_worker(rank: int, world: int, port: int, seed: int):
    """elx_comm_reduce_scatter / allreduce in f16 and bf16 over the host
    backend against the rank-order fold with per-addition 16-bit rounding."""
    import ctypes
    import oracle
    from elemental_amd import _lib as L
    el, comm = init(rank, world, port)
    try:
        count = 37
        for dt, fmt in ((el.F16, "f16"), (el.BF16, "bf16")):
            npdt = _host_dt(dt)
            contrib = [oracle.hash_matrix(count * world, 1, seed + q, 0.0, 8.0, npdt).ravel(order="F")
                       for q in range(world)]
            send = np.ascontiguousarray(contrib[rank])
            recv = np.zeros(count, dtype=send.dtype)
            L.call("elx_comm_reduce_scatter", comm.h, dt, send.ctypes.data_as(ctypes.c_void_p),
                   recv.ctypes.data_as(ctypes.c_void_p), count, None)

            def fold(parts):
                acc = oracle.to_f64(parts[0], fmt)
                for q in range(1, len(parts)):
                    s32 = (oracle.to_f64(parts[q], fmt).astype(np.float32) + acc.astype(np.float32))
                    acc = oracle.round_to_format(s32.astype(np.float64), fmt)
                return acc

            want = fold([c[rank * count:(rank + 1) * count] for c in contrib])
            assert np.array_equal(oracle.to_f64(recv, fmt), want), (fmt, rank)
        finish()
    except Exception:
        traceback.print_exc()
        raise


def raw_coll_worker(rank: int, world: int, port: int):
    """The raw El::mpi collectives of the C-ABI (elx_comm_*) on the world and on
    a Split of it: AllGather, ReduceScatter (SUM), AllReduce (SUM), Bcast,
    AllToAll, SendRecv (src/core/imports/mpi/*.hpp), exact integer-valued f64."""
    el, comm = init(rank, world, port)
    rccl = os.environ.get("ELX_TEST_BACKEND") == "rccl"
    if rccl:  # RCCL comms take device buffers
        import torch
        from elemental_amd import _lib as L

        class Dev:
            def __init__(self, a):
                self.t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
                torch.cuda.synchronize()

            def np(self):
                L.call("elx_device_synchronize")
                return self.t.cpu().numpy()
        buf = lambda a: Dev(a)
        ptr = lambda b: b.t.data_ptr()
        get = lambda b: b.np()
    else:
        buf = lambda a: np.array(a, dtype=np.float64)
        ptr = lambda b: b
        get = lambda b: b
    try:
        def check(c, tag):
            p, r = c.size, c.rank
            n = 5
            mine_h = np.arange(n, dtype=np.float64) + 100 * r
            mine, out = buf(mine_h), buf(np.zeros(n * p))
            c.allgather(el.F64, ptr(mine), ptr(out), n)
            assert np.array_equal(get(out), np.concatenate([np.arange(n) + 100 * q for q in range(p)])), tag
            send = buf(np.concatenate([np.arange(n) + 10 * q + r for q in range(p)]).astype(np.float64))
            rs = buf(np.zeros(n))
            c.reduce_scatter(el.F64, ptr(send), ptr(rs), n)
            assert np.array_equal(get(rs), p * (np.arange(n) + 10 * r) + sum(range(p))), tag
            ar = buf(np.zeros(n))
            c.allreduce(el.F64, ptr(mine), ptr(ar), n)
            assert np.array_equal(get(ar), p * np.arange(n) + 100 * sum(range(p))), tag
            root = p - 1
            b = buf(mine_h.copy())
            c.bcast(el.F64, ptr(b), n, root)
            assert np.array_equal(get(b), np.arange(n) + 100 * root), tag
            a2a_send = buf(np.concatenate([np.full(n, 1000 * r + q, dtype=np.float64) for q in range(p)]))
            a2a = buf(np.zeros(n * p))
            c.alltoall(el.F64, ptr(a2a_send), ptr(a2a), n)
            assert np.array_equal(get(a2a), np.concatenate([np.full(n, 1000 * q + r) for q in range(p)])), tag
            ring = buf(np.zeros(n))
            c.sendrecv(el.F64, ptr(mine), (r + 1) % p, ptr(ring), (r - 1) % p, n)
            assert np.array_equal(get(ring), np.arange(n) + 100 * ((r - 1) % p)), tag

        check(comm, "world")
        sub = comm.split(rank % 2, -rank)  # key reverses the order inside each half
        members = [q for q in range(world) if q % 2 == rank % 2]
        assert sub.size == len(members)
        assert sub.rank == sorted(members, reverse=True).index(rank)
        check(sub, "split")
        finish()
    except Exception:
        traceback.print_exc()
        raise


def mpi_typed_worker(rank: int, world: int, port: int, device: int):
    """El::mpi's typed collectives with an explicit buffer device (elx_mpi_*,
    what El.hpp's El::mpi::AllGather / ReduceScatter / AllReduce / AllToAll /
    Broadcast / SendRecv(..., SyncInfo<D>) bind; imports/mpi.hpp:593-1400):
    every op (SUM, PROD, MAX, MIN) in f64, f32, f16 and bf16 against a rank-order
    numpy fold, on the world and on a split.  device = GPU: device buffers (RCCL,
    or staged through the host backend); device = CPU: host buffers (staged
    through device memory on an RCCL communicator).  Integer-valued inputs, so
    every op is exact in every type and every backend's order."""
    import ctypes
    import oracle
    from elemental_amd import _lib as L
    el, comm = init(rank, world, port)
    rccl = os.environ.get("ELX_TEST_BACKEND") == "rccl"
    if device == el.GPU:
        import torch

        def buf(a):
            return torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()

        def ptr(b):
            return ctypes.c_void_p(b.data_ptr())

        def get(b):
            L.call("elx_device_synchronize")
            torch.cuda.synchronize()
            return b.cpu().numpy()
    else:
        def buf(a):
            return np.ascontiguousarray(a).copy()

        def ptr(b):
            return b.ctypes.data_as(ctypes.c_void_p)

        def get(b):
            return b
    fmts = ((el.F64, "f64", np.float64), (el.F32, "f32", np.float32), (el.F16, "f16", np.float16),
            (el.BF16, "bf16", np.uint16), (L.I32, "i32", np.int32), (L.I64, "i64", np.int64))
    folds = {0: lambda a, b: b + a, 1: lambda a, b: b * a, 2: np.maximum, 3: np.minimum}

    def enc(x, fmt, npdt):  # exact small integers in the storage format
        if fmt == "bf16":
            return oracle.convert(np.asarray(x, dtype=np.float64), "f64", "bf16")
        return np.asarray(x, dtype=npdt)

    def dec(x, fmt):
        return np.asarray(x).astype(np.float64) if fmt in ("i32", "i64") else oracle.to_f64(x, fmt)

    try:
        def check(c, tag):
            p, r = c.size, c.rank
            n = 7
            for dt, fmt, npdt in fmts:
                def vals(q, salt):
                    i = (np.arange(n * p) * 3 + 5 * q + salt) % 7
                    if salt % 10 == 1:  # PROD: signed powers of two stay exact in every format
                        return np.array([-1.0, 1.0, 2.0, 1.0, -2.0, 1.0, 1.0])[i]
                    return (i - 3).astype(np.float64)
                # AllGather
                mine = buf(enc(vals(r, 1)[:n], fmt, npdt))
                out = buf(enc(np.zeros(n * p), fmt, npdt))
                L.call("elx_mpi_allgather", c.h, dt, device, ptr(mine), ptr(out), n, None)
                want = np.concatenate([vals(q, 1)[:n] for q in range(p)])
                assert np.array_equal(dec(get(out), fmt), want), (tag, fmt, "allgather")
                for op in (0, 1, 2, 3):
                    # AllReduce: fold rank 0..p-1 in order (exact on small integers)
                    send = buf(enc(vals(r, op)[:n], fmt, npdt))
                    recv = buf(enc(np.zeros(n), fmt, npdt))
                    L.call("elx_mpi_allreduce", c.h, dt, device, op, ptr(send), ptr(recv), n, None)
                    acc = vals(0, op)[:n]
                    for q in range(1, p):
                        acc = folds[op](acc, vals(q, op)[:n])
                    assert np.array_equal(dec(get(recv), fmt), acc), (tag, fmt, "allreduce", op)
                    # in place (send == recv)
                    io = buf(enc(vals(r, op)[:n], fmt, npdt))
                    L.call("elx_mpi_allreduce", c.h, dt, device, op, ptr(io), ptr(io), n, None)
                    assert np.array_equal(dec(get(io), fmt), acc), (tag, fmt, "allreduce in place", op)
                    # ReduceScatter: my slice of every rank's n*p vector
                    send = buf(enc(vals(r, op + 10), fmt, npdt))
                    recv = buf(enc(np.zeros(n), fmt, npdt))
                    L.call("elx_mpi_reduce_scatter", c.h, dt, device, op, ptr(send), ptr(recv), n, None)
                    acc = vals(0, op + 10)[r * n:(r + 1) * n]
                    for q in range(1, p):
                        acc = folds[op](acc, vals(q, op + 10)[r * n:(r + 1) * n])
                    assert np.array_equal(dec(get(recv), fmt), acc), (tag, fmt, "reduce_scatter", op)
                # AllToAll
                send = buf(enc(np.concatenate([np.full(n, (10 * r + q) % 50) for q in range(p)]), fmt, npdt))
                recv = buf(enc(np.zeros(n * p), fmt, npdt))
                L.call("elx_mpi_alltoall", c.h, dt, device, ptr(send), ptr(recv), n, None)
                want = np.concatenate([np.full(n, (10 * q + r) % 50) for q in range(p)])
                assert np.array_equal(dec(get(recv), fmt), want), (tag, fmt, "alltoall")
                # Broadcast from the last rank
                b = buf(enc(vals(r, 3)[:n], fmt, npdt))
                L.call("elx_mpi_bcast", c.h, dt, device, ptr(b), n, p - 1, None)
                assert np.array_equal(dec(get(b), fmt), vals(p - 1, 3)[:n]), (tag, fmt, "bcast")
                # SendRecv around the ring; unequal counts where the backend allows them
                rc_ = n if not rccl else n - 2 + ((r - 1) % p) % 3
                sc_ = n if not rccl else n - 2 + r % 3
                send = buf(enc(vals(r, 4)[:sc_], fmt, npdt))
                recv = buf(enc(np.zeros(max(rc_, 1)), fmt, npdt))
                L.call("elx_mpi_sendrecv", c.h, dt, device, ptr(send), sc_, (r + 1) % p, ptr(recv), rc_,
                       (r - 1) % p, None)
                assert np.array_equal(dec(get(recv), fmt)[:rc_], vals((r - 1) % p, 4)[:rc_]), (tag, fmt, "sendrecv")
            # bytes (El::byte buffers): gather and broadcast, bit-exact
            if p > 0:
                mine = buf(np.arange(5, dtype=np.uint8) + 17 * r)
                out = buf(np.zeros(5 * p, dtype=np.uint8))
                L.call("elx_mpi_allgather", c.h, L.U8, device, ptr(mine), ptr(out), 5, None)
                want = np.concatenate([np.arange(5, dtype=np.uint8) + 17 * q for q in range(p)])
                assert np.array_equal(np.asarray(get(out)).astype(np.uint8), want), (tag, "u8")
            # error mapping: a bad op and a bad root are LogicErrors
            x = buf(np.zeros(2))
            for call in (lambda: L.call("elx_mpi_allreduce", c.h, el.F64, device, 9, ptr(x), ptr(x), 2, None),
                         lambda: L.call("elx_mpi_bcast", c.h, el.F64, device, ptr(x), 2, p, None)):
                try:
                    call()
                    raise AssertionError("expected a LogicError")
                except L.LogicError:
                    pass

        check(comm, "world")
        if world > 1:
            sub = comm.split(rank % 2, rank)
            check(sub, "split")
        finish()
    except Exception:
        traceback.print_exc()
        raise


def frobenius_worker(rank: int, world: int, port: int, height: int, device: int):
    """El::FrobeniusNorm (src/lapack_like/props/Norm/Frobenius.cpp:20-60) of
    DistMatrices against numpy's norm of the same global values: f64, f32, f16,
    bf16; ragged shapes wider than 128 columns; [MC,MR], the replicated
    [STAR,STAR] and [MC,STAR] (each entry counted once), [VC,STAR]; a NaN
    anywhere gives NaN, an inf gives inf, values near the f64 overflow
    threshold stay finite (the scaled sum of squares)."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        g = el.Grid(comm, height)
        r, c = g.height, g.width
        dists = [(el.MC, el.MR), (el.STAR, el.STAR), (el.MC, el.STAR), (el.VC, el.STAR)]
        for dt in (el.F64, el.F32, el.F16, el.BF16):
            fmt, npdt = W_FMT[dt], _host_dt(dt)
            rtol = 1e-13 if dt == el.F64 else 1e-6
            for (m, n) in ((37, 300), (130, 129), (1, 517), (0, 5)):
                Xg = oracle.hash_matrix(m, n, 17 + m, -1.0, 3.0, npdt)
                want = float(np.linalg.norm(oracle.to_f64(Xg, fmt))) if Xg.size else 0.0
                for (U, V) in dists:
                    X = el.DistMatrix(g, dt, U, V, device, height=m, width=n)
                    X.set_local(oracle.local_block(Xg, U, V, r, c, g.vc_rank))
                    got = el.FrobeniusNorm(X)
                    assert abs(got - want) <= rtol * max(want, 1e-300), (fmt, m, n, U, V, got, want)
        # special values (f64 and f32 only: the 16-bit hash has no large range)
        for dt, big in ((el.F64, 1e300), (el.F32, 3e37)):
            npdt = _host_dt(dt)
            m, n = 20, 140
            base = np.asfortranarray(np.full((m, n), big, dtype=npdt))
            X = el.DistMatrix(g, dt, el.MC, el.MR, device, height=m, width=n)
            X.set_local(oracle.local_block(base, el.MC, el.MR, r, c, g.vc_rank))
            got = el.FrobeniusNorm(X)
            want = float(big) * np.sqrt(m * n)
            assert np.isfinite(got) and abs(got - want) <= 1e-6 * want, (dt, got, want)
            for bad, check in ((np.nan, np.isnan), (np.inf, np.isposinf)):
                Y = base.copy()
                Y[7, 133] = bad
                X.set_local(oracle.local_block(Y, el.MC, el.MR, r, c, g.vc_rank))
                got = el.FrobeniusNorm(X)
                assert check(got), (dt, bad, got)
        finish()
    except Exception:
        traceback.print_exc()
        raise


# tests/golden/mkl_summa.npz cases: dtype_grid_nb_mxnxk
# tests/golden/mkl_summa_orient.npz: NT / TN / TT through SUMMA_C, TN / NN through SUMMA_DOT
MKL_ORIENT = [f"{t}_{g}_{o}_C" for t in ("f64", "f32")
              for g in ("2x2_nb16_45x37x61", "2x4_nb16_53x66x130") for o in ("NT", "TN", "TT")] + \
             [f"{t}_{g}_{o}_DOT" for t in ("f64", "f32")
              for g in ("2x2_nb16_20x24x130", "2x4_nb16_19x30x257") for o in ("TN", "NN")]
MKL_C1 = ["f64_2x2_nb128_4096x4096x4096_NN_C_sample"]
MKL_SUMMA = ["f64_2x2_nb16_45x37x61", "f64_1x2_nb8_30x41x27", "f64_2x4_nb16_53x66x130", "f64_2x2_nb128_260x200x300",
             "f32_2x2_nb16_45x37x61", "f32_1x2_nb8_30x41x27", "f32_2x4_nb16_53x66x130", "f32_2x2_nb128_260x200x300"]


def mkl_summa_worker(rank: int, world: int, port: int, height: int, device: int, keys,
                     fixture: str = "mkl_summa.npz"):
    """El::Gemm with the fixture's orientation, algorithm and Blocksize on its
    grid, against the reference's SUMMA evaluated through MKL rank by rank
    (tests/golden/mkl_summa*.npz, tools/make_mkl_golden.py): each rank checks
    its own local block with the north_star normwise bound (global norms).
    Keys: {f64,f32}_{r}x{c}_nb{nb}_{m}x{n}x{k}[_{oA}{oB}_{C,DOT}[_sample]]; a
    _sample fixture holds rows 0::sr x columns 0::sc of the result and only
    those entries are compared."""
    import oracle
    el, comm = init(rank, world, port)
    try:
        gold = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", fixture))
        for key in keys:
            parts = key.split("_")
            r, c = map(int, parts[1].split("x"))
            if r * c != world:
                continue
            nb = int(parts[2][2:])
            m, n, k = map(int, parts[3].split("x"))
            oa, ob = (parts[4][0], parts[4][1]) if len(parts) > 4 else ("N", "N")
            alg = {"C": el.GEMM_SUMMA_C, "DOT": el.GEMM_SUMMA_DOT}[parts[5]] if len(parts) > 5 else el.GEMM_SUMMA_C
            sample = parts[-1] == "sample"
            dt = np.float64 if parts[0] == "f64" else np.float32
            dtype = el.F64 if dt == np.float64 else el.F32
            s = [int(x) for x in gold[key + "_seed"]]
            ah, aw = (m, k) if oa == "N" else (k, m)
            bh, bw = (k, n) if ob == "N" else (n, k)
            Ag = oracle.hash_matrix(ah, aw, s[0], 0.0, 0.1, dt)
            Bg = oracle.hash_matrix(bh, bw, s[1], 0.0, 0.1, dt)
            Cg = oracle.hash_matrix(m, n, s[2], 0.0, 0.1, dt)
            g = el.Grid(comm, r)
            assert (g.height, g.width) == (r, c)
            el.SetBlocksize(nb)
            A = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=ah, width=aw)
            B = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=bh, width=bw)
            C = el.DistMatrix(g, dtype, el.MC, el.MR, device, height=m, width=n)
            A.set_local(oracle.local_block(Ag, el.MC, el.MR, r, c, g.vc_rank))
            B.set_local(oracle.local_block(Bg, el.MC, el.MR, r, c, g.vc_rank))
            C.set_local(oracle.local_block(Cg, el.MC, el.MR, r, c, g.vc_rank))
            orient = {"N": el.NORMAL, "T": el.TRANSPOSE}
            el.Gemm(orient[oa], orient[ob], 0.5, A, B, -0.5, C, alg)
            got = C.get_local().astype(np.float64)
            den = np.linalg.norm(Ag.astype(np.float64)) * np.linalg.norm(Bg.astype(np.float64)) * k * np.finfo(dt).eps
            if sample:
                sr, sc = (int(x) for x in gold[key + "_stride"])
                mc, mr = g.vc_rank % r, g.vc_rank // r
                rows = np.arange(mc, m, r)   # this rank's global rows / columns ([MC,MR], alignment 0)
                cols = np.arange(mr, n, c)
                ri, ci = np.nonzero(rows % sr == 0)[0], np.nonzero(cols % sc == 0)[0]
                got = got[np.ix_(ri, ci)]
                want = gold[key][np.ix_(rows[ri] // sr, cols[ci] // sc)].astype(np.float64)
            else:
                want = oracle.local_block(gold[key], el.MC, el.MR, r, c, g.vc_rank).astype(np.float64)
            num = np.linalg.norm(got - want) if got.size else 0.0
            assert np.isfinite(got).all() and num <= 10 * den, f"{key} rank {rank}: {num / den:.3g}"
            if sample:  # the sampled entries are checked one by one as well
                assert np.all(np.abs(got - want) <= 64 * np.finfo(dt).eps * k * 0.01), f"{key} rank {rank}"
        el.SetBlocksize(128)
        finish()
    except Exception:
        traceback.print_exc()
        raise
