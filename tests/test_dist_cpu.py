"""Multi-rank CPU tests (gloo, world sizes 2 and 4): the SAME C++ redistribution
engine and SUMMA drivers that run on RCCL, on Device::CPU matrices over a
host-collective bridge.  Grids 1x2, 2x1, 2x2."""
import socket

import pytest
import torch.multiprocessing as mp

import _dist_workers as W
from elemental_amd import el


def _port():
    """A free rendezvous port below the kernel's ephemeral range (32768-60999):
    a port picked by bind(0) comes from that range, and the outgoing gloo sockets
    of the test before can take it again before the store listens (EADDRINUSE)."""
    import random
    for _ in range(200):
        p = random.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port in 20000-32000")


def _spawn(fn, world, *args):
    mp.spawn(fn, args=(world, _port()) + args, nprocs=world, join=True)


def test_gemm_multistream_ids_on_cpu():
    """_MS ids on Device::CPU matrices run the plain variants (the reference warns
    "CPU doesn't support multistream variants", TN.hpp:114-118); TT rejects them."""
    algs = [el.GEMM_SUMMA_A_MS, el.GEMM_SUMMA_B_MS, el.GEMM_SUMMA_C_MS, el.GEMM_DEFAULT]
    _spawn(W.gemm_worker, 2, 1, el.CPU, el.F64, [(19, 13, 23)], algs, 4, 61, 8, 3)


@pytest.mark.parametrize("world,height", [(2, 1), (2, 2), (4, 2), (8, 2)])
def test_redistribution_all_pairs_bit_exact(world, height):
    """tests/core/DistMatrix.cpp: every [X,Y] <- [U,V] of the 14 distributions
    with random alignments and roots (2x4: MD diagonals of length lcm = 4)."""
    _spawn(W.redist_worker, world, height, el.CPU, el.F64, 13, 11, 1234 + world + height)


def test_redistribution_f16_bit_exact():
    _spawn(W.redist_worker, 2, 1, el.CPU, el.F16, 9, 7, 99)


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2)])
def test_gemm_all_orientations_all_algorithms(world, height):
    """SUMMA A/B/C/Dot x NN/NT/TN/TT against the oracle (north_star tolerance)."""
    algs = [el.GEMM_DEFAULT, el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT,
            el.GEMM_SUMMA_C_MS]
    _spawn(W.gemm_worker, world, height, el.CPU, el.F64, [(19, 13, 23), (8, 9, 40)], algs, 4, 7)


def test_gemm_f32_grid_2x2():
    _spawn(W.gemm_worker, 4, 2, el.CPU, el.F32, [(17, 21, 15)], [el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT], 4, 11)


@pytest.mark.parametrize("dtype", [el.F64, el.F32])
def test_gemm_grid_2x4(dtype):
    """C3's grid shape: 8 ranks as 2x4 (Grid::DefaultHeight(8) = 2), every
    orientation and algorithm (f32: C and Dot)."""
    algs = [el.GEMM_DEFAULT, el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT] \
        if dtype == el.F64 else [el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT]
    _spawn(W.gemm_worker, 8, 2, el.CPU, dtype, [(19, 26, 21)], algs, 4, 13)


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2), (8, 2)])
def test_gemm_multi_panel_pipeline(world, height):
    """SUMMA_C with the compute panel forced to 8 columns and k = 61: eight panels
    through the two slots on 1x2 / 2x2 / 2x4 grids, so every slot is regathered
    while the previous update may still read it (NN.hpp:371-384)."""
    _spawn(W.gemm_worker, world, height, el.CPU, el.F64, [(21, 18, 61)], [el.GEMM_SUMMA_C, el.GEMM_SUMMA_C_MS],
           4, 19, 8)


@pytest.mark.parametrize("world,height", [(2, 1), (8, 2)])
def test_gemm_first_panel_ramp(world, height):
    """Compute panel 16 = 4 x nb on a grid larger than 1x1: the panels ramp up a
    quarter and a half deep, then 16 columns, and a ragged last one (k = 61:
    4, 8, 16, 16, 16, 1); k = 13 < kc (4, 8, 1) and k = 20 (4, 8, 8) end inside
    the ramp."""
    _spawn(W.gemm_worker, world, height, el.CPU, el.F64, [(21, 18, 61), (9, 11, 13), (10, 7, 20)],
           [el.GEMM_SUMMA_C], 4, 47, 16)


@pytest.mark.parametrize("dtype", [el.F16, el.BF16])
@pytest.mark.parametrize("world,height", [(2, 1), (4, 2)])
def test_gemm_16bit_distributed(dtype, world, height):
    """C5's distributed 16-bit El::Gemm on [MC,MR] (f32 accumulation), every
    orientation and algorithm, against the exact product of the 16-bit inputs."""
    algs = [el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT]
    _spawn(W.gemm_worker, world, height, el.CPU, dtype, [(23, 17, 29)], algs, 4, 23)


def test_syrk_multi_panel_pipeline():
    """Syrk/Trrk/Syr2k through the triangular pipeline with 4-column compute
    panels on a 2x2 grid (k = 30: eight panels)."""
    _spawn(W.syrk_worker, 4, 2, el.CPU, el.F64, [(23, 30)], 4, 29, 4)


def test_host_backend_16bit_sums():
    """Reduce-scatter / all-reduce of f16 and bf16 on the host backend: the
    library folds contributions in rank order, each addition in float rounded
    back to 16 bits (GPUHalfSumFunc, src/core/environment.cpp:135-142)."""
    _spawn(W.half_sum_worker, 4, 3)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_raw_collectives(world):
    """elx_comm_{allgather,reduce_scatter,allreduce,bcast,alltoall,sendrecv,split}
    on the host backend, on the world and on a split with reversed keys."""
    _spawn(W.raw_coll_worker, world)


@pytest.mark.parametrize("world,height", [(1, 1), (2, 2), (4, 2)])
def test_frobenius_norm(world, height):
    """El::FrobeniusNorm over distributions, types, replication and specials."""
    _spawn(W.frobenius_worker, world, height, el.CPU)


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_mpi_typed_collectives(world):
    """elx_mpi_* (El.hpp's El::mpi::AllGather / ReduceScatter / AllReduce /
    AllToAll / Broadcast / SendRecv on SyncInfo<Device::CPU>): SUM, PROD, MAX,
    MIN in every element type, host buffers, world and split."""
    _spawn(W.mpi_typed_worker, world, el.CPU)


@pytest.mark.parametrize("world,height,cols", [(1, 1, 0), (2, 1, 0), (4, 2, 0), (1, 1, 3), (4, 2, 2), (2, 2, 5)])
def test_syrk_herk(world, height, cols, monkeypatch):
    """El::Syrk / El::Herk LN/LT/UN/UT on 1x1, 1x2, 2x1 and 2x2 grids (Syrk/*.hpp);
    cols > 0 cuts the local triangular update into many ragged column blocks."""
    if cols:
        monkeypatch.setenv("ELX_TRRK_COLS", str(cols))
        monkeypatch.setenv("ELX_TRRK_ROWS", str(1 + cols % 3))
    _spawn(W.syrk_worker, world, height, el.CPU, el.F64, [(23, 9), (7, 30)], 4, 17)


@pytest.mark.parametrize("world,height,flat", [(1, 1, 0), (2, 1, 0), (2, 2, 0), (4, 2, 0), (1, 1, 1),
                                               (4, 2, 1)])
def test_trsm(world, height, flat, monkeypatch):
    """El::Trsm LEFT/RIGHT x LOWER/UPPER x N/T x NON_UNIT/UNIT, ragged blocks (nb = 4):
    the recursive split (deep updates), and flat = 1 the reference's nb-step sweep."""
    if flat:
        monkeypatch.setenv("ELX_TRSM_FLAT", "1")
    _spawn(W.trsm_worker, world, height, el.CPU, el.F64, 19, 13, 4, 31)


@pytest.mark.parametrize("world,height", [(1, 1), (2, 1), (4, 2)])
def test_symm_hemm(world, height):
    """El::Symm / El::Hemm, LEFT/RIGHT x LOWER/UPPER; A's other triangle is NaN."""
    _spawn(W.symm_worker, world, height, el.CPU, el.F64, 17, 11, 51)


@pytest.mark.parametrize("world,height", [(1, 1), (4, 2), (2, 1)])
def test_gemm_cannon(world, height):
    """Cannon_NN on 1x1 and 2x2 with random alignments; LogicError on a 2x1 grid,
    for width(A) % sqrt(p) != 0 and for non-NN orientations."""
    _spawn(W.cannon_worker, world, height, el.CPU, el.F64, [(19, 13, 24), (8, 9, 40), (5, 7, 9)], 5)


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2)])
def test_uniform_reference_draws(world, height):
    """El::Uniform = the reference's per-rank mt19937 draws + redundant broadcast."""
    _spawn(W.uniform_worker, world, height, el.CPU)


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2), (8, 2)])
def test_blas1_distributed(world, height):
    _spawn(W.blas1_worker, world, height, el.CPU, 5)


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2)])
def test_write_read_binary(world, height, tmp_path):
    """El::Write / El::Read, BINARY and BINARY_FLAT (src/io/Write.cpp, Read.cpp)."""
    _spawn(W.io_worker, world, height, el.CPU, str(tmp_path))


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2)])
def test_copy_type_conversion(world, height):
    """El::Copy between element types (CopyDistMatrix.hpp:28-57) on CPU matrices:
    all 12 ordered pairs of {f32, f64, f16, bf16}, bit-exact vs the oracle."""
    _spawn(W.convert_worker, world, height, el.CPU, 7)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_summa_matches_mkl_reference_path(world):
    """The library's SUMMA_C on Device::CPU (gloo) against the reference CPU
    path's own arithmetic: SUMMA_NNC evaluated rank by rank through MKL
    2021.4.0 (tests/golden/mkl_summa.npz), 1x2 / 2x2 / 2x4 grids, f64 and f32."""
    _spawn(W.mkl_summa_worker, world, 2 if world > 2 else 1, el.CPU, W.MKL_SUMMA)


@pytest.mark.parametrize("world", [4, 8])
def test_summa_orientations_match_mkl_reference_path(world):
    """NT / TN / TT through SUMMA_C and TN / NN through SUMMA_DOT on 2x2 and 2x4
    (Device::CPU over gloo) against the reference's loops evaluated rank by rank
    through MKL (tests/golden/mkl_summa_orient.npz; TN.hpp:252-291,371-416,
    NT.hpp:251-294, TT.hpp:195-240, NN.hpp:461-511)."""
    _spawn(W.mkl_summa_worker, world, 2, el.CPU, W.MKL_ORIENT, "mkl_summa_orient.npz")
