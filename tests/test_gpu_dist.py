"""Distributed path on the GPU: DistMatrix redistributions and SUMMA on
Device::GPU matrices.  Multi-rank cases run 2 or 4 processes on the one GPU of
the box with a host-staged (gloo) comm, so the device pack/unpack kernels,
panel pipeline and MFMA updates run for real on every rank."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import _dist_workers as W
import oracle
from elemental_amd import el

pytestmark = pytest.mark.gpu


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


@pytest.mark.parametrize("world,height", [(1, 1), (2, 1), (4, 2)])
def test_gpu_redistribution_bit_exact(world, height):
    _spawn(W.redist_worker, world, height, el.GPU, el.F64, 13, 11, 4321 + world)


def test_gpu_redistribution_bf16_bit_exact():
    _spawn(W.redist_worker, 2, 2, el.GPU, el.BF16, 9, 10, 5)


@pytest.mark.parametrize("world,height", [(1, 1), (2, 2), (4, 2)])
def test_gpu_summa_all_variants(world, height):
    algs = [el.GEMM_DEFAULT, el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT]
    _spawn(W.gemm_worker, world, height, el.GPU, el.F64, [(45, 37, 61), (16, 12, 130)], algs, 16, 3)


@pytest.mark.parametrize("world,height", [(1, 1), (4, 2)])
def test_gpu_cannon(world, height):
    """Cannon_NN on Device::GPU (the reference is CPU-only): skew + ring shifts
    through Comm::SendRecv, local MFMA updates, random alignments."""
    _spawn(W.cannon_worker, world, height, el.GPU, el.F64, [(45, 37, 62), (16, 12, 130)], 5)


@pytest.mark.parametrize("world,height", [(1, 1), (4, 2)])
def test_gpu_uniform_reference_draws(world, height):
    _spawn(W.uniform_worker, world, height, el.GPU)


def test_gpu_summa_f32():
    _spawn(W.gemm_worker, 2, 1, el.GPU, el.F32, [(65, 33, 97)], [el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT], 8, 9)


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2), (8, 2)])
def test_gpu_blas1_distributed(world, height):
    _spawn(W.blas1_worker, world, height, el.GPU, 17)


@pytest.mark.parametrize("dtype,world,height", [(el.F16, 2, 1), (el.BF16, 4, 2), (el.BF16, 1, 1)])
def test_gpu_summa_16bit(dtype, world, height):
    """C5: distributed 16-bit El::Gemm on DistMatrix[MC,MR] (MFMA f32 accumulate)
    through every SUMMA variant, against the exact product (eps 2^-11 / 2^-8)."""
    algs = [el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT]
    _spawn(W.gemm_worker, world, height, el.GPU, dtype, [(45, 37, 61)], algs, 16, 31)


@pytest.mark.parametrize("dtype", [el.F64, el.F32])
def test_gpu_summa_grid_2x4(dtype):
    """C3's 2x4 grid (8 host-staged ranks on the one device)."""
    algs = [el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT] if dtype == el.F64 \
        else [el.GEMM_SUMMA_C]
    _spawn(W.gemm_worker, 8, 2, el.GPU, dtype, [(45, 37, 61)], algs, 8, 37)


@pytest.mark.parametrize("world,height", [(2, 1), (4, 2)])
def test_gpu_summa_multi_panel_distributed(world, height):
    """k = 130 with 16-column compute panels: nine panels through the two GPU
    slots on 1x2 and 2x2 grids; each slot is regathered on the comm stream while
    the previous MFMA update reads the other (the slot's `done` event fence)."""
    _spawn(W.gemm_worker, world, height, el.GPU, el.F64, [(45, 37, 130)], [el.GEMM_SUMMA_C], 16, 43, 16)


@pytest.mark.parametrize("world,height", [(2, 1), (8, 2)])
def test_gpu_summa_first_panel_ramp(world, height):
    """Compute panel 64 = 4 x nb on a grid larger than 1x1: the panels ramp up
    16, 32, then 64 columns (k = 130: 16, 32, 64, 18; k = 80: 16, 32, 32)."""
    _spawn(W.gemm_worker, world, height, el.GPU, el.F64, [(45, 37, 130), (33, 20, 80)], [el.GEMM_SUMMA_C], 16, 53,
           64)


@pytest.mark.parametrize("world,height,pool", [(1, 1, 2), (2, 1, 3), (4, 2, 2)])
def test_gpu_summa_multistream(world, height, pool):
    """GEMM_SUMMA_{A,B,C}_MS with a stream pool (H_STREAMPOOL_SIZE = pool):
    panels round-robin over teams with their own streams (and per-team C copies
    for C_MS, summed at the end, NN_Multistream.hpp:340-411) for NN, NT and TN;
    GEMM_DEFAULT picks the _MS variants; TT rejects them (TT.hpp:410-433).
    k = 130 with 16-column panels: nine C_MS panels over the teams."""
    algs = [el.GEMM_DEFAULT, el.GEMM_SUMMA_A_MS, el.GEMM_SUMMA_B_MS, el.GEMM_SUMMA_C_MS]
    _spawn(W.gemm_worker, world, height, el.GPU, el.F64, [(45, 37, 130), (16, 12, 70)], algs, 16, 59, 16, pool)


def test_gpu_syrk_multi_panel_distributed():
    _spawn(W.syrk_worker, 4, 2, el.GPU, el.F64, [(45, 70)], 16, 47, 16)


@pytest.mark.parametrize("world,height", [(1, 1), (2, 1)])
def test_gpu_cross_device_copies_and_mixed_operands(world, height):
    """CPU <-> GPU DistMatrix copies both ways across distributions, bit-exact;
    Gemm / Trsm with operands on different devices (proxied to C's / X's)."""
    _spawn(W.xdevice_worker, world, height, 53)


def test_gpu_operands_on_other_streams():
    """A and B on caller streams other than C's: the Level-3 drivers fence C's
    stream after A's/B's queued work on entry and A's/B's after theirs on exit
    (MultiSync, include/hydrogen/MultiSync.hpp:33-78), so A can be refilled on its
    own stream right after the call without disturbing the product."""
    import torch
    m, n, k = 300, 257, 411
    g = el.Grid()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    Ah, Bh, Ch = oracle.hash_matrix(m, k, 1), oracle.hash_matrix(k, n, 2), oracle.hash_matrix(m, n, 3)
    for alg in (el.GEMM_SUMMA_C, el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_DOT):
        A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=k)
        B = el.DistMatrix(g, el.F64, el.VC, el.STAR, el.GPU, height=k, width=n)
        C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=n)
        A.set_stream(sa.cuda_stream)
        B.set_stream(sb.cuda_stream)
        A.fill_hash(1, 0.0, 1.0)   # queued on A's stream
        B.fill_hash(2, 0.0, 1.0)   # queued on B's stream
        C.set_local(Ch)
        el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C, alg)
        A.fill_hash(9, 5.0, 1.0)   # overwrite A on its own stream at once
        el.device_synchronize()
        want = oracle.gemm("N", "N", 0.5, Ah, Bh, -0.5, Ch)
        assert oracle.parity_ratio(C.get_local(), want, Ah, Bh, k, np.finfo(np.float64).eps) <= 10, alg


def test_gpu_el_api_cpp():
    """The drop-in C++ header on Device::GPU matrices (tests/cpp/test_el_api.cpp
    built with -DEL_TEST_GPU): Gemm, Matrix<T,GPU>/LockedMatrix Gemm, Syrk/Herk,
    Trsm (+ checkIfSingular), redistributions, Get/Set, Fill, level-1, Attach,
    Write/Read."""
    _run_prebuilt("test_el_api_gpu")


def _run_prebuilt(name: str):
    """Run a C++ program __graft_entry__.build() compiled into tests/cpp/_build."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "_build", name)
    assert os.path.exists(exe), f"{exe} missing: run __graft_entry__.build()"
    res = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "OK" in res.stdout


def test_gpu_entrywise_functor():
    """Functor-generic El::EntrywiseMap / El::Combine (include/El/EntrywiseMap.hip.hpp,
    the reference's EntrywiseMapImpl / CombineImpl device templates) with user
    device lambdas and a functor struct, compiled by hipcc as a caller would."""
    _run_prebuilt("test_entrywise_functor")


def test_gpu_summa_pipeline_multi_panel():
    """1x1 grid, compute panel < k: several pipelined panels over two slots."""
    m, n, k = 700, 513, 900
    g = el.Grid()
    el.SetBlocksize(128)
    el.SetComputePanel(256)
    try:
        A = el.DistMatrix(g, el.F64, height=m, width=k).fill_hash(1, -0.1, 0.1)
        B = el.DistMatrix(g, el.F64, height=k, width=n).fill_hash(2, -0.1, 0.1)
        C = el.DistMatrix(g, el.F64, height=m, width=n).fill_hash(3, -0.1, 0.1)
        el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C, el.GEMM_SUMMA_C)
        got = C.get_local()
    finally:
        el.SetComputePanel(0)
    Ag, Bg, Cg = (oracle.hash_matrix(*s, seed, -0.1, 0.1) for s, seed in (((m, k), 1), ((k, n), 2), ((m, n), 3)))
    ref = oracle.gemm("N", "N", 0.5, Ag, Bg, -0.5, Cg)
    assert oracle.parity_ratio(got, ref, Ag, Bg, k, np.finfo(np.float64).eps) <= 10


_COPIED_PANELS = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import oracle
from elemental_amd import el
m, n, k = 1300, 1100, 2100
g = el.Grid()
el.SetBlocksize(128)
el.SetComputePanel(256)
for oA in (el.NORMAL, el.TRANSPOSE):
    for oB in (el.NORMAL, el.TRANSPOSE):
        sa = (m, k) if oA == el.NORMAL else (k, m)
        sb = (k, n) if oB == el.NORMAL else (n, k)
        A = el.DistMatrix(g, el.F64, height=sa[0], width=sa[1]).fill_hash(1, -0.1, 0.1)
        B = el.DistMatrix(g, el.F64, height=sb[0], width=sb[1]).fill_hash(2, -0.1, 0.1)
        C = el.DistMatrix(g, el.F64, height=m, width=n).fill_hash(3, -0.1, 0.1)
        el.Gemm(oA, oB, 0.5, A, B, -0.5, C, el.GEMM_SUMMA_C)
        got = C.get_local()
        Ag, Bg, Cg = (oracle.hash_matrix(*sh, seed, -0.1, 0.1) for sh, seed in ((sa, 1), (sb, 2), ((m, n), 3)))
        ref = oracle.gemm("NT"[oA], "NT"[oB], 0.5, Ag, Bg, -0.5, Cg)
        r = oracle.parity_ratio(got, ref, Ag, Bg, k, np.finfo(np.float64).eps)
        assert r <= 10, (oA, oB, r)
print("ok")
"""


def test_gpu_summa_pipeline_copied_panels():
    """ELX_SUMMA_COPY=1 (a child process: the knob is read once): every panel of
    a 1x1 SUMMA_C is COPIED into the two slots on the comm stream while the MFMA
    kernels read the other slot - the N > 1 pipeline's stream pattern and
    write-after-read fences with the LDS-DMA kernels at full tile counts
    (9 panels of 256, all four orientations), against the oracle."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ELX_SUMMA_COPY="1")
    out = subprocess.run([sys.executable, "-c", _COPIED_PANELS, root], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0 and "ok" in out.stdout, out.stdout + out.stderr


@pytest.mark.parametrize("oA,oB", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gpu_gemm_associativity_large(oA, oB):
    """tests/blas_like/Gemm.cpp:15-49 at n = 4096 fp64 (size-independent check):
    ||(alpha op(A)op(B) + beta C) X - C_final X||_F / ||Y||_F."""
    n = 4096
    g = el.Grid()
    A = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(5, -0.1, 0.1)
    B = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(6, -0.1, 0.1)
    C = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(7, -0.1, 0.1)
    el.Gemm(oA, oB, 0.5, A, B, -0.5, C)
    Cf = C.get_local()
    Ag, Bg, Cg = (oracle.hash_matrix(n, n, s, -0.1, 0.1) for s in (5, 6, 7))
    X = oracle.hash_matrix(n, 100, 8, 0.0, 1.0)
    opA = Ag if oA == 0 else Ag.T
    opB = Bg if oB == 0 else Bg.T
    Y = 0.5 * (opA @ (opB @ X)) - 0.5 * (Cg @ X)
    E = Y - Cf @ X
    res = np.linalg.norm(E) / np.linalg.norm(Y)
    assert res < 1e-13, res  # reference measured 2.3e-16 at 4096


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gpu_summa_matches_mkl_reference_path(world):
    """GPU SUMMA_C (host-staged panels, MFMA local updates) against the
    reference CPU path's SUMMA_NNC evaluated through MKL rank by rank
    (tests/golden/mkl_summa.npz): 1x2 / 2x2 / 2x4, f64 and f32, north_star bound."""
    _spawn(W.mkl_summa_worker, world, 2 if world > 2 else 1, el.GPU, W.MKL_SUMMA)
    if world > 2:
        _spawn(W.mkl_summa_worker, world, 2, el.GPU, W.MKL_ORIENT, "mkl_summa_orient.npz")


def test_gpu_summa_matches_mkl_at_c1_size():
    """C1 at its own size (El::Gemm NN f64 4096^3 on a 2x2 grid, Blocksize 128)
    on the GPU path (MFMA updates, host-staged panels) against the reference's
    SUMMA_NNC through MKL rank by rank: a 111 x 100 sample of the result
    (tests/golden/mkl_summa_orient.npz), normwise and entrywise."""
    _spawn(W.mkl_summa_worker, 4, 2, el.GPU, W.MKL_C1, "mkl_summa_orient.npz")


def _rccl_spawn(fn, world, *args):
    import os
    os.environ["ELX_TEST_BACKEND"] = "rccl"
    try:
        _spawn(fn, world, *args)
    finally:
        os.environ.pop("ELX_TEST_BACKEND", None)


def test_gpu_rccl_single_rank_redistribution_and_summa():
    """The RCCL backend end to end at world size 1 (init, the four grid
    splits, the self-copy paths) - the only RCCL shape a 1-GPU box can run."""
    _rccl_spawn(W.redist_worker, 1, 1, el.GPU, el.F64, 13, 11, 77)
    _rccl_spawn(W.gemm_worker, 1, 1, el.GPU, el.F64, [(45, 37, 61)], [el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT], 16, 5)
    # multistream teams over RCCL: each team's grid is a split duplicate of the world
    _rccl_spawn(W.gemm_worker, 1, 1, el.GPU, el.F64, [(45, 37, 61)],
                [el.GEMM_SUMMA_C_MS, el.GEMM_SUMMA_A_MS, el.GEMM_DEFAULT], 16, 7, 16, 3)
    # the raw El::mpi collectives of the C-ABI (incl. Split, Bcast, AllToAll, SendRecv) on device buffers
    _rccl_spawn(W.raw_coll_worker, 1)


def _failsafe(*args, env=None, timeout=120):
    import os
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_failsafe_worker.py")
    full = dict(os.environ, **(env or {}))
    return subprocess.run([sys.executable, worker, *map(str, args)], capture_output=True, text=True,
                          timeout=timeout, env=full)


def test_gpu_rccl_watchdog_aborts_overrunning_stage():
    """World-1 RCCL (init and the four grid splits),
    a GEMM over it, then a stage that overruns its deadline: the watchdog aborts
    the RCCL communicators and exits with ELX_WATCHDOG_EXIT naming the stage."""
    p = _failsafe("rccl_hang", 2.0)
    assert p.returncode == el.WATCHDOG_EXIT, p.stdout + p.stderr
    assert "FATAL in stage 'rccl stage'" in p.stderr and "RCCL communicator(s)" in p.stderr
    assert "aborting 0 RCCL" not in p.stderr
    assert "survived" not in p.stdout


def test_gpu_initialize_rccl_world_from_launcher_env():
    """El::Initialize under torch.distributed.run's variables builds COMM_WORLD
    over RCCL (unique id through the TCP rendezvous; size 1 on this box)."""
    port = _port()
    p = _failsafe("init_env", env={"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0",
                                   "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    assert p.returncode == 0, p.stdout + p.stderr
    assert "init ok" in p.stdout


@pytest.mark.parametrize("hang,line", [("timed", False), ("cpu_baseline", True)])
def test_gpu_bench_stage_hang(hang, line):
    """bench.py under an injected hang (ELX_BENCH_HANG): the watchdog ends the
    run with ELX_WATCHDOG_EXIT naming the stage.  In the timed stage no line is
    printed; in a stage after the main point the line is still printed, with
    that stage marked and an "incomplete" field, and the exit status is STILL
    non-zero, so a hang in an optional stage never reads as success."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--n", "2048", "--steps", "1",
                        "--warmup", "1"], capture_output=True, text=True, timeout=200,
                       env=dict(os.environ, ELX_BENCH_HANG=hang))
    assert p.returncode == el.WATCHDOG_EXIT, p.stdout + p.stderr
    assert f"FATAL in stage '{hang}'" in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if not line:
        assert not lines
    else:
        assert len(lines) == 1 and p.stdout.strip() == lines[0], p.stdout  # stdout holds the line only
        rec = json.loads(lines[0])
        assert rec["value"] > 0 and rec["verify"]["ok"] and "error" in rec[hang] and "incomplete" in rec


def test_gpu_bench_launches_its_own_ranks():
    """`python3 bench.py --gpus 2` with no launcher (WORLD_SIZE unset): the script
    starts its two rank processes itself (bench.launch_ranks) and the caller reads
    exactly one line on stdout, the complete N = 2 line (host-staged panels, both
    ranks on this box's one GPU: ELX_BENCH_COMM=host), with the residual checked
    on its own grid and exit status 0."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ELX_BENCH_COMM"] = "host"
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--size", "2048", "--steps", "1",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stdout + p.stderr[-4000:]
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["grid"] == "1x2" and rec["value"] > 0
    assert rec["residual"]["ok"] and rec["verify"]["ok"]
    assert "collectives" in rec and "c4" not in rec and "c5" not in rec  # N > 1 default: C3 + residual only


def _need_gpus(world):
    return pytest.mark.skipif(el.device_count() < world, reason=f"needs >= {world} GPUs (one RCCL rank per GPU)")


# C3's grids: 1x2, 2x2, 2x4 (Grid::DefaultHeight), one RCCL rank per GPU; each
# case runs only where the box has that many GPUs (the driver's 8-GPU node)
@pytest.mark.parametrize("world,height", [pytest.param(2, 1, marks=_need_gpus(2)),
                                          pytest.param(4, 2, marks=_need_gpus(4)),
                                          pytest.param(8, 2, marks=_need_gpus(8))])
def test_gpu_rccl_multi_gpu(world, height):
    """RCCL at world > 1 against the oracle: every redistribution pair (the
    grouped send/recv over VC), SUMMA A / B / C / Dot in all orientations
    (AxpyContract's ncclReduceScatter over MC / MR / VC), several panels
    through the two-slot pipeline with the CopyGroup exchange (A and B gathered
    in ONE RCCL group), the multistream teams (ncclCommSplit duplicates), f32
    TN Dot (C4's shape family), bf16 SUMMA (C5), the raw and typed El::mpi
    collectives on device and host buffers."""
    _rccl_spawn(W.redist_worker, world, height, el.GPU, el.F64, 13, 11, 99)
    _rccl_spawn(W.redist_worker, world, height, el.GPU, el.BF16, 9, 10, 5)
    algs = [el.GEMM_SUMMA_A, el.GEMM_SUMMA_B, el.GEMM_SUMMA_C, el.GEMM_SUMMA_DOT]
    _rccl_spawn(W.gemm_worker, world, height, el.GPU, el.F64, [(45, 37, 61)], algs, 16, 6)
    _rccl_spawn(W.gemm_worker, world, height, el.GPU, el.F64, [(45, 37, 130)],
                [el.GEMM_SUMMA_C, el.GEMM_SUMMA_C_MS, el.GEMM_SUMMA_A_MS], 16, 8, 16, 2)
    _rccl_spawn(W.gemm_worker, world, height, el.GPU, el.F32, [(40, 24, 300)], [el.GEMM_SUMMA_DOT], 16, 9)
    _rccl_spawn(W.gemm_worker, world, height, el.GPU, el.BF16, [(64, 48, 96)], [el.GEMM_SUMMA_C], 16, 10, 32)
    _rccl_spawn(W.raw_coll_worker, world)
    _rccl_spawn(W.mpi_typed_worker, world, el.GPU)
    _rccl_spawn(W.mpi_typed_worker, world, el.CPU)


@pytest.mark.parametrize("world,height", [(1, 1), (2, 1), (4, 2)])
def test_gpu_frobenius_norm(world, height):
    """El::FrobeniusNorm on device matrices (norm_partial_kernel + grid
    reductions) against numpy: f64 / f32 / f16 / bf16, ragged, replicated
    distributions, NaN / inf / near-overflow (the bench's verify divides two)."""
    _spawn(W.frobenius_worker, world, height, el.GPU)


def test_gpu_mpi_typed_collectives():
    """elx_mpi_* (El::mpi::* on SyncInfo<Device::GPU> / <Device::CPU>): the
    world-1 RCCL communicator (device buffers, and host buffers staged through
    device memory), and 1/2/4 host-staged processes on the one device."""
    _rccl_spawn(W.mpi_typed_worker, 1, el.GPU)
    _rccl_spawn(W.mpi_typed_worker, 1, el.CPU)
    for world in (2, 4):
        _spawn(W.mpi_typed_worker, world, el.GPU)


def test_gpu_attach_torch_storage():
    """ElementalMatrix::Attach on device memory owned by the caller (a torch
    tensor): El::Gemm writes into it in place, padding rows untouched."""
    import torch
    m, n, k = 300, 200, 170
    g = el.Grid()
    Ah, Bh = oracle.hash_matrix(m, k, 1), oracle.hash_matrix(k, n, 2)
    # column-major (ld x cols) == row-major (cols x ld) tensor
    At = torch.from_numpy(np.ascontiguousarray(Ah.T)).cuda()
    Bt = torch.from_numpy(np.ascontiguousarray(Bh.T)).cuda()
    Ct = torch.full((n, m + 4), 3.0, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU).attach(m, k, 0, 0, At.data_ptr(), m)
    B = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU).attach(k, n, 0, 0, Bt.data_ptr(), k)
    C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU).attach(m, n, 0, 0, Ct.data_ptr(), m + 4)
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, A, B, 0.0, C)
    el.device_synchronize()
    got = Ct.cpu().numpy().T
    want = oracle.gemm("N", "N", 1.0, Ah, Bh, 0.0, np.zeros((m, n), order="F"))
    assert oracle.parity_ratio(got[:m], want, Ah, Bh, k, np.finfo(np.float64).eps) <= 10
    assert (got[m:] == 3.0).all()


@pytest.mark.parametrize("world,height", [(1, 1), (2, 1)])
def test_gpu_write_read_binary(world, height, tmp_path):
    _spawn(W.io_worker, world, height, el.GPU, str(tmp_path))


def test_gpu_set_stream():
    """El::SetSyncInfo / SyncInfoFromMatrix: a matrix moved to a caller stream
    runs its work there, ordered after what was queued on its old stream."""
    import torch
    m, n, k = 257, 190, 300
    g = el.Grid()
    A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=k)
    B = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=k, width=n)
    C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=n)
    A.fill_hash(1, 0.0, 1.0)
    B.fill_hash(2, 0.0, 1.0)
    C.fill_hash(3, 0.0, 1.0)
    lib_stream = C.stream()
    s = torch.cuda.Stream()
    for M in (A, B, C):
        M.set_stream(s.cuda_stream)
        assert M.stream() == s.cuda_stream
    el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)
    s.synchronize()
    Ah, Bh, Ch = oracle.hash_matrix(m, k, 1), oracle.hash_matrix(k, n, 2), oracle.hash_matrix(m, n, 3)
    want = oracle.gemm("N", "N", 0.5, Ah, Bh, -0.5, Ch)
    assert oracle.parity_ratio(C.get_local(), want, Ah, Bh, k, np.finfo(np.float64).eps) <= 10
    C.set_stream(None)  # back to the library's compute stream
    assert C.stream() == lib_stream
    el.device_synchronize()


@pytest.mark.parametrize("world,height", [(1, 1), (2, 2)])
def test_gpu_copy_type_conversion(world, height):
    """El::Copy between element types on GPU matrices (convert2d_kernel), bit-exact."""
    _spawn(W.convert_worker, world, height, el.GPU, 8)


@pytest.mark.parametrize("world,height,cols", [(1, 1, 0), (2, 1, 0), (4, 2, 3)])
def test_gpu_syrk_distributed(world, height, cols, monkeypatch):
    """El::Syrk / El::Herk LN/LT/UN/UT through the GPU pipeline and the trapezoid
    kernel (host-staged ranks on one device); cols > 0: many ragged column blocks."""
    if cols:
        monkeypatch.setenv("ELX_TRRK_COLS", str(cols))
        monkeypatch.setenv("ELX_TRRK_ROWS", "2")
    _spawn(W.syrk_worker, world, height, el.GPU, el.F64, [(45, 19), (16, 70)], 16, 21)


@pytest.mark.parametrize("dtype", [el.F64, el.F32])
def test_gpu_syrk_large(dtype):
    """1x1 grid, n = 2500 (five 512-column blocks, a ragged last one), k = 640:
    every uplo x orientation against a float64 numpy product, the other triangle
    bit-identical to its input."""
    n, k = 2500, 640
    npdt = np.float64 if dtype == el.F64 else np.float32
    eps = np.finfo(npdt).eps
    g = el.Grid()
    i, j = np.indices((n, n))
    for uplo in (el.LOWER, el.UPPER):
        for orient in (el.NORMAL, el.TRANSPOSE):
            shape = (n, k) if orient == el.NORMAL else (k, n)
            A = el.DistMatrix(g, dtype, height=shape[0], width=shape[1]).fill_hash(11, -0.1, 0.1)
            C = el.DistMatrix(g, dtype, height=n, width=n).fill_hash(12, -0.1, 0.1)
            el.Syrk(uplo, orient, 0.5, A, -0.5, C)
            got = C.get_local()
            Ag = oracle.hash_matrix(*shape, 11, -0.1, 0.1, npdt).astype(np.float64)
            Cg = oracle.hash_matrix(n, n, 12, -0.1, 0.1, npdt)
            P = Ag @ Ag.T if orient == el.NORMAL else Ag.T @ Ag
            inside = (i >= j) if uplo == el.LOWER else (i <= j)
            assert np.array_equal(got[~inside], Cg[~inside])
            ref = 0.5 * P - 0.5 * Cg.astype(np.float64)
            num = np.linalg.norm((got.astype(np.float64) - ref)[inside])
            den = np.linalg.norm(Ag) ** 2 * k * eps
            assert num <= 10 * den, (uplo, orient, num / den)


@pytest.mark.parametrize("world,height,flat", [(1, 1, 0), (2, 1, 0), (4, 2, 0), (4, 2, 1)])
def test_gpu_trsm_distributed(world, height, flat, monkeypatch):
    """El::Trsm, all 16 side/uplo/orientation/diag cases, on the GPU (trsm_kernel +
    the SUMMA trailing update), host-staged ranks on one device; flat = 1 the
    reference's nb-step sweep instead of the recursive split."""
    if flat:
        monkeypatch.setenv("ELX_TRSM_FLAT", "1")
    _spawn(W.trsm_worker, world, height, el.GPU, el.F64, 45, 23, 16, 41)


@pytest.mark.parametrize("dtype", [el.F64, el.F32])
@pytest.mark.parametrize("m,n", [(1500, 700), (2100, 1100)])
def test_gpu_trsm_large(dtype, m, n):
    """1x1 grid, m = 1500 (12 blocks of 128, a ragged last one), 700 right-hand
    sides; m = 2100, 1100 right-hand sides takes the 256-row diagonal blocks of
    the batched path (ragged last block): LEFT LOWER and UPPER, NORMAL and
    TRANSPOSE, against oracle.trsm."""
    npdt = np.float64 if dtype == el.F64 else np.float32
    g = el.Grid()
    el.SetBlocksize(128)
    Ag = oracle.hash_matrix(m, m, 51, 0.0, 0.05, npdt)
    Ag[np.diag_indices(m)] += npdt(2.0)
    Bg = oracle.hash_matrix(m, n, 52, -1.0, 1.0, npdt)
    for uplo in (el.LOWER, el.UPPER):
        for orient in (el.NORMAL, el.TRANSPOSE):
            A = el.DistMatrix(g, dtype, height=m, width=m)
            B = el.DistMatrix(g, dtype, height=m, width=n)
            A.set_local(Ag)
            B.set_local(Bg)
            el.Trsm(el.LEFT, uplo, orient, el.NON_UNIT, 1.0, A, B)
            got = B.get_local().astype(np.float64)
            ref = oracle.trsm("L", "LU"[uplo], "NT"[orient], "N", 1.0, Ag, Bg)
            err = np.linalg.norm(got - ref) / (np.linalg.norm(ref) * m * np.finfo(npdt).eps)
            assert err <= 10, (uplo, orient, err)


@pytest.mark.parametrize("world,height", [(1, 1), (2, 1), (4, 2)])
def test_gpu_symm_distributed(world, height):
    """El::Symm / El::Hemm on the GPU (trapezoid copy + SUMMA), host-staged ranks."""
    _spawn(W.symm_worker, world, height, el.GPU, el.F64, 45, 29, 61)


@pytest.mark.parametrize("cache", [None, "0"])
def test_gpu_gemm_suite_driver(tmp_path, cache):
    """The reference suite's experiment files run unchanged through the drop-in
    header on Device::GPU (tests/cpp/gemm_suite.cpp): every algorithm id,
    double / float / half / bfloat16, warm-up associativity residuals enforced
    (--check), one results line per experiment in the suite's format.  Also with
    the allocator's cache off (ELX_POOL_CACHE=0: every block returns to the
    driver at its free), where round 4 saw wrong products on the second warm-up
    (DESIGN.md section 2)."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "_build", "gemm_suite")
    assert os.path.exists(exe), f"{exe} missing: run __graft_entry__.build()"
    algs = ["DEFAULT", "SUMMA_A", "SUMMA_B", "SUMMA_C", "SUMMA_DOT", "SUMMA_A_MS", "SUMMA_C_MS", "CANNON"]
    lines = [f"GPU:Double:N:N:{a}:300:260:520:64" for a in algs]
    lines += ["GPU:Double:T:N:SUMMA_C:257:129:700:128", "GPU:Float:N:T:SUMMA_C:512:384:640:128",
              "GPU:Half:N:N:SUMMA_C:512:512:1024:128", "GPU:Bfloat:T:N:SUMMA_C:512:256:512:128",
              "GPU:Double:T:T:SUMMA_DOT:64:64:20000:128"]
    exp = tmp_path / "exp.txt"
    exp.write_text("\n".join(lines) + "\n")
    res = tmp_path / "res.txt"
    env = dict(os.environ)
    if cache is not None:
        env["ELX_POOL_CACHE"] = cache
    r = subprocess.run([exe, "--f", str(exp), "--o", str(res), "--warmup", "3" if cache else "2", "--runs", "3",
                        "--check"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    out = res.read_text().splitlines()
    assert len(out) == len(lines) and all(ln.startswith("GPU:") and len(ln.split(":")) == 12 for ln in out)
