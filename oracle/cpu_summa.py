"""CPU SUMMA restatement for bench.py's cpu_baseline leg — TEST INFRASTRUCTURE ONLY.

The default leg is the native oracle/cpu_summa.c (forked ranks, shared-memory
all-gathers, MKL dgemm_ per panel); what follows is the Python restatement over
gloo it replaced, kept as the fallback where MKL is absent.

BASELINE.md §3's planned CPU baseline: BASELINE.json configs[0] (C1),
El::Gemm NN fp64 m=n=k=4096 on a 2x2 grid with Blocksize 128, run the way the
reference's CPU path runs it (SUMMA_NNC, src/blas_like/level3/Gemm/NN.hpp:341-385):
one process per grid rank (column-major grid, Grid.cpp:147-148), element-cyclic
[MC,MR] local blocks (indexing/impl.hpp:33-36,244-245), and per nb-panel

  A1[MC,*]  <- A(:, k:k+nb)   all-gather over the grid row    (RowAllGather)
  B1[*,MR]  <- B(k:k+nb, :)   all-gather over the grid column (the transposed
                                [MR,*] gather of NN.hpp:370-372, untransposed)
  C_loc    += alpha A1 B1     local GEMM

with beta applied to C first (Gemm.cpp:282).  As on the GPU path, the gathered
nb-panels are accumulated into a deeper compute panel (kc = 1024) before the
local update (the summation order changes, not the data moved: cpu_gemm.c is at
half speed on k = 128).  The local GEMM is cpu_gemm.c's
blocked OpenMP dgemm (the role of the reference's MKL call); the gathers are
torch.distributed gloo all-gathers between the processes.  OpenMP threads per
process = cores / ranks.  A few entries of the result are checked against
direct dot products before the timing is reported.
"""
from __future__ import annotations

import ctypes
import os
import socket
import time

import numpy as np


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


MKL_PATH = "/opt/conda/lib/libmkl_rt.so"  # the reference's BLAS in its documented build


def _mkl_gemm(threads: int):
    """dgemm_ of MKL 2021.4 (GNU OpenMP threading layer, as the reference's runs
    require) with `threads` threads, or None when MKL is absent."""
    if not os.path.exists(MKL_PATH):
        return None
    os.environ["MKL_THREADING_LAYER"] = "GNU"
    lib = ctypes.CDLL(MKL_PATH)
    lib.mkl_set_num_threads(ctypes.byref(ctypes.c_int(threads)))
    i = lambda x: ctypes.byref(ctypes.c_int(int(x)))
    d = lambda x: ctypes.byref(ctypes.c_double(x))

    def gemm(m, n, k, alpha, A, lda, B, ldb, beta, C, ldc):
        lib.dgemm_(ctypes.c_char_p(b"N"), ctypes.c_char_p(b"N"), i(m), i(n), i(k), d(alpha), A, i(lda), B, i(ldb),
                   d(beta), C, i(ldc))
    return gemm


def _worker(rank: int, world: int, port: int, r: int, n: int, nb: int, kc: int, seconds: float, threads: int, out,
            blas: str = "port"):
    os.environ["OMP_NUM_THREADS"] = str(threads)  # read by the OpenMP runtime when liboracle loads
    os.environ["OMP_WAIT_POLICY"] = "PASSIVE"     # idle workers must not spin on cores another rank computes on
    import torch
    import torch.distributed as dist

    import oracle

    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    c = world // r
    mc, mr = rank % r, rank // r
    # every rank creates every group, in the same order (gloo new_group is collective)
    rows = [dist.new_group([i + r * j for j in range(c)]) for i in range(r)]
    cols = [dist.new_group([i + r * j for i in range(r)]) for j in range(c)]
    g_row, g_col = rows[mc], cols[mr]
    # [MC,MR] local blocks of the synthetic inputs (Gemm_Suite's Uniform(-0.1, 0.1) shape)
    A = np.asfortranarray(oracle.hash_matrix(n, n, 1, -0.1, 0.1)[mc::r, mr::c])
    B = np.asfortranarray(oracle.hash_matrix(n, n, 2, -0.1, 0.1)[mc::r, mr::c])
    C0 = np.asfortranarray(oracle.hash_matrix(n, n, 3, -0.1, 0.1)[mc::r, mr::c])
    lh, lw = A.shape
    C = C0.copy(order="F")
    L = oracle.lib()
    L.orc_cpu_set_threads(threads)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    mkl = _mkl_gemm(threads) if blas == "mkl" else None
    if mkl is not None:
        kc = nb  # the reference's own structure: one MKL update per Blocksize() panel (NN.hpp:373-384)
    alpha, beta = 0.5, -0.5

    A1 = np.empty((lh, kc), order="F")
    B1 = np.empty((kc, lw), order="F")

    def step():
        np.multiply(C0, beta, out=C)
        for k0 in range(0, n, nb):
            # this rank's columns of A(:, k0:k0+nb) (global j = mr + jl*c) and rows
            # of B(k0:k0+nb, :) (global i = mc + il*r); panels are multiples of r, c
            a_loc = np.ascontiguousarray(A[:, (k0 + c - 1 - mr) // c:(k0 + nb + c - 1 - mr) // c].T)
            b_loc = np.ascontiguousarray(B[(k0 + r - 1 - mc) // r:(k0 + nb + r - 1 - mc) // r, :])
            ga = [torch.empty(a_loc.shape, dtype=torch.float64) for _ in range(c)]
            gb = [torch.empty(b_loc.shape, dtype=torch.float64) for _ in range(r)]
            dist.all_gather(ga, torch.from_numpy(a_loc), group=g_row)
            dist.all_gather(gb, torch.from_numpy(b_loc), group=g_col)
            # interleave into the compute panel: column q of the nb-panel came from
            # grid column (k0 + q) mod c (and row q of B's from grid row (k0 + q) mod r)
            q0 = k0 % kc
            for j in range(c):
                A1[:, q0 + (j - k0) % c:q0 + nb:c] = ga[j].numpy().T
            for i in range(r):
                B1[q0 + (i - k0) % r:q0 + nb:r, :] = gb[i].numpy()
            if q0 + nb == kc or k0 + nb == n:
                kk = q0 + nb
                if mkl is not None:
                    mkl(lh, lw, kk, alpha, p(A1), lh, p(B1), kc, 1.0, p(C), lh)
                else:
                    L.orc_cpu_gemm_f64(b"N", b"N", lh, lw, kk, alpha, p(A1), lh, p(B1), kc, 1.0, p(C), lh)

    step()  # warm-up (thread pool, pages, gloo pairs)
    # correctness of a few entries against direct dot products of the global inputs
    Ag = oracle.hash_matrix(n, n, 1, -0.1, 0.1)
    Bg = oracle.hash_matrix(n, n, 2, -0.1, 0.1)
    Cg = oracle.hash_matrix(n, n, 3, -0.1, 0.1)
    rng = np.random.default_rng(rank)
    for _ in range(8):
        il, jl = int(rng.integers(lh)), int(rng.integers(lw))
        i, j = mc + il * r, mr + jl * c
        want = alpha * float(Ag[i, :] @ Bg[:, j]) + beta * Cg[i, j]
        assert abs(C[il, jl] - want) <= 1e-12, (rank, i, j, C[il, jl], want)
    del Ag, Bg, Cg
    # as many steps as fill `seconds` (decided on rank 0, same count everywhere)
    dist.barrier()
    t0 = time.perf_counter()
    step()
    dist.barrier()
    t1 = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.broadcast(t1, src=0)
    steps = max(2, int(seconds / max(float(t1.item()), 1e-3)))
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        out.put((steps, float(el.item())))
    dist.barrier()
    dist.destroy_process_group()


NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "cpu_summa")


def run_native(n: int, nb: int, r: int, c: int, seconds: float, threads: int) -> dict:
    """oracle/cpu_summa.c: forked ranks, shared-memory all-gathers, one MKL dgemm_
    per nb-panel; returns the cpu_baseline dict with the GEMM / exchange split."""
    import json
    import subprocess
    world = r * c
    p = subprocess.run([NATIVE, str(n), str(nb), str(r), str(c), str(threads), str(seconds), MKL_PATH],
                       capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        raise RuntimeError(f"cpu_summa failed ({p.returncode}): {p.stderr[-2000:]}")
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    return {"value": rec["value"], "unit": "TFLOP/s", "cores": threads * world, "kind": "port",
            "blas": "MKL 2021.4 dgemm_ (the reference's BLAS), AVX-512 kernels",
            "split_s_per_rank": {"dgemm": rec["gemm_s"], "allgather": rec["exchange_s"], "elapsed": rec["elapsed_s"]},
            "sample": f"C1: CPU SUMMA_NNC NN f64 m=n=k={n}, nb={nb} panels, {r}x{c} grid of {world} forked "
                      f"processes x {threads} MKL threads (oracle/cpu_summa.c: shared-memory all-gathers per "
                      f"panel, one MKL 2021.4 dgemm_ per panel, GNU threading layer), {rec['steps']} steps in "
                      f"{rec['elapsed_s']:.1f} s; the reference measured 0.288 s/step (477 GFLOP/s) on 8 cores, "
                      f"BASELINE.md §2"}


def run(n: int = 4096, nb: int = 128, kc: int = 1024, r: int = 2, c: int = 2, seconds: float = 10.0,
        cores: int = 0, blas: str = "auto") -> dict:
    """Time the CPU SUMMA on an r x c grid of processes; returns the cpu_baseline dict.
    blas: "native" oracle/cpu_summa.c (shared-memory exchanges, MKL per nb-panel),
    "mkl" the gloo restatement below with MKL's dgemm_ per nb-panel, "port" the
    gloo restatement over cpu_gemm.c; "auto" native when MKL and the binary are
    present, else port."""
    import torch.multiprocessing as mp

    import oracle
    world = r * c
    cores = cores or oracle.cpu_threads()
    threads = max(1, cores // world)
    if blas == "auto" and os.path.exists(MKL_PATH) and os.path.exists(NATIVE):
        blas = "native"
    if blas == "native":
        return run_native(n, nb, r, c, seconds, threads)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    saved = {v: os.environ.get(v) for v in ("OMP_NUM_THREADS", "OMP_WAIT_POLICY")}
    os.environ["OMP_NUM_THREADS"] = str(threads)  # the children's OpenMP runtime reads it when it loads
    os.environ["OMP_WAIT_POLICY"] = "PASSIVE"
    if blas == "auto":
        blas = "mkl" if os.path.exists(MKL_PATH) else "port"
    try:
        mp.spawn(_worker, args=(world, _port(), r, n, nb, kc, seconds, threads, q, blas), nprocs=world, join=True)
    finally:
        for v, x in saved.items():
            if x is None:
                os.environ.pop(v, None)
            else:
                os.environ[v] = x
    steps, elapsed = q.get()
    return {"value": round(2.0 * n ** 3 * steps / elapsed / 1e12, 4), "unit": "TFLOP/s", "cores": threads * world,
            "kind": "port",
            "blas": "MKL 2021.4 dgemm_ (the reference's BLAS)" if blas == "mkl" else "cpu_gemm.c",
            "sample": f"C1: CPU SUMMA_NNC NN f64 m=n=k={n}, nb={nb} panels gathered, local update every "
                      f"{nb if blas == 'mkl' else kc} columns, {r}x{c} grid of {world} processes x {threads} "
                      f"threads (oracle/cpu_summa.py: gloo all-gathers + "
                      f"{'MKL 2021.4 dgemm_, GNU threading layer' if blas == 'mkl' else 'cpu_gemm.c blocked dgemm'}), "
                      f"{steps} steps in {elapsed:.1f} s; the reference measured 0.288 s/step (477 GFLOP/s) "
                      f"on 8 cores, BASELINE.md §2"}


if __name__ == "__main__":
    import json
    print(json.dumps(run()))
