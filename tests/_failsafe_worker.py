"""Subprocess bodies for the fail-safe tests (tests/test_failsafe_cpu.py and the
GPU RCCL case in tests/test_gpu_dist.py).  Run as
  python tests/_failsafe_worker.py <mode> [args...]
Each mode exits 0 on success; the watchdog modes are expected to be ended by
the library's watchdog with exit status el.WATCHDOG_EXIT."""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def deadline(stage: str, seconds: float, sleep: float):
    from elemental_amd import el
    el.watchdog_stage(stage, seconds)
    time.sleep(sleep)
    print("survived", flush=True)


def disarm(seconds: float, sleep: float):
    from elemental_amd import el
    el.watchdog_stage("armed", seconds)
    el.watchdog_stage("disarmed", 0.0)
    time.sleep(sleep)
    print("survived", flush=True)


def gloo_hang(rank: int, world: int, port: int):
    """Rank 0 enters a 1x2-grid El::Gemm (panel gathers over the host
    collective) under a short stage deadline; rank 1 never joins it."""
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from elemental_amd import el
    from elemental_amd.torch_bridge import GlooBridge
    comm = el.Comm.host(GlooBridge())
    grid = el.Grid(comm, 1)
    mk = lambda h, w, s: el.DistMatrix(grid, el.F64, el.MC, el.MR, el.CPU, height=h, width=w).fill_hash(s, 0.0, 1.0)
    A, B, C = mk(64, 64, 1), mk(64, 64, 2), mk(64, 64, 3)
    dist.barrier()
    if rank == 0:
        el.watchdog_stage("c3 timed", 3.0)
        el.Gemm(el.NORMAL, el.NORMAL, 1.0, A, B, 0.0, C)
        print("gemm returned", flush=True)
    else:
        el.watchdog_stage("straggler", 6.0)
        time.sleep(60)
    print("survived", flush=True)


def rendezvous(rank: int, world: int, port: int):
    from elemental_amd import el
    payload = bytes((7 * i + 3) % 256 for i in range(128)) if rank == 0 else None
    got = el.rendezvous_bcast(payload, 128, rank, world, "127.0.0.1", port, 30.0)
    want = bytes((7 * i + 3) % 256 for i in range(128))
    if got != want:
        print(f"rank {rank}: wrong bytes", flush=True)
        sys.exit(1)
    print(f"rank {rank} ok", flush=True)


def rccl_hang(seconds: float):
    """World-1 RCCL communicator (nonblocking init), then a stage that overruns."""
    from elemental_amd import el
    uid = el.Comm.unique_id()
    comm = el.Comm.rccl(0, 1, uid)
    grid = el.Grid(comm, 1)
    A = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=256, width=256).fill_hash(1, 0.0, 1.0)
    C = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=256, width=256)
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, A, A, 0.0, C)
    el.device_synchronize()
    el.watchdog_stage("rccl stage", seconds)
    time.sleep(60)
    print("survived", flush=True)


def init_env():
    """El::Initialize under a launcher's environment (RANK / WORLD_SIZE set):
    an RCCL world of size 1, a grid over COMM_WORLD, a GEMM on it."""
    import numpy as np
    from elemental_amd import el
    el.Initialize()
    w = el.Comm.world()
    assert w.size == 1 and w.rank == 0
    grid = el.Grid(w)
    A = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=64, width=64).fill_hash(1, 0.0, 1.0)
    C = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=64, width=64)
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, A, A, 0.0, C)
    a = A.get_local()
    assert np.allclose(C.get_local(), a @ a, rtol=1e-12, atol=1e-12)
    assert el.Blocksize() == 128
    el.Finalize()
    print("init ok", flush=True)


if __name__ == "__main__":
    mode, args = sys.argv[1], sys.argv[2:]
    if mode == "deadline":
        deadline(args[0], float(args[1]), float(args[2]))
    elif mode == "disarm":
        disarm(float(args[0]), float(args[1]))
    elif mode == "gloo_hang":
        gloo_hang(int(args[0]), int(args[1]), int(args[2]))
    elif mode == "rendezvous":
        rendezvous(int(args[0]), int(args[1]), int(args[2]))
    elif mode == "init_env":
        init_env()
    elif mode == "rccl_hang":
        rccl_hang(float(args[0]))
    else:
        raise SystemExit(f"unknown mode {mode}")
