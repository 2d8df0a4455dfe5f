#!/usr/bin/env python3
"""Headline benchmark: distributed El::Gemm TFLOP/s on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W
  (N > 1: launched by torch.distributed.run, one process per GPU; RANK /
   LOCAL_RANK / WORLD_SIZE / MASTER_* come from the environment)

One step = one El::Gemm(NORMAL, NORMAL, alpha=0.5, A, B, beta=-0.5, C) on
DistMatrix<double,MC,MR,ELEMENT,GPU> operands already resident in HBM,
inputs Uniform(-0.1, 0.1) as tests/blas_like/Gemm_Suite.cpp:158-172 (from the
grid-independent counter hash, synthetic data).  The whole SUMMA runs inside
the timed region: Scale(beta, C), every panel redistribution over RCCL, every
MFMA update.
  N = 1 : config C2, m=n=k=32768 on a 1x1 grid (BASELINE.json configs[1]).
  N > 1 : config C3, m=n=k=65536 on Grid::DefaultHeight(N) (1x2, 2x2, 2x4):
          strong scaling of the same problem.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}  # MI355X dense MFMA, datasheet (MI355X_MICROARCH.md / SURVEY §6)


def cpu_baseline(seconds_target: float = 15.0) -> dict:
    """The oracle's CPU GEMM (oracle/oracle.c, the reference's loop nest), single
    thread, on a bounded sample of the same workload: an NN fp64 GEMM of
    s x s x s with the same input distribution, s grown until ~seconds_target."""
    import numpy as np
    import oracle
    s, t = 256, 0.0
    while True:
        A = oracle.hash_matrix(s, s, 1, 0.0, 0.1)
        B = oracle.hash_matrix(s, s, 2, 0.0, 0.1)
        C = oracle.hash_matrix(s, s, 3, 0.0, 0.1)
        t0 = time.perf_counter()
        oracle.gemm("N", "N", 0.5, A, B, -0.5, C)
        t = time.perf_counter() - t0
        if t * 8 > seconds_target or s >= 4096:
            break
        s *= 2
    reps, total = 1, t
    while total < 10.0:  # about 10-30 s of CPU work in all
        t0 = time.perf_counter()
        oracle.gemm("N", "N", 0.5, A, B, -0.5, C)
        total += time.perf_counter() - t0
        reps += 1
    return {"value": 2.0 * s ** 3 * reps / total / 1e12, "unit": "TFLOP/s", "cores": 1, "kind": "port",
            "sample": f"oracle C GEMM NN fp64 {s}x{s}x{s} x{reps}, 1 thread, {total:.2f} s"}


def measured_traffic(dtype: str, n: int, world: int):
    """Per-launch HBM bytes of the GEMM kernel from the committed rocprofv3 PMC
    passes of this same bench command (tools/collect_profiles.sh ->
    profiles/traffic_index.json), or None when that configuration was not profiled."""
    path = os.path.join(ROOT, "profiles", "traffic_index.json")
    if not os.path.exists(path):
        return None
    ent = json.load(open(path)).get(f"{dtype}:{n}:{world}")
    return ent["hbm_bytes_per_launch"] if ent else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=0, help="override m=n=k")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--nb", type=int, default=128, help="El::Blocksize (communication panel)")
    ap.add_argument("--kc", type=int, default=0, help="compute panel (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    from elemental_amd import el
    from elemental_amd import _lib as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    L.call("elx_set_device", local)
    torch.cuda.set_device(local)

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only (uid, barrier, max); data goes over RCCL
        obj = [el.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = el.Comm.rccl(rank, world, obj[0])
    else:
        comm = el.Comm.self_comm()
    grid = el.Grid(comm, 0)
    n = args.n or (32768 if world == 1 else 65536)
    dt = el.F64 if args.dtype == "f64" else el.F32
    el.SetBlocksize(args.nb)
    el.SetComputePanel(args.kc)

    A = el.DistMatrix(grid, dt, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(1, 0.0, 0.1)
    B = el.DistMatrix(grid, dt, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(2, 0.0, 0.1)
    C = el.DistMatrix(grid, dt, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(3, 0.0, 0.1)

    def barrier():
        el.device_synchronize()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    def step():
        return el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)

    for _ in range(args.warmup):
        step()
    barrier()
    L.call("elx_set_profiling", 1)
    el.comm_stats_reset()
    barrier()
    t0 = time.perf_counter()
    alg = el.GEMM_DEFAULT
    for _ in range(args.steps):
        alg = step()
    barrier()
    elapsed = time.perf_counter() - t0

    import ctypes
    gemm_ms, launches, flops = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    comm_ms, comm_bytes = ctypes.c_double(), ctypes.c_int64()
    L.call("elx_profile_stats", ctypes.byref(gemm_ms), ctypes.byref(launches), ctypes.byref(flops),
           ctypes.byref(comm_ms), ctypes.byref(comm_bytes))
    L.call("elx_set_profiling", 0)

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_flops = 2.0 * n * n * n * args.steps
    value = total_flops / elapsed / 1e12
    avg_ms = gemm_ms.value / max(launches.value, 1)
    flops_per_launch = flops.value / max(launches.value, 1)
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    peak = PEAK_TFLOPS[args.dtype]
    out = {
        "metric": "distributed Gemm TFLOP/s (fp64/fp32) at 1/2/4/8 GPUs; % of MFMA peak",
        "value": round(value, 3),
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (grid-independent hash, Uniform(-0.1,0.1)); alpha=0.5, beta=-0.5",
        "config": {
            "workload": ("C2: El::Gemm NN fp64 m=n=k=32768, Grid 1x1" if world == 1 and n == 32768 else
                         f"C3: SUMMA El::Gemm NN {args.dtype} m=n=k={n}, Grid {grid.height}x{grid.width}"),
            "m": n, "n": n, "k": n,
            "grid": f"{grid.height}x{grid.width}",
            "algorithm": {2: "SUMMA_A", 4: "SUMMA_B", 6: "SUMMA_C", 7: "SUMMA_DOT"}.get(alg, str(alg)),
            "blocksize": args.nb,
            "compute_panel": args.kc or "auto",
            "parallelism": f"grid{grid.height}x{grid.width}",
        },
        "pct_of_mfma_peak": round(100.0 * value / (peak * world), 2),
        "roofline": {
            "bound": "mfma",
            "kernel": f"gemm_tile_kernel<{'double' if args.dtype == 'f64' else 'float'}> (local panel update)",
            "achieved": round(achieved, 3),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": measured_traffic(args.dtype, n, world),
            "traffic_unit": "bytes/launch (PMC FETCH_SIZE*2 + WRITE_SIZE)",
            "launches_timed": launches.value,
            "avg_launch_ms": round(avg_ms, 3),
            "flops_per_launch": flops_per_launch,
        },
        "collectives": {
            "bytes_per_rank": comm_bytes.value,
            "transfer_ms_per_rank": round(comm_ms.value, 3),
            "GB_per_s": round(comm_bytes.value / (comm_ms.value * 1e-3) / 1e9, 2) if comm_ms.value > 0 else None,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
