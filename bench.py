#!/usr/bin/env python3
"""Headline benchmark: distributed El::Gemm TFLOP/s on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W [--config c2|c3|c4|c5]
  (N > 1: one process per GPU.  Under torch.distributed.run RANK / LOCAL_RANK /
   WORLD_SIZE / MASTER_* come from the environment; with WORLD_SIZE unset this
   script starts the N rank processes itself with that same environment
   (launch_ranks) and exits with the first failing rank's status)

One step = one El::Gemm(...) on DistMatrix operands already resident in HBM,
inputs from the grid-independent counter hash (synthetic data, Uniform(-0.1,
0.1) as tests/blas_like/Gemm_Suite.cpp:158-172, alpha = 0.5, beta = -0.5).
The whole SUMMA runs inside the timed region: every panel redistribution over
RCCL and every MFMA update (beta is folded into the first panel's update).
Default workload (the driver's line):
  N = 1 : C2, El::Gemm NN fp64 m=n=k=32768 on a 1x1 grid (BASELINE.json configs[1]).
  N > 1 : C3, SUMMA El::Gemm NN fp64 m=n=k=65536 on Grid::DefaultHeight(N)
          (1x2, 2x2, 2x4): strong scaling of the same problem.
  N = 1 also reports "c3_1gpu": C3's n = 65536 on the one GPU through the same
          kc = 8192 panel path (the automatic panel at K = 65536 on grids
          larger than 1x1), the same-problem denominator for strong scaling.
  N > 1 first checks the reference's associativity residual through the
          distributed path (n = 4096) and reports xGMI GB/s from transfer-only
          events plus the compute-stream gaps the panel pipeline left exposed.
  N > 1 runs C3 and the residual only (--extra-configs adds the C4 / C5 points
          after it).
Extra lines (evidence, not the driver's default):
  --config c4 : TN fp32 m=n=8192, k=524288*N, inputs [VC,STAR] (LBANN's
                weight-gradient shape, SUMMA_DOT); weak scaling, = C4 at N=8.
  --config c5 : NN bf16 (or --dtype f16) m=n=k=32768 on [MC,MR], plus
                DistMatrix Axpy and Hadamard on the same operands (GB/s).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X dense peaks (MI355X_MICROARCH.md: fp64/fp32 MFMA = vector rate; bf16/f16 2.5 PF dense)
PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3, "bf16": 2500.0, "f16": 2500.0}
HBM_PEAK_GBS = 8000.0
METRIC = "distributed Gemm TFLOP/s (fp64/fp32) at 1/2/4/8 GPUs; % of MFMA peak"
KERNEL = {"f64": "gemm_f64r_kernel (LDS-DMA ring)", "f32": "gemm_f32r_kernel (LDS-DMA ring)",
          "bf16": "gemm_h4w_kernel<bf16> (four-wave)", "f16": "gemm_h4w_kernel<f16> (four-wave)"}


_WATCHDOG = None  # elemental_amd.el once imported


def stage(name: str, seconds: float):
    """Progress line on stderr and a watchdog deadline for the next stage: past
    it (or on an asynchronous RCCL error) the library aborts its RCCL
    communicators and the process exits naming the stage (elx_watchdog_stage),
    instead of hanging a multi-GPU run."""
    if _WATCHDOG is None:
        return
    if os.environ.get("ELX_BENCH_HANG") == name:
        # fault injection for tests/test_gpu_dist.py: this stage hangs
        _WATCHDOG.watchdog_stage(name, 2.0)
        time.sleep(120)
    _WATCHDOG.watchdog_stage(name, seconds)


def cpu_baseline(seconds_target: float = 10.0) -> dict:
    """The CPU leg: C1 (BASELINE.json configs[0]), El::Gemm NN
    fp64 4096^3 on a 2x2 grid, run as the reference's CPU path runs it: SUMMA_NNC
    over 4 processes with nb = 128 all-gathers and one MKL dgemm_ per panel
    (oracle/cpu_summa.c), for ~seconds_target.  On 8 cores (2 per rank, each
    rank pinned to its own): the core count of the reference's own C1 figure
    (0.477 TF on 8 cores), so the two compare per core; the
    same run on every core the box grants (16) is reported beside it.
    MKL runs its AVX-512 kernels, as on the reference's Xeon (its CPU dispatch
    would pick its AVX2 code on the box's AMD EPYC 9575F: half the speed; see
    oracle/cpu_summa.c).  Placement measured on the box
    (profiles/r04_cpu_baseline_sweep2.log): 1 / 2 / 4 MKL threads per rank =
    137 / 84 / 107 GF per core with the AVX-512 kernels, 69 / 55 / 52 with AVX2."""
    import oracle
    from oracle import cpu_summa
    out = cpu_summa.run(n=4096, nb=128, r=2, c=2, seconds=seconds_target, cores=8)
    allc = oracle.cpu_threads()
    if allc > 8:
        try:
            wide = cpu_summa.run(n=4096, nb=128, r=2, c=2, seconds=seconds_target / 2, cores=allc)
            out["all_cores"] = {"value": wide["value"], "cores": wide["cores"]}
        except Exception as e:  # context only
            out["all_cores"] = {"error": str(e)}
    out["per_core_gflops"] = round(out["value"] * 1e3 / out["cores"], 1)
    out["reference_per_core_gflops"] = round(477.0 / 8, 1)
    return out


def measured_traffic(dtype: str, n: int, world: int):
    """Per-launch HBM bytes of the GEMM kernel from the committed rocprofv3 PMC
    passes of this same bench command (tools/collect_profiles.sh ->
    profiles/traffic_index.json), or None when that configuration was not profiled."""
    path = os.path.join(ROOT, "profiles", "traffic_index.json")
    if not os.path.exists(path):
        return None
    ent = json.load(open(path)).get(f"{dtype}:{n}:{world}")
    return ent["hbm_bytes_per_launch"] if ent else None


def profile_summary(L, ctypes_mod):
    """Event-timed stats of the profiled region: local MFMA launches, panel
    transfers (whole redistribution incl. pack/unpack), RCCL transfers only,
    and the compute-stream gaps between consecutive panel updates."""
    c = ctypes_mod
    gemm_ms, launches, flops = c.c_double(), c.c_int64(), c.c_double()
    comm_ms, comm_bytes = c.c_double(), c.c_int64()
    L.call("elx_profile_stats", c.byref(gemm_ms), c.byref(launches), c.byref(flops), c.byref(comm_ms),
           c.byref(comm_bytes))
    x_ms, x_bytes, x_n = c.c_double(), c.c_int64(), c.c_int64()
    L.call("elx_profile_transfers", c.byref(x_ms), c.byref(x_bytes), c.byref(x_n))
    gap_ms, gaps = c.c_double(), c.c_int64()
    L.call("elx_profile_pipeline", c.byref(gap_ms), c.byref(gaps))
    return {"gemm_ms": gemm_ms.value, "launches": launches.value, "flops": flops.value,
            "redist_ms": comm_ms.value, "redist_bytes": comm_bytes.value,
            "xfer_ms": x_ms.value, "xfer_bytes": x_bytes.value, "xfers": x_n.value,
            "gap_ms": gap_ms.value, "gaps": gaps.value}


def collectives_summary(prof: dict, steps: int) -> dict:
    """Per-rank panel traffic: RCCL transfer-only GB/s (events around each grouped
    send/recv; bytes = algorithmic bytes received), the whole redistribution time
    (pack + transfer + unpack), and how much compute-stream time the pipeline
    left exposed between panel updates."""
    x = prof
    return {
        "bytes_per_rank_per_step": x["xfer_bytes"] // max(steps, 1),
        "transfers_timed": x["xfers"],
        "transfer_ms_per_rank": round(x["xfer_ms"], 3),
        "GB_per_s": round(x["xfer_bytes"] / (x["xfer_ms"] * 1e-3) / 1e9, 2) if x["xfer_ms"] > 0 else None,
        "redistribution_ms_per_rank": round(x["redist_ms"], 3),
        "exposed_compute_gap_ms_per_step": round(x["gap_ms"] / max(steps, 1), 3),
        "panel_gaps_timed": x["gaps"],
    }


def associativity_residual(el, grid, n: int = 4096, nrhs: int = 100) -> float:
    """tests/blas_like/Gemm.cpp:15-49 on the distributed path itself (no oracle):
    C_f = 0.5 A B - 0.5 C, then ||(0.5 A (B X) - 0.5 C X) - C_f X||_F / ||Y||_F
    with every product an El::Gemm on this grid; norms on VC rank 0."""
    import numpy as np
    mk = lambda h, w, seed: el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=h, width=w).fill_hash(seed, 0.0, 0.1)
    A, B, C, X = mk(n, n, 5), mk(n, n, 6), mk(n, n, 7), mk(n, nrhs, 8)
    BX = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=n, width=nrhs)
    Y = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=n, width=nrhs)
    CX = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=n, width=nrhs)
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, B, X, 0.0, BX)
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, C, X, 0.0, CX)
    el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, BX, 0.0, Y)
    el.Axpy(-0.5, CX, Y)                                   # Y = 0.5 A B X - 0.5 C X
    el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)     # C_f
    E = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=n, width=nrhs)
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, C, X, 0.0, E)
    el.Axpy(-1.0, Y, E)                                    # E = C_f X - Y
    out = []
    for M in (E, Y):
        R = el.DistMatrix(grid, el.F64, el.CIRC, el.CIRC, el.GPU)
        R.assign(M)
        out.append(R.get_local())
    if grid.vc_rank != 0:
        return float("nan")
    return float(np.linalg.norm(out[0]) / np.linalg.norm(out[1]))


# unit roundoff of each storage type
UNIT_ROUNDOFF = {"f64": 2.0 ** -53, "f32": 2.0 ** -24, "bf16": 2.0 ** -8, "f16": 2.0 ** -11}


def check_tolerance(dtype: str, k: int) -> tuple[float, str]:
    """Bound for the associativity residual of a full-size point: 10 u sqrt(k)
    for f64 / f32 (the probabilistic normwise bound of a length-k sum), 16 u for
    f16 / bf16 (f32 accumulation: the storage roundings of Z, Y and C_f
    dominate, a few u)."""
    u = UNIT_ROUNDOFF[dtype]
    if dtype in ("f64", "f32"):
        return 10.0 * u * k ** 0.5, "10 u sqrt(k)"
    return 16.0 * u, "16 u (f32 accumulation)"


def verify_point(el, grid, DT, dtype: str, oA, step, A, B, C, k: int, alpha: float = 0.5, beta: float = -0.5,
                 nrhs: int = 100) -> dict:
    """The reference's associativity check on a timed configuration itself
    (tests/blas_like/Gemm_Suite.cpp:91-132,190-195; tests/blas_like/Gemm.cpp:15-49):
    C0 := C, one more step() through the very path that was timed (C_f = alpha
    op(A) B + beta C0), then Y = alpha op(A) (B X) + beta C0 X and
    ||Y - C_f X||_F / ||Y||_F with X Uniform-like in [-0.25, 0.25), n x 100,
    every product an El::Gemm on the same grid.  No oracle: self-consistency at
    BASELINE sizes, as the reference checks its own runs."""
    m, n = C.Height(), C.Width()
    C0 = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU)
    C0.assign(C)
    step()
    X = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=n, width=nrhs).fill_hash(11, 0.0, 0.25)
    Z = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=k, width=nrhs)
    Y = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=m, width=nrhs)
    el.Gemm(el.NORMAL, el.NORMAL, 1.0, B, X, 0.0, Z)          # Z = B X
    el.Gemm(oA, el.NORMAL, alpha, A, Z, 0.0, Y)               # Y = alpha op(A) Z
    el.Gemm(el.NORMAL, el.NORMAL, beta, C0, X, 1.0, Y)        # Y += beta C0 X
    ynorm = el.FrobeniusNorm(Y)
    el.Gemm(el.NORMAL, el.NORMAL, -1.0, C, X, 1.0, Y)         # E = Y - C_f X
    enorm = el.FrobeniusNorm(Y)
    del C0, X, Z, Y
    r = enorm / ynorm if ynorm > 0 else float("inf")
    tol, rule = check_tolerance(dtype, k)
    return {"check": f"associativity ||Y - C_f X||_F/||Y||_F, {nrhs} rhs, at this point's full size "
                     "(tests/blas_like/Gemm.cpp:15-49)",
            "residual": r, "tol": tol, "tol_rule": rule, "ok": bool(r <= tol)}


def est_seconds(flops: float, dtype: str, world: int) -> float:
    """Pessimistic duration of `flops` on `world` GPUs (half the measured rates),
    for the watchdog deadlines."""
    rate = {"f64": 35e12, "f32": 70e12, "bf16": 600e12, "f16": 600e12}[dtype] * world
    return flops / rate


def c3_one_gpu(el, L, grid, barrier, steps: int, warmup: int, kc_restore: int, n: int = 65536,
               kc: int = 8192, dtype: str = "f64") -> dict:
    """C3 (El::Gemm NN fp64 / fp32 m=n=k=65536) on a 1x1 grid through the panel path:
    k in uniform kc-deep compute panels (8 launches of 65536^2 x 8192).  The
    1x2 / 2x2 / 2x4 grids gather their panels and ramp the first ones (kc/4,
    kc/2, kc, ..., gemm.cpp SummaC), so they run 9 launches whose first two are
    shallower; value_N / (N * value) is a same-problem strong-scaling
    efficiency that charges that ramp to the N > 1 side."""
    el.SetComputePanel(kc)
    DT = {"f64": el.F64, "f32": el.F32}[dtype]
    name = "c3_1gpu" if dtype == "f64" else f"c3_1gpu_{dtype}"
    stage(name, 120 + 4 * (steps + warmup) * est_seconds(2.0 * n ** 3, dtype, 1))
    try:
        A = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(1, 0.0, 0.1)
        B = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(2, 0.0, 0.1)
        C = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(3, 0.0, 0.1)
        for _ in range(warmup):
            el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)
        barrier()
        L.call("elx_set_profiling", 1)
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)
        barrier()
        elapsed = time.perf_counter() - t0
        prof = profile_summary(L, ctypes)
        L.call("elx_set_profiling", 0)
        stage(f"{name} verify", 120 + 4 * est_seconds(2.0 * n ** 3, dtype, 1))
        check = verify_point(el, grid, DT, dtype, el.NORMAL,
                             lambda: el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C), A, B, C, n)
        del A, B, C
    finally:
        el.SetComputePanel(kc_restore)
    value = 2.0 * n ** 3 * steps / elapsed / 1e12
    avg_ms = prof["gemm_ms"] / max(prof["launches"], 1)
    fpl = prof["flops"] / max(prof["launches"], 1)
    ach = fpl / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    return {"workload": f"C3 on 1 GPU: El::Gemm NN {dtype} m=n=k={n}, Grid 1x1, compute panel kc={kc} "
                        f"({n // kc} uniform MFMA launches per step; grids > 1x1 ramp the first panels kc/4, kc/2)",
            "value": round(value, 3), "unit": "TFLOP/s", "dtype": dtype, "steps": steps, "warmup": warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "pct_of_mfma_peak": round(100.0 * value / PEAK_TFLOPS[dtype], 2),
            "roofline": {"bound": "mfma", "kernel": KERNEL[dtype], "achieved": round(ach, 3),
                         "peak": PEAK_TFLOPS[dtype], "frac": round(ach / PEAK_TFLOPS[dtype], 4),
                         "launches_timed": prof["launches"], "avg_launch_ms": round(avg_ms, 3)},
            "exposed_compute_gap_ms_per_step": round(prof["gap_ms"] / max(steps, 1), 3),
            "verify": check}


def config_point(el, L, grid, barrier, maxr, config: str, steps: int, warmup: int, world: int, size: int = 0,
                 half: str = "bf16") -> dict:
    """The other BASELINE configs as sub-results of the default line (evidence
    beside the driver's C2 / C3 value, measured in the same run on the same
    grid): C4, TN fp32 m=n=8192 k=524288*N with [VC,STAR] inputs (SUMMA_DOT,
    LBANN's weight-gradient shape; weak scaling, = C4 at N=8), and C5, NN bf16
    32768^3 on [MC,MR] plus DistMatrix Axpy / Hadamard on the same operands.
    size > 0 (rehearsals only): m = n = min(8192, size), k = size*N for C4, n = size for C5."""
    gshape = f"{grid.height}x{grid.width}"
    if config == "c4":
        m = n = min(8192, size) if size else 8192
        k = (size or 524288) * world
        DT, dtype, oA = el.F32, "f32", el.TRANSPOSE
        A = el.DistMatrix(grid, DT, el.VC, el.STAR, el.GPU, height=k, width=m).fill_hash(1, 0.0, 0.1)
        B = el.DistMatrix(grid, DT, el.VC, el.STAR, el.GPU, height=k, width=n).fill_hash(2, 0.0, 0.1)
        workload = f"C4: El::Gemm TN f32 m=n={m} k={k} (SUMMA_DOT), A,B [VC,STAR], Grid {gshape}"
    else:
        m = n = k = size or 32768
        DT, dtype, oA = {"bf16": el.BF16, "f16": el.F16}[half], half, el.NORMAL
        A = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=m, width=k).fill_hash(1, 0.0, 0.1)
        B = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=k, width=n).fill_hash(2, 0.0, 0.1)
        workload = f"C5: El::Gemm NN {half} m=n=k={m} on [MC,MR], Grid {gshape}"
    C = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=m, width=n).fill_hash(3, 0.0, 0.1)
    sname = config if dtype in ("f32", "bf16") else f"{config}_{dtype}"
    stage(sname, 120 + 4 * (warmup + steps) * est_seconds(2.0 * m * n * k, dtype, world))
    for _ in range(warmup):
        el.Gemm(oA, el.NORMAL, 0.5, A, B, -0.5, C)
    barrier()
    L.call("elx_set_profiling", 1)
    t0 = time.perf_counter()
    for _ in range(steps):
        el.Gemm(oA, el.NORMAL, 0.5, A, B, -0.5, C)
    barrier()
    elapsed = maxr(time.perf_counter() - t0)
    prof = profile_summary(L, ctypes)
    L.call("elx_set_profiling", 0)
    value = 2.0 * m * n * k * steps / elapsed / 1e12
    avg_ms = prof["gemm_ms"] / max(prof["launches"], 1)
    fpl = prof["flops"] / max(prof["launches"], 1)
    ach = fpl / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    out = {"workload": workload, "value": round(value, 3), "unit": "TFLOP/s", "dtype": dtype, "steps": steps,
           "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
           "pct_of_mfma_peak": round(100.0 * value / (PEAK_TFLOPS[dtype] * world), 2),
           "roofline": {"bound": "mfma", "kernel": KERNEL[dtype],
                        "achieved": round(ach, 3), "peak": PEAK_TFLOPS[dtype], "frac": round(ach / PEAK_TFLOPS[dtype], 4),
                        "launches_timed": prof["launches"], "avg_launch_ms": round(avg_ms, 3)}}
    if world > 1:
        out["collectives"] = collectives_summary(prof, steps)
    stage(f"{sname} verify", 120 + 4 * est_seconds(2.0 * m * n * k, dtype, world))
    out["verify"] = verify_point(el, grid, DT, dtype, oA, lambda: el.Gemm(oA, el.NORMAL, 0.5, A, B, -0.5, C),
                                 A, B, C, k)
    if config == "c5":
        stage(f"{sname} entrywise", 120)
        loc = A.LocalHeight() * A.LocalWidth()
        ew = {}
        for name, fn in (("axpy", lambda: el.Axpy(0.5, A, C)), ("hadamard", lambda: el.Hadamard(A, B, C))):
            fn()
            barrier()
            t1 = time.perf_counter()
            for _ in range(20):
                fn()
            barrier()
            dt = maxr((time.perf_counter() - t1) / 20)
            gbs = 3 * 2 * loc / dt / 1e9  # both 16-bit types
            ew[name] = {"ms": round(dt * 1e3, 4), "GB_per_s_per_gpu": round(gbs, 1),
                        "frac_of_hbm": round(gbs / HBM_PEAK_GBS, 4)}
        out["entrywise"] = ew
    del A, B, C
    return out


def _free_port() -> int:
    """A loopback port that is free now, with port + 1 free too (the library's own
    rendezvous defaults to MASTER_PORT + 1, comm.cpp InitWorldFromEnv), drawn below
    the ephemeral range so no outgoing connection can take it meanwhile."""
    import random
    import socket
    for _ in range(256):
        port = random.randrange(20000, 32000)
        try:
            with socket.socket() as s, socket.socket() as s2:
                s.bind(("127.0.0.1", port))
                s2.bind(("127.0.0.1", port + 1))
            return port
        except OSError:
            continue
    raise RuntimeError("no free loopback port pair in 20000-32000")


def rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    """The environment torch.distributed.run gives rank `rank` of a one-node job:
    the launcher variables the reference maps to a device
    (src/hydrogen/device/GPU.cpp:30-50: LOCAL_RANK picks the GPU)."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", ROLE_RANK=str(rank), ROLE_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1")
    return env


def launch_ranks(argv: list[str], world: int, child_cmd: list[str] | None = None, grace_s: float = 45.0,
                 poll_s: float = 0.2) -> int:
    """`python3 bench.py --gpus N` with no launcher around it (WORLD_SIZE unset):
    start N child processes of this script, one per GPU, with the environment
    torch.distributed.run would give them (rank_env), and wait.  Called before
    torch or the library is imported, so this process never touches the GPU and
    never execs.  Children inherit stdout, so rank 0's JSON line is the line the
    caller reads.  Exit status: 0 when every rank exits 0; otherwise the first
    failing rank's status (a signal death maps to 128 + signal).  After the first
    failure the others get `grace_s` to end on their own (their watchdog aborts
    RCCL and exits naming the stage), then SIGTERM, then SIGKILL -- by PID, only
    the processes started here.  SIGTERM / SIGINT to this process are forwarded."""
    import signal
    import subprocess
    port = _free_port()
    cmd = child_cmd or [sys.executable, "-u", os.path.abspath(__file__)]
    procs = []

    def stop_all(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    def on_signal(signum, _frame):
        stop_all(signum)

    # forward SIGTERM / SIGINT from before the first child starts
    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    status = 0
    failed_at = None
    try:
        for r in range(world):
            procs.append(subprocess.Popen(cmd + list(argv), env=rank_env(os.environ, r, world, port)))
        while True:
            codes = [p.poll() for p in procs]
            for r, c in enumerate(codes):
                if c is not None and c != 0 and status == 0:
                    status = c if c > 0 else 128 - c
                    failed_at = time.monotonic()
                    print(f"[bench launcher] rank {r} exited with status {c}; "
                          f"stopping the others in {grace_s:.0f} s", file=sys.stderr, flush=True)
            if all(c is not None for c in codes):
                break
            if failed_at is not None:
                waited = time.monotonic() - failed_at
                if waited > grace_s + 10:
                    stop_all(signal.SIGKILL)
                elif waited > grace_s:
                    stop_all(signal.SIGTERM)
            time.sleep(poll_s)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return status


def main():
    # N > 1 without a launcher: become the launcher (decided before torch or the
    # library is loaded; this process never initialises the GPU)
    if "WORLD_SIZE" not in os.environ:
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        n, _ = pre.parse_known_args()
        if n.gpus > 1:
            sys.exit(launch_ranks(sys.argv[1:], n.gpus))

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=["auto", "c2", "c3", "c4", "c5"], default="auto")
    ap.add_argument("--n", "--size", dest="n", type=int, default=0,
                    help="override m=n=k (c2/c3/c5); --size under torch.distributed.run, whose parser takes --n")
    ap.add_argument("--dtype", choices=["f64", "f32", "bf16", "f16"], default=None)
    ap.add_argument("--nb", type=int, default=128, help="El::Blocksize (communication panel)")
    ap.add_argument("--kc", type=int, default=0, help="compute panel (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-residual", action="store_true", help="skip the N>1 associativity check")
    ap.add_argument("--c3-steps", type=int, default=2, help="timed steps of the N=1 C3 point")
    ap.add_argument("--no-c3-1gpu", action="store_true",
                    help="N=1: skip the same-problem C3 point (n=65536 through the panel path)")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="N=1: skip the C4 / C5 single-GPU points of the default line")
    ap.add_argument("--extra-configs", action="store_true",
                    help="N>1: also run the C4 / C5 points after C3 (off by default, so an "
                         "overrun there cannot touch the C3 line; --config c4 / c5 print them alone)")
    args = ap.parse_args()

    # stdout carries exactly one line, the JSON: whatever the libraries print on
    # file descriptor 1 (gloo's "[Gloo] Rank ... connected" lines, RCCL's INFO
    # output) goes to stderr from here on, and the line goes out through a
    # duplicate of the original descriptor
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    os.environ["ELX_WATCHDOG_FD"] = str(line_out.fileno())  # the watchdog's epitaph line goes there too

    import torch
    from elemental_amd import el
    from elemental_amd import _lib as L
    global _WATCHDOG
    _WATCHDOG = el
    stage("init", 600)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    # ELX_BENCH_COMM=host: rehearsal of the N>1 line on a one-GPU box — every
    # rank on device 0, panels host-staged over gloo instead of RCCL (RCCL refuses
    # two ranks on one GPU); never the driver's configuration
    rehearse = world > 1 and os.environ.get("ELX_BENCH_COMM") == "host"
    dev = 0 if rehearse else local
    L.call("elx_set_device", dev)
    torch.cuda.set_device(dev)

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only (uid, barrier, max); data goes over RCCL
        if rehearse:
            from elemental_amd.torch_bridge import GlooBridge
            comm = el.Comm.host(GlooBridge())
        else:
            obj = [el.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            comm = el.Comm.rccl(rank, world, obj[0])
    else:
        comm = el.Comm.self_comm()
    grid = el.Grid(comm, 0)
    gshape = f"{grid.height}x{grid.width}"

    config = args.config if args.config != "auto" else ("c2" if world == 1 else "c3")
    dtype = args.dtype or {"c2": "f64", "c3": "f64", "c4": "f32", "c5": "bf16"}[config]
    DT = {"f64": el.F64, "f32": el.F32, "bf16": el.BF16, "f16": el.F16}[dtype]
    el.SetBlocksize(args.nb)
    el.SetComputePanel(args.kc)
    scaling = "strong"
    if config == "c4":
        m = n = 8192
        k = 524288 * world
        oA = el.TRANSPOSE
        # A is k x m and B is k x n, both [VC,STAR] (k over all ranks, LBANN-native)
        A = el.DistMatrix(grid, DT, el.VC, el.STAR, el.GPU, height=k, width=m).fill_hash(1, 0.0, 0.1)
        B = el.DistMatrix(grid, DT, el.VC, el.STAR, el.GPU, height=k, width=n).fill_hash(2, 0.0, 0.1)
        scaling = "weak"
        workload = f"C4: El::Gemm TN {dtype} m=n=8192 k={k} (SUMMA_DOT), A,B [VC,STAR], Grid {gshape}"
    else:
        m = n = k = args.n or {"c2": 32768, "c3": 65536, "c5": 32768}[config]
        oA = el.NORMAL
        A = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=m, width=k).fill_hash(1, 0.0, 0.1)
        B = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=k, width=n).fill_hash(2, 0.0, 0.1)
        workload = (f"C2: El::Gemm NN {dtype} m=n=k={m}, Grid {gshape}" if config == "c2" else
                    f"C3: SUMMA El::Gemm NN {dtype} m=n=k={m}, Grid {gshape}" if config == "c3" else
                    f"C5: SUMMA El::Gemm NN {dtype} m=n=k={m} + DistMatrix Axpy/Hadamard, Grid {gshape}")
    C = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=m, width=n).fill_hash(3, 0.0, 0.1)

    def barrier():
        el.device_synchronize()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    def step():
        return el.Gemm(oA, el.NORMAL, 0.5, A, B, -0.5, C)

    step_flops = 2.0 * m * n * k
    residual = None
    if world > 1 and not args.no_residual:
        # correctness on this very grid before timing (no oracle): the reference's
        # associativity check through the distributed path
        stage("residual", 300)
        try:
            residual = associativity_residual(el, grid)
        except Exception as e:  # report, never lose the timed line to the check
            residual = f"error: {e}"
        barrier()

    stage("warmup", 120 + 4 * args.warmup * est_seconds(step_flops, dtype, world))
    for _ in range(args.warmup):
        step()
    barrier()
    stage("timed", 120 + 4 * args.steps * est_seconds(step_flops, dtype, world))
    L.call("elx_set_profiling", 1)
    el.comm_stats_reset()
    barrier()
    t0 = time.perf_counter()
    alg = el.GEMM_DEFAULT
    for _ in range(args.steps):
        alg = step()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = profile_summary(L, ctypes)
    L.call("elx_set_profiling", 0)

    def max_over_ranks(x: float) -> float:
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    elapsed = max_over_ranks(elapsed)
    total_flops = step_flops * args.steps
    value = total_flops / elapsed / 1e12
    avg_ms = prof["gemm_ms"] / max(prof["launches"], 1)
    flops_per_launch = prof["flops"] / max(prof["launches"], 1)
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    peak = PEAK_TFLOPS[dtype]
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (grid-independent hash, Uniform(-0.1,0.1)); alpha=0.5, beta=-0.5",
        "config": {
            "workload": workload,
            "m": m, "n": n, "k": k,
            "grid": gshape,
            "algorithm": {2: "SUMMA_A", 4: "SUMMA_B", 6: "SUMMA_C", 7: "SUMMA_DOT"}.get(alg, str(alg)),
            "blocksize": args.nb,
            "compute_panel": args.kc or "auto",
            "parallelism": f"grid{gshape}",
            **({"comm": "host-staged gloo, all ranks on device 0 (rehearsal)"} if rehearse else {}),
        },
        "pct_of_mfma_peak": round(100.0 * value / (peak * world), 2),
        "roofline": {
            "bound": "mfma",
            "kernel": f"{KERNEL[dtype]} (local panel update)",
            "achieved": round(achieved, 3),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": measured_traffic(dtype, m, world) if config in ("c2", "c3") else None,
            "traffic_unit": "bytes/launch (PMC FETCH_SIZE*2 + WRITE_SIZE)",
            "launches_timed": prof["launches"],
            "avg_launch_ms": round(avg_ms, 3),
            "flops_per_launch": flops_per_launch,
        },
        "collectives": collectives_summary(prof, args.steps),
    }
    if residual is not None:
        out["residual"] = {"check": "associativity ||(aAB+bC)X - C_f X||_F/||Y||_F, n=4096, 100 rhs "
                                    "(tests/blas_like/Gemm.cpp:15-49)", "value": residual,
                           "ok": isinstance(residual, float) and residual < 1e-13}
    cus = ctypes.c_int()
    L.call("elx_reserved_cus", ctypes.byref(cus))
    out["config"]["comm_reserved_cus"] = cus.value

    # the timed point itself, checked at full size through the same path (one
    # more, untimed step)
    stage("verify", 120 + 4 * est_seconds(step_flops, dtype, world))
    try:
        out["verify"] = verify_point(el, grid, DT, dtype, oA, step, A, B, C, k)
    except Exception as e:
        out["verify"] = {"error": str(e), "ok": False}
    barrier()

    # from here on the line exists: if a later (optional) stage overruns, the
    # watchdog prints it with that stage marked and the process still exits
    # NON-ZERO (ELX_WATCHDOG_EXIT), so a hang is never recorded as success
    def epitaph(pending: str | None):
        if rank != 0:
            el.watchdog_epitaph("", el.WATCHDOG_EXIT)
            return
        line = dict(out)
        if pending:
            line[pending] = {"error": f"watchdog: stage {pending} overran its deadline (RCCL aborted)"}
            line["incomplete"] = f"stage {pending} overran; exit status {el.WATCHDOG_EXIT}"
        el.watchdog_epitaph(json.dumps(line), el.WATCHDOG_EXIT)

    def extra(key: str, fn):
        epitaph(key)
        try:
            out[key] = fn()
        except Exception as e:  # evidence only: never lose the driver's line to it
            out[key] = {"error": str(e)}
        epitaph(None)

    if config == "c5":
        # DistMatrix Axpy / Hadamard on the [MC,MR] operands (no exchange: each
        # rank updates its local block); HBM bytes 3 x local elements x size
        def entrywise():
            stage("entrywise", 120)
            es = {"f64": 8, "f32": 4, "bf16": 2, "f16": 2}[dtype]
            loc = A.LocalHeight() * A.LocalWidth()
            ew = {}
            for name, fn, reps in (("axpy", lambda: el.Axpy(0.5, A, C), 20),
                                   ("hadamard", lambda: el.Hadamard(A, B, C), 20)):
                fn()
                barrier()
                t1 = time.perf_counter()
                for _ in range(reps):
                    fn()
                barrier()
                dt = max_over_ranks((time.perf_counter() - t1) / reps)
                gbs = 3 * es * loc / dt / 1e9
                ew[name] = {"ms": round(dt * 1e3, 4), "GB_per_s_per_gpu": round(gbs, 1),
                            "frac_of_hbm": round(gbs / HBM_PEAK_GBS, 4)}
            return ew
        extra("entrywise", entrywise)
    if config == "c4":
        # the same product with [MC,MR] inputs: SUMMA_DOT's read
        # proxies first redistribute A and B to [VC,*] (TN.hpp:384-391), inside
        # the timed region
        def mcmr():
            nonlocal A, B
            A = B = None
            stage("c4_mcmr_inputs", 120 + 4 * (args.steps + 1) * est_seconds(step_flops, dtype, world))
            Am = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=k, width=m).fill_hash(1, 0.0, 0.1)
            Bm = el.DistMatrix(grid, DT, el.MC, el.MR, el.GPU, height=k, width=n).fill_hash(2, 0.0, 0.1)
            el.Gemm(oA, el.NORMAL, 0.5, Am, Bm, -0.5, C)
            barrier()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                el.Gemm(oA, el.NORMAL, 0.5, Am, Bm, -0.5, C)
            barrier()
            dt = max_over_ranks(time.perf_counter() - t1)
            return {"workload": workload.replace("[VC,STAR]", "[MC,MR] (proxied to [VC,STAR] each call)"),
                    "value": round(2.0 * m * n * k * args.steps / dt / 1e12, 3), "unit": "TFLOP/s",
                    "ms_per_step": round(dt / args.steps * 1e3, 3)}
        extra("c4_mcmr_inputs", mcmr)
    if world == 1 and config == "c2" and not args.n and not args.no_c3_1gpu:
        # the same problem as the driver's N>1 lines (C3, n = 65536, kc = 8192
        # compute panels as EffectivePanel picks on grids > 1x1), on this one GPU
        A = B = C = None  # release the C2 operands before the n = 65536 ones
        extra("c3_1gpu", lambda: c3_one_gpu(el, L, grid, barrier, args.c3_steps, 1, args.kc))
        # C3 is "fp64/fp32": the fp32 half of the same problem
        extra("c3_1gpu_f32", lambda: c3_one_gpu(el, L, grid, barrier, args.c3_steps, 1, args.kc, dtype="f32"))
    extras = (world == 1 and not args.no_extra_configs) or (world > 1 and args.extra_configs)
    if config in ("c2", "c3") and (not args.n or rehearse) and extras:
        # the other BASELINE configs, measured in the same run on the same grid
        # (N = 1: c4_1gpu / c5_1gpu; N > 1 with --extra-configs: c4 / c5 on
        # Grid::DefaultHeight(N))
        A = B = C = None  # release the main operands (no-op when already released)
        # C5 is "bf16/half": both 16-bit types
        for cfg, st, half in (("c4", 2, "bf16"), ("c5", 5, "bf16"), ("c5", 5, "f16")):
            key = (f"{cfg}_1gpu" if world == 1 else cfg) + ("_f16" if half == "f16" else "")
            extra(key, lambda cfg=cfg, st=st, half=half: config_point(el, L, grid, barrier, max_over_ranks, cfg, st, 1,
                                                                      world, args.n, half))
    if world == 1 and config == "c2" and not args.n and not args.no_extra_configs:
        # C1's problem (NN f64 4096^3) on the GPU, beside the CPU leg's same problem
        def c1():
            stage("c1_1gpu", 120)
            n1 = 4096
            A1 = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=n1, width=n1).fill_hash(1, 0.0, 0.1)
            B1 = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=n1, width=n1).fill_hash(2, 0.0, 0.1)
            C1 = el.DistMatrix(grid, el.F64, el.MC, el.MR, el.GPU, height=n1, width=n1).fill_hash(3, 0.0, 0.1)
            for _ in range(3):
                el.Gemm(el.NORMAL, el.NORMAL, 0.5, A1, B1, -0.5, C1)
            barrier()
            t1 = time.perf_counter()
            for _ in range(20):
                el.Gemm(el.NORMAL, el.NORMAL, 0.5, A1, B1, -0.5, C1)
            barrier()
            dt = (time.perf_counter() - t1) / 20
            return {"workload": "C1's problem on the GPU: El::Gemm NN f64 m=n=k=4096, Grid 1x1",
                    "value": round(2.0 * n1 ** 3 / dt / 1e12, 3), "unit": "TFLOP/s", "steps": 20,
                    "ms_per_step": round(dt * 1e3, 3)}
        extra("c1_1gpu", c1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        def cpu():
            stage("cpu_baseline", 300)
            return cpu_baseline()
        extra("cpu_baseline", cpu)
    stage("report", 300)
    if rank == 0:
        print(json.dumps(out), file=line_out, flush=True)
    el.watchdog_epitaph("", 0)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    stage("done", 0)


if __name__ == "__main__":
    main()
