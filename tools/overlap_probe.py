#!/usr/bin/env python3
"""Can panel-transfer kernels run while the MFMA update fills the machine?

On one MI355X: an fp64 El::Gemm (n = 16384, kc = 2048 compute panels, the
C-stationary update of every SUMMA step) on the library's compute stream, and
pack/unpack-sized device copies (256 MiB, what one C3 panel gather moves per
peer) injected on the library's high-priority comm stream every `gap_ms`
while it runs.  Reported: the GEMM time alone and with the copies, and each
copy's event-timed duration alone and under the GEMM (a copy whose workgroups
cannot find a CU waits for GEMM workgroups to retire).  Run once per
ELX_COMM_CUS setting (CUs masked off the compute stream, read at init);
OVERLAP_OP=sum injects a reduction instead (workgroups that need LDS, as RCCL's
kernels do, beside a GEMM whose ring kernel holds every CU's LDS):

  ELX_COMM_CUS=0 python tools/overlap_probe.py ; ELX_COMM_CUS=8 python tools/overlap_probe.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from elemental_amd import _lib as L
    from elemental_amd import el

    n, kc, copy_mib, gap_ms = 16384, 2048, 256, 40.0
    g = el.Grid()
    A = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(1, 0.0, 0.1)
    B = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(2, 0.0, 0.1)
    C = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(3, 0.0, 0.1)
    el.SetComputePanel(kc)
    cp, mp = ctypes.c_void_p(), ctypes.c_void_p()
    L.call("elx_default_stream", ctypes.byref(cp))
    L.call("elx_comm_stream", ctypes.byref(mp))
    cus = ctypes.c_int()
    L.call("elx_reserved_cus", ctypes.byref(cus))
    cstream = torch.cuda.ExternalStream(cp.value)
    mstream = torch.cuda.ExternalStream(mp.value)
    src = torch.rand(copy_mib * (1 << 20) // 8, dtype=torch.float64, device="cuda")
    dst = torch.empty_like(src)
    red = torch.empty((), dtype=torch.float64, device="cuda")
    op = os.environ.get("OVERLAP_OP", "copy")
    torch.cuda.synchronize()

    def gemm_ms():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(cstream)
        el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)
        b.record(cstream)
        return a, b

    def copy_ev():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(mstream):
            a.record(mstream)
            if op == "sum":  # a reduction: workgroups that need LDS, as RCCL's kernels do
                torch.sum(src, dim=0, out=red)
            else:
                dst.copy_(src)
            b.record(mstream)
        return a, b

    gemm_ms()
    torch.cuda.synchronize()
    # alone
    ga = [gemm_ms() for _ in range(2)]
    torch.cuda.synchronize()
    gemm_alone = sum(a.elapsed_time(b) for a, b in ga) / len(ga)
    ca = [copy_ev() for _ in range(10)]
    torch.cuda.synchronize()
    copy_alone = sorted(a.elapsed_time(b) for a, b in ca)
    # together: copies injected from the host every gap_ms while the GEMMs run
    gt = [gemm_ms() for _ in range(2)]
    ct = []
    t_end = time.perf_counter() + 2 * gemm_alone * 1e-3 * 0.9
    while time.perf_counter() < t_end:
        ct.append(copy_ev())
        time.sleep(gap_ms * 1e-3)
    torch.cuda.synchronize()
    gemm_with = sum(a.elapsed_time(b) for a, b in gt) / len(gt)
    copy_with = sorted(a.elapsed_time(b) for a, b in ct)
    el.SetComputePanel(0)
    gbs = lambda ms: round(2 * copy_mib * (1 << 20) / (ms * 1e-3) / 1e9, 1)
    print(json.dumps({
        "reserved_cus": cus.value,
        "gemm": f"El::Gemm NN f64 n={n}, kc={kc}",
        "gemm_ms_alone": round(gemm_alone, 2),
        "gemm_ms_with_copies": round(gemm_with, 2),
        "gemm_slowdown": round(gemm_with / gemm_alone, 4),
        "gemm_tflops_alone": round(2 * n ** 3 / (gemm_alone * 1e-3) / 1e12, 2),
        "injected": "torch.sum (LDS-using reduction)" if op == "sum" else "device copy",
        "copy_mib": copy_mib,
        "copy_ms_alone_median": round(copy_alone[len(copy_alone) // 2], 3),
        "copy_GBps_alone_median": gbs(copy_alone[len(copy_alone) // 2]),
        "copies_under_gemm": len(copy_with),
        "copy_ms_under_gemm_median": round(copy_with[len(copy_with) // 2], 3),
        "copy_ms_under_gemm_max": round(copy_with[-1], 3),
    }), flush=True)


if __name__ == "__main__":
    main()
