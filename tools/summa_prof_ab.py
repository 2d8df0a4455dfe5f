"""SUMMA_C on one GPU with the panels COPIED through the comm stream
(ELX_SUMMA_COPY=1: the N > 1 pipeline's stream pattern, minus RCCL): wall
time per El::Gemm with the library's event profiling on and off, interleaved
in one process.  NN f64, n = 32768, compute panel 4096 (8 panels)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elemental_amd import el
from elemental_amd import _lib as L

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
g = el.Grid()
el.SetComputePanel(4096)
A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(1, 0.0, 0.1)
B = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(2, 0.0, 0.1)
C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=n, width=n).fill_hash(3, 0.0, 0.1)
el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)
el.device_synchronize()
for rep in range(3):
    for prof in (1, 0):
        L.call("elx_set_profiling", prof)
        t = time.perf_counter()
        el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)
        el.device_synchronize()
        dt = time.perf_counter() - t
        L.call("elx_set_profiling", 0)
        print(f"copy={os.environ.get('ELX_SUMMA_COPY', '0')} profiling={prof}: {dt * 1e3:.1f} ms  "
              f"{2.0 * n ** 3 / dt / 1e12:.2f} TFLOP/s", flush=True)
