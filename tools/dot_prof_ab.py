"""C4 (SUMMA_DOT, TN f32 8192^2 x 524288, [VC,STAR]) on one GPU: wall time per
El::Gemm with the library's event profiling on and off, interleaved in one
process (the overlap mode is ELX_DOT_OVERLAP in the environment)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elemental_amd import el
from elemental_amd import _lib as L

g = el.Grid()
k, m = 524288, 8192
A = el.DistMatrix(g, el.F32, el.VC, el.STAR, el.GPU, height=k, width=m).fill_hash(1, 0.0, 0.1)
B = el.DistMatrix(g, el.F32, el.VC, el.STAR, el.GPU, height=k, width=m).fill_hash(2, 0.0, 0.1)
C = el.DistMatrix(g, el.F32, el.MC, el.MR, el.GPU, height=m, width=m).fill_hash(3, 0.0, 0.1)
el.Gemm(el.TRANSPOSE, el.NORMAL, 0.5, A, B, -0.5, C)
el.device_synchronize()
for rep in range(3):
    for prof in (1, 0):
        L.call("elx_set_profiling", prof)
        t = time.perf_counter()
        el.Gemm(el.TRANSPOSE, el.NORMAL, 0.5, A, B, -0.5, C)
        el.device_synchronize()
        dt = time.perf_counter() - t
        L.call("elx_set_profiling", 0)
        print(f"overlap={os.environ.get('ELX_DOT_OVERLAP', '1')} profiling={prof}: {dt * 1e3:.1f} ms  "
              f"{2.0 * m * m * k / dt / 1e12:.1f} TFLOP/s", flush=True)
