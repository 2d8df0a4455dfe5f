"""Per-call latency of El::Gemm on a 1x1 grid at small sizes (host overhead of
the SUMMA machinery) vs the bare local kernel entry elx_gemm_f64, both through
ctypes, 200 back-to-back calls each, one MI355X."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elemental_amd import el
from elemental_amd import _lib as L

g = el.Grid()
for n in (128, 256, 512, 1024, 2048):
    A = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(1, -0.1, 0.1)
    B = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(2, -0.1, 0.1)
    C = el.DistMatrix(g, el.F64, height=n, width=n).fill_hash(3, -0.1, 0.1)
    for name, fn in (("El::Gemm", lambda: el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C)),
                     ("elx_gemm_f64", lambda: L.call("elx_gemm_f64", 0, 0, n, n, n, 0.5, A.Buffer(), n, B.Buffer(), n,
                                                     -0.5, C.Buffer(), n, None))):
        for _ in range(10):
            fn()
        el.device_synchronize()
        t = time.perf_counter()
        for _ in range(200):
            fn()
        el.device_synchronize()
        dt = (time.perf_counter() - t) / 200
        print(f"n={n:5d} {name:13s} {dt * 1e6:9.1f} us/call  {2.0 * n ** 3 / dt / 1e12:7.2f} TFLOP/s", flush=True)
