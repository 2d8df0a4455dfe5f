"""El::Trsm on one MI355X (Grid 1x1, DistMatrix API).

  python tools/trsm_bench.py [m] [n] [dtype] [blocksize ...]

LEFT solves op(A) X = B with A m x m and n right-hand sides: m^2 n algorithmic
FLOPs.  One line per (uplo, orientation) and block size.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elemental_amd import el
from elemental_amd import _lib as L


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    dt = {"f64": el.F64, "f32": el.F32}[sys.argv[3] if len(sys.argv) > 3 else "f64"]
    nbs = [int(x) for x in sys.argv[4:]] or [128]
    g = el.Grid()
    A = el.DistMatrix(g, dt, height=m, width=m).fill_hash(1, 0.0, 0.01)
    # a dominant diagonal keeps the solve well conditioned: A += 2 I
    D = el.DistMatrix(g, dt, height=m, width=m)
    B0 = el.DistMatrix(g, dt, height=m, width=n).fill_hash(2, -1.0, 1.0)
    B = el.DistMatrix(g, dt, height=m, width=n)
    import numpy as np
    d = np.zeros((m, m), dtype=np.float64 if dt == el.F64 else np.float32)
    np.fill_diagonal(d, 2.0)
    D.set_local(d)
    el.Axpy(1.0, D, A)
    for nb in nbs:
        el.SetBlocksize(nb)
        for uplo in (el.LOWER, el.UPPER):
            for orient in (el.NORMAL, el.TRANSPOSE):
                best = 1e30
                for _ in range(3):
                    B.assign(B0)
                    L.call("elx_device_synchronize")
                    t = time.perf_counter()
                    el.Trsm(el.LEFT, uplo, orient, el.NON_UNIT, 1.0, A, B)
                    L.call("elx_device_synchronize")
                    best = min(best, time.perf_counter() - t)
                print(f"Trsm L{'LU'[uplo]}{'NT'[orient]} m={m} n={n} nb={nb}: {m*m*n/best/1e12:7.2f} TFLOP/s "
                      f"({best*1e3:.1f} ms)", flush=True)


if __name__ == "__main__":
    main()
