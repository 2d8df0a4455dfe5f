"""El::Syrk vs El::Gemm on one MI355X (Grid 1x1, DistMatrix API).

  python tools/syrk_bench.py [n] [k] [dtype]

Syrk's algorithmic FLOPs are n(n+1)k (one triangle of the product); the same
C := alpha A A^T + beta C through El::Gemm costs 2 n^2 k.  Reports both rates and
the Syrk-vs-Gemm wall-time ratio (ideal 0.5 + strip overhead ~ TrrkCols/n).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from elemental_amd import el
from elemental_amd import _lib as L


def best(go, reps=3):
    go()
    L.call("elx_device_synchronize")
    t_best = 1e30
    for _ in range(reps):
        t = time.perf_counter()
        go()
        L.call("elx_device_synchronize")
        t_best = min(t_best, time.perf_counter() - t)
    return t_best


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    dt = {"f64": el.F64, "f32": el.F32}[sys.argv[3] if len(sys.argv) > 3 else "f64"]
    g = el.Grid()
    for orient in (el.NORMAL, el.TRANSPOSE):
        shape = (n, k) if orient == el.NORMAL else (k, n)
        A = el.DistMatrix(g, dt, height=shape[0], width=shape[1]).fill_hash(1, -0.1, 0.1)
        C = el.DistMatrix(g, dt, height=n, width=n).fill_hash(3, -0.1, 0.1)
        for uplo in (el.LOWER, el.UPPER):
            ts = best(lambda: el.Syrk(uplo, orient, 0.5, A, 1.0, C))
            print(f"Syrk {'LU'[uplo]}{'NT'[orient]} n={n} k={k}: {n*(n+1)*k/ts/1e12:7.2f} TFLOP/s "
                  f"({ts*1e3:.1f} ms)", flush=True)
        oB = el.TRANSPOSE if orient == el.NORMAL else el.NORMAL
        tg = best(lambda: el.Gemm(orient, oB, 0.5, A, A, 1.0, C, el.GEMM_SUMMA_C))
        print(f"Gemm {'NT'[orient]}{'NT'[oB]} same product: {2*n*n*k/tg/1e12:7.2f} TFLOP/s ({tg*1e3:.1f} ms); "
              f"Syrk/Gemm time {ts/tg:.3f}", flush=True)


if __name__ == "__main__":
    main()
