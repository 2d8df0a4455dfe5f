"""Where do the NaNs of gemm_suite under ELX_POOL_CACHE=0 come from?  Replays the
suite's SUMMA_A / SUMMA_C experiment (300 x 260 x 520, nb 64, one rank) and its
associativity check step by step through el.py, checking each intermediate for
non-finite entries and the product against the oracle.

  ELX_POOL_CACHE=0 [ELX_POOL_RELEASE_THRESHOLD=0] python tools/pool_nan_debug.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from elemental_amd import el  # noqa: E402


def bad(name, M):
    a = M.get_local()
    n = int(np.count_nonzero(~np.isfinite(a)))
    print(f"    {name}: {a.shape} non-finite {n}", flush=True)
    return a


def main():
    g = el.Grid()
    m, n, k = 300, 260, 520
    el.SetBlocksize(64)
    for alg_name in ("SUMMA_A", "SUMMA_C", "SUMMA_B", "DEFAULT"):
        alg = getattr(el, "GEMM_" + alg_name)
        print(f"== {alg_name}", flush=True)
        A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=k).fill_hash(1, -0.1, 0.1)
        B = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=k, width=n).fill_hash(2, -0.1, 0.1)
        CO = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=n).fill_hash(3, -0.1, 0.1)
        for warm in range(3):
            C = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU)
            el.Copy(CO, C)
            el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, B, -0.5, C, alg)
            c = bad(f"warm {warm} C", C)
            ref = oracle.gemm("N", "N", 0.5, A.get_local(), B.get_local(), -0.5, CO.get_local())
            print(f"    warm {warm} max |C - ref| = {np.nanmax(np.abs(c - ref)):.3e}", flush=True)
            el.InitializeRandom()
            X = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU)
            Y = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU)
            Z = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU)
            el.Uniform(X, n, 100, -0.25, 0.25)
            bad("X", X)
            Z.Resize(k, 100)
            Y.Resize(m, 100)
            el.Gemm(el.NORMAL, el.NORMAL, 1.0, B, X, 0.0, Z, el.GEMM_DEFAULT)
            bad("Z = B X", Z)
            el.Gemm(el.NORMAL, el.NORMAL, 0.5, A, Z, 0.0, Y, el.GEMM_DEFAULT)
            bad("Y = a A Z", Y)
            el.Gemm(el.NORMAL, el.NORMAL, -0.5, CO, X, 1.0, Y, el.GEMM_DEFAULT)
            bad("Y += b CO X", Y)
            el.Gemm(el.NORMAL, el.NORMAL, -1.0, C, X, 1.0, Y, el.GEMM_DEFAULT)
            y = bad("Y -= C X", Y)
            print(f"    warm {warm} residual {np.linalg.norm(y):.3e}", flush=True)
            del X, Y, Z, C


if __name__ == "__main__":
    main()
