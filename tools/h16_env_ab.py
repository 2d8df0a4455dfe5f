"""In-process A/B of one per-call knob of the 16-bit GEMM (any ELX_H16_* the
library reads on every call), interleaved so clock drift hits all arms alike.

  python tools/h16_env_ab.py VAR v1,v2[,...] [--beta B] [--reps R] dt,ta,tb,m,n,k ...
  (values that contain commas themselves: separate them with ';', e.g. "2,8;2,4")

Each line: the shape, TFLOP/s per value (best and mean of R interleaved
rounds, each the best of timeit's repetitions).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402
from gemm_bench import timeit  # noqa: E402

TD = {"f16": torch.float16, "bf16": torch.bfloat16}


def main():
    args = sys.argv[1:]
    var = args[0]
    vals = args[1].split(";") if ";" in args[1] else args[1].split(",")
    beta, reps, shapes = 1.0, 3, []
    it = iter(args[2:])
    for a in it:
        if a == "--beta":
            beta = float(next(it))
        elif a == "--reps":
            reps = int(next(it))
        else:
            shapes.append(a)
    for spec in shapes:
        dt, ta, tb, m, n, k = spec.split(",")
        ta, tb, m, n, k = int(ta), int(tb), int(m), int(n), int(k)
        lda, ldb = (k if ta else m), (n if tb else k)
        A = torch.rand(lda * (m if ta else k), device="cuda").sub_(0.5).to(TD[dt])
        B = torch.rand(ldb * (k if tb else n), device="cuda").sub_(0.5).to(TD[dt])
        C = torch.rand(m * n, device="cuda").sub_(0.5).to(TD[dt])
        fn = L.lib().elx_gemm_bf16 if dt == "bf16" else L.lib().elx_gemm_f16
        go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, beta,  # noqa: E731
                                C.data_ptr(), m, None))
        res = {v: [] for v in vals}
        for _ in range(reps):
            for v in vals:
                os.environ[var] = v
                res[v].append(2.0 * m * n * k / timeit(go, 2) / 1e12)
        os.environ.pop(var, None)
        print(f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k} beta={beta:g}: " +
              "  ".join(f"{var}={v} best {max(res[v]):7.1f} mean {sum(res[v]) / reps:7.1f}" for v in vals) + " TF",
              flush=True)
        del A, B, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
