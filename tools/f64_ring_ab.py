"""In-process A/B of the fp64 kernels on 128-tile grids: the two-stage slab
kernel (ELX_F64G_RING=0) against the ring kernel (ELX_F64G_RING=1), read per
call by the library, interleaved.

  python tools/f64_ring_ab.py [ta,tb,m,n,k ...] [--reps 3]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402
from gemm_bench import timeit  # noqa: E402

SHAPES = ["0,0,32768,32768,32768", "0,0,16384,16384,16384", "1,0,16384,16384,16384", "0,1,16384,16384,16384",
          "1,1,16384,16384,16384", "0,0,4096,4096,4096", "0,0,2048,2048,16384", "0,0,2048,2048,2048"]


def run(spec, reps):
    ta, tb, m, n, k = (int(x) for x in spec.split(","))
    lda = k if ta else m
    ldb = n if tb else k
    A = torch.rand(lda * (m if ta else k), dtype=torch.float64, device="cuda") - 0.5
    B = torch.rand(ldb * (k if tb else n), dtype=torch.float64, device="cuda") - 0.5
    C = torch.rand(m * n, dtype=torch.float64, device="cuda") - 0.5
    go = lambda: L.check(L.lib().elx_gemm_f64(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 1.0,
                                              C.data_ptr(), m, None))
    res = {"0": [], "1": []}
    for _ in range(reps):
        for v in res:
            os.environ["ELX_F64G_RING"] = v
            res[v].append(2 * m * n * k / timeit(go, 2) / 1e12)
    os.environ.pop("ELX_F64G_RING")
    print(f"f64 {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}: slab best {max(res['0']):6.2f} mean "
          f"{sum(res['0']) / reps:6.2f}   ring best {max(res['1']):6.2f} mean {sum(res['1']) / reps:6.2f} TF",
          flush=True)
    del A, B, C
    torch.cuda.empty_cache()


if __name__ == "__main__":
    reps, args = 3, []
    it = iter(sys.argv[1:])
    for a in it:
        if a == "--reps":
            reps = int(next(it))
        else:
            args.append(a)
    for spec in args or SHAPES:
        run(spec, reps)
