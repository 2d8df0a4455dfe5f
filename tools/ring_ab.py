"""In-process A/B of the LDS-DMA GEMM kernels against the ring kernels, chosen
per call by ELX_F64G_RING / ELX_F32G_RING (read per call by the library) and
interleaved so that clock drift hits all variants alike.

  python tools/ring_ab.py [dt,ta,tb,m,n,k ...] [--reps 3] [--modes 0,1]

dt f64: modes 0 (slab) / 1 (ring).  dt f32: modes 0 (slab), 1 (128 x 128 ring on
grids of 128-tiles), 2 (64 x 64 ring on grids of 64-tiles), 3 (both).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402
from gemm_bench import timeit  # noqa: E402

SHAPES = ["f64,0,0,32768,32768,32768", "f64,0,0,16384,16384,16384", "f64,1,0,16384,16384,16384",
          "f64,0,1,16384,16384,16384", "f64,1,1,16384,16384,16384", "f64,0,0,4096,4096,4096",
          "f64,0,0,2048,2048,16384", "f64,0,0,2048,2048,2048"]
TD = {"f64": torch.float64, "f32": torch.float32}
ENV = {"f64": "ELX_F64G_RING", "f32": "ELX_F32G_RING"}


def run(spec, reps, modes):
    dt, ta, tb, m, n, k = spec.split(",")
    ta, tb, m, n, k = int(ta), int(tb), int(m), int(n), int(k)
    lda = k if ta else m
    ldb = n if tb else k
    A = torch.rand(lda * (m if ta else k), dtype=TD[dt], device="cuda") - 0.5
    B = torch.rand(ldb * (k if tb else n), dtype=TD[dt], device="cuda") - 0.5
    C = torch.rand(m * n, dtype=TD[dt], device="cuda") - 0.5
    fn = L.lib().elx_gemm_f64 if dt == "f64" else L.lib().elx_gemm_f32
    go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 1.0, C.data_ptr(), m, None))
    res = {v: [] for v in modes}
    for _ in range(reps):
        for v in modes:
            os.environ[ENV[dt]] = v
            res[v].append(2 * m * n * k / timeit(go, 2) / 1e12)
    os.environ.pop(ENV[dt])
    line = f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}:"
    for v in modes:
        line += f"  mode{v} best {max(res[v]):7.2f} mean {sum(res[v]) / reps:7.2f}"
    print(line + " TF", flush=True)
    del A, B, C
    torch.cuda.empty_cache()


if __name__ == "__main__":
    reps, args, modes = 3, [], None
    it = iter(sys.argv[1:])
    for a in it:
        if a == "--reps":
            reps = int(next(it))
        elif a == "--modes":
            modes = next(it).split(",")
        else:
            args.append(a)
    for spec in args or SHAPES:
        run(spec, reps, modes or ["0", "1"])
