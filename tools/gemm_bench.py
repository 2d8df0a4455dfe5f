"""Local-kernel microbenchmark: elx_gemm_{f64,f32,f16,bf16} on device buffers (no SUMMA).

  python tools/gemm_bench.py [dt,ta,tb,m,n,k ...] [--vendor]

Random Uniform(-0.5, 0.5) operands (column-major), beta = 1; each timing is the best
of 3 runs of back-to-back calls (launch latency amortised).  --vendor also
times torch.matmul (hipBLASLt) on the same shape as a reference point, and ours
at beta = 0 beside it (the vendor call's C = op(A) op(B) reads no C).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L

TD = {"f64": torch.float64, "f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}
DEFAULT = ["f64,0,0,16384,16384,16384", "f64,0,0,32768,16384,4096", "f32,0,0,16384,16384,16384",
           "f64,1,0,2000,2000,524288", "f32,1,0,2000,2000,524288",
           "bf16,0,0,8192,8192,8192", "bf16,1,0,8192,8192,8192", "f16,0,0,8192,8192,8192"]


def timeit(go, reps):
    """Best of `reps` timings of `inner` back-to-back calls (inner sized to fill
    ~30 ms, so launch and sync latency do not count for small shapes); returns
    seconds per call."""
    go()
    torch.cuda.synchronize()
    L.call("elx_device_synchronize")
    t = time.perf_counter()
    go()
    L.call("elx_device_synchronize")
    torch.cuda.synchronize()
    inner = max(1, min(200, int(0.03 / max(time.perf_counter() - t, 1e-6))))
    best = 1e30
    for _ in range(reps):
        t = time.perf_counter()
        for _ in range(inner):
            go()
        L.call("elx_device_synchronize")
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / inner)
    return best


def run(dt, ta, tb, m, n, k, vendor, reps=3):
    tdt = TD[dt]
    lda = k if ta else m
    ldb = n if tb else k
    A = torch.rand(lda * (m if ta else k), dtype=torch.float32, device="cuda").sub_(0.5).to(tdt)
    B = torch.rand(ldb * (k if tb else n), dtype=torch.float32, device="cuda").sub_(0.5).to(tdt)
    C = torch.rand(m * n, dtype=torch.float32, device="cuda").sub_(0.5).to(tdt)
    if dt in ("f64", "f32"):
        fn = L.lib().elx_gemm_f64 if dt == "f64" else L.lib().elx_gemm_f32
        go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 1.0, C.data_ptr(), m, None))
    else:
        fn = L.lib().elx_gemm_bf16 if dt == "bf16" else L.lib().elx_gemm_f16
        go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 1.0, C.data_ptr(), m, None))
    t = timeit(go, reps)
    line = f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}: {2*m*n*k/t/1e12:8.2f} TFLOP/s ({t*1e3:.2f} ms)"
    if vendor:
        # torch.matmul(out=) is C = op(A) op(B), beta = 0 (no C read): ours likewise beside it
        go0 = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 0.0, C.data_ptr(), m,
                                 None))
        t0 = timeit(go0, reps)
        line += f"   beta=0 {2*m*n*k/t0/1e12:8.2f}"
        # same column-major problem through torch (row-major views): C^T = op(B)^T op(A)^T
        At = A.view(m if ta else k, lda)  # row-major view of column-major A: At[c, r] = A(r, c)
        Bt = B.view(k if tb else n, ldb)
        opA = At if ta else At.t()       # op(A) as an m x k view
        opB = Bt if tb else Bt.t()
        Cv = torch.empty(m, n, dtype=tdt, device="cuda")
        tv = timeit(lambda: torch.matmul(opA, opB, out=Cv), reps)
        line += f"   vendor torch.matmul {2*m*n*k/tv/1e12:8.2f} TFLOP/s"
    print(line, flush=True)
    del A, B, C


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    vendor = "--vendor" in sys.argv
    for spec in args or DEFAULT:
        d, ta, tb, m, n, k = spec.split(",")
        run(d, int(ta), int(tb), int(m), int(n), int(k), vendor)
