"""Local-kernel microbenchmark: elx_gemm_{f64,f32} on device tensors (no SUMMA)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L

def run(dt, ta, tb, m, n, k, reps=3):
    tdt = torch.float64 if dt == "f64" else torch.float32
    A = (torch.rand((k, m) if ta else (m, k), dtype=tdt, device="cuda") - 0.5).t().contiguous().t() if False else None
    # column-major buffers: allocate flat and pass leading dims
    lda = k if ta else m; ldb = n if tb else k
    A = torch.rand(lda * (m if ta else k), dtype=tdt, device="cuda") - 0.5
    B = torch.rand(ldb * (k if tb else n), dtype=tdt, device="cuda") - 0.5
    C = torch.rand(m * n, dtype=tdt, device="cuda") - 0.5
    fn = L.lib().elx_gemm_f64 if dt == "f64" else L.lib().elx_gemm_f32
    torch.cuda.synchronize()
    def go():
        L.check(fn(int(ta), int(tb), m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 1.0, C.data_ptr(), m, None))
    go(); L.call("elx_device_synchronize")
    t = time.perf_counter()
    for _ in range(reps): go()
    L.call("elx_device_synchronize")
    dtm = (time.perf_counter() - t) / reps
    print(f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}: {2*m*n*k/dtm/1e12:.2f} TFLOP/s ({dtm*1e3:.2f} ms)", flush=True)

for args in [("f64",0,0,8192,8192,8192), ("f64",0,0,16384,16384,16384), ("f64",0,1,16384,16384,16384),
             ("f64",1,0,16384,16384,16384), ("f64",1,1,16384,16384,16384),
             ("f64",0,0,32768,16384,2048), ("f64",0,0,32768,32768,32768),
             ("f32",0,0,16384,16384,16384), ("f64",1,0,2000,2000,524288)]:
    run(*args)
