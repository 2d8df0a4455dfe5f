"""Effect of the leading-dimension padding on the local kernel (power-of-two ld vs padded)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L
def run(n, pad, dt="f64", reps=3):
    tdt = torch.float64 if dt == "f64" else torch.float32
    ld = n + pad
    A = torch.rand(ld * n, dtype=tdt, device="cuda"); B = torch.rand(ld * n, dtype=tdt, device="cuda")
    C = torch.rand(ld * n, dtype=tdt, device="cuda"); torch.cuda.synchronize()
    fn = L.lib().elx_gemm_f64 if dt == "f64" else L.lib().elx_gemm_f32
    go = lambda: L.check(fn(0, 0, n, n, n, 1.0, A.data_ptr(), ld, B.data_ptr(), ld, 1.0, C.data_ptr(), ld, None))
    go(); L.call("elx_device_synchronize"); t = time.perf_counter()
    for _ in range(reps): go()
    L.call("elx_device_synchronize"); d = (time.perf_counter() - t) / reps
    print(f"{dt} n={n} ld=n+{pad}: {2*n**3/d/1e12:.2f} TFLOP/s", flush=True)
for r in range(2):
    for pad in (0, 16, 32, 64, 128, 512):
        run(16384, pad)
    run(32768, 0); run(32768, 32); run(32768, 128)
    run(16384, 0, "f32"); run(16384, 32, "f32")
