"""One local-kernel shape for counter collection: elx_gemm_<dt> (ta, tb) n^3.

  python tools/prof_gemm.py [f64|f32|bf16|f16] [n] [ta] [tb] [reps] [--vendor]

reps launches (default 2) after a ~1 s warm-up on the same operands (so the
clock has settled when the counted launches run); --vendor times torch.matmul
(hipBLASLt) on the same column-major problem instead, for side-by-side counters.
"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L
args = [a for a in sys.argv[1:] if not a.startswith("--")]
vendor = "--vendor" in sys.argv
dt = args[0] if len(args) > 0 else "f64"
n = int(args[1]) if len(args) > 1 else 16384
ta = int(args[2]) if len(args) > 2 else 0
tb = int(args[3]) if len(args) > 3 else 0
reps = int(args[4]) if len(args) > 4 else 2
tdt = {"f64": torch.float64, "f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[dt]
mk = lambda: torch.rand(n * n, dtype=torch.float32, device="cuda").sub_(0.5).to(tdt)
A, B, C = mk(), mk(), mk()
torch.cuda.synchronize()
if vendor:
    At, Bt = A.view(n, n), B.view(n, n)   # row-major views of column-major storage
    opA = At if ta else At.t()
    opB = Bt if tb else Bt.t()
    Cv = torch.empty(n, n, dtype=tdt, device="cuda")
    go = lambda: torch.matmul(opA, opB, out=Cv)
else:
    fn = {"f64": L.lib().elx_gemm_f64, "f32": L.lib().elx_gemm_f32, "bf16": L.lib().elx_gemm_bf16,
          "f16": L.lib().elx_gemm_f16}[dt]
    go = lambda: L.check(fn(ta, tb, n, n, n, 1.0, A.data_ptr(), n, B.data_ptr(), n, 1.0, C.data_ptr(), n, None))
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:
    go()
    torch.cuda.synchronize()
    L.call("elx_device_synchronize")
for _ in range(reps):
    go()
torch.cuda.synchronize()
L.call("elx_device_synchronize")
