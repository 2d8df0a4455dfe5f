"""One local-kernel shape for counter collection: elx_gemm_<dt> (ta, tb) n^3, 2 launches.

  python tools/prof_gemm.py [f64|f32|bf16|f16] [n] [ta] [tb]
"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L
dt = sys.argv[1] if len(sys.argv) > 1 else "f64"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
ta = int(sys.argv[3]) if len(sys.argv) > 3 else 0
tb = int(sys.argv[4]) if len(sys.argv) > 4 else 0
tdt = {"f64": torch.float64, "f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[dt]
mk = lambda: torch.rand(n * n, dtype=torch.float32, device="cuda").sub_(0.5).to(tdt)
A, B, C = mk(), mk(), mk()
torch.cuda.synchronize()
fn = {"f64": L.lib().elx_gemm_f64, "f32": L.lib().elx_gemm_f32, "bf16": L.lib().elx_gemm_bf16,
      "f16": L.lib().elx_gemm_f16}[dt]
for _ in range(2):
    L.check(fn(ta, tb, n, n, n, 1.0, A.data_ptr(), n, B.data_ptr(), n, 1.0, C.data_ptr(), n, None))
L.call("elx_device_synchronize")
