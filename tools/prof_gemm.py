"""One local-kernel shape for counter collection: elx_gemm_f64 NN 16384^3, 2 launches."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L
dt = sys.argv[1] if len(sys.argv) > 1 else "f64"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
tdt = torch.float64 if dt == "f64" else torch.float32
A = torch.rand(n * n, dtype=tdt, device="cuda"); B = torch.rand(n * n, dtype=tdt, device="cuda")
C = torch.rand(n * n, dtype=tdt, device="cuda"); torch.cuda.synchronize()
fn = L.lib().elx_gemm_f64 if dt == "f64" else L.lib().elx_gemm_f32
for _ in range(2):
    L.check(fn(0, 0, n, n, n, 1.0, A.data_ptr(), n, B.data_ptr(), n, 1.0, C.data_ptr(), n, None))
L.call("elx_device_synchronize")
