"""Debug the buffer-descriptor staging (ELX_F64G_FLAGS=16): small NN GEMMs vs numpy."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from elemental_amd import _lib as L
for (m, n, k) in [(256, 256, 32), (256, 256, 16), (1024, 1024, 64), (3000, 2900, 100)]:
    A = np.random.rand(m, k); B = np.random.rand(k, n); C = np.zeros((m, n))
    dA = torch.tensor(A.T.copy().ravel(), device="cuda"); dB = torch.tensor(B.T.copy().ravel(), device="cuda")
    dC = torch.zeros(m * n, dtype=torch.float64, device="cuda")
    L.check(L.lib().elx_gemm_f64(0, 0, m, n, k, 1.0, dA.data_ptr(), m, dB.data_ptr(), k, 1.0, dC.data_ptr(), m, None))
    L.call("elx_device_synchronize")
    got = dC.cpu().numpy().reshape(n, m).T
    want = A @ B
    bad = ~np.isclose(got, want)
    print(m, n, k, "bad", bad.sum(), "nan", np.isnan(got).sum())
    if bad.any():
        idx = np.argwhere(bad)[:5]
        for i, j in idx: print("  ", i, j, got[i, j], want[i, j])
        # is the error = missing k-slabs? compare with partial sums
        for s in range(0, k, 16):
            part = A[:, :s + 16] @ B[:s + 16, :]
            if np.allclose(got[:8, :8], part[:8, :8]): print("  matches partial k <", s + 16)
