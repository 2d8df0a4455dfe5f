"""Schedule-knob sweep of the f64 NN local kernel (ELX_GEMM_FLAGS, see gemm_mfma.hip KF_*).
Each variant runs in its own process (the env var is read once per process)."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, os, time
sys.path.insert(0, %r)
import torch
from elemental_amd import _lib as L
for (m, n, k) in [(16384, 16384, 16384), (32768, 16384, 4096), (32768, 32768, 8192)]:
    A = torch.rand(m * k, dtype=torch.float64, device="cuda") - 0.5
    B = torch.rand(k * n, dtype=torch.float64, device="cuda") - 0.5
    C = torch.rand(m * n, dtype=torch.float64, device="cuda") - 0.5
    go = lambda: L.check(L.lib().elx_gemm_f64(0, 0, m, n, k, 1.0, A.data_ptr(), m, B.data_ptr(), k, 1.0, C.data_ptr(), m, None))
    go(); L.call("elx_device_synchronize")
    best = 1e9
    for _ in range(3):
        t = time.perf_counter(); go(); go(); L.call("elx_device_synchronize"); best = min(best, (time.perf_counter() - t) / 2)
    print(f"flags=%s NN {m}x{n}x{k}: {2*m*n*k/best/1e12:.2f} TFLOP/s", flush=True)
    del A, B, C
'''
for f in sys.argv[1:] or ["0", "1", "2", "3", "4", "5", "7"]:
    env = dict(os.environ, ELX_GEMM_FLAGS=f, ELX_F64G_FLAGS=f.split(":")[0])
    if ":" in f:
        env["ELX_F64G_BM"] = f.split(":")[1]
    subprocess.run([sys.executable, "-c", code % (ROOT, f)], env=env, check=True)
