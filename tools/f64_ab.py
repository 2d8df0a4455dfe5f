"""A/B of the two fp64 (or fp32: --f32) local kernels (ELX_F64_KERNEL /
ELX_F32_KERNEL = reg|dma), each in its own process, same shapes/data; prints
TFLOP/s and a sanity residual against torch.matmul
(||C - C_vendor||_F / (||A|| ||B|| k eps))."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, time
sys.path.insert(0, %r)
import torch
from elemental_amd import _lib as L
kind = %r
dt = %r
tdt = torch.float64 if dt == 'f64' else torch.float32
fn = L.lib().elx_gemm_f64 if dt == 'f64' else L.lib().elx_gemm_f32
eps = 2.0 ** -52 if dt == 'f64' else 2.0 ** -23
for (ta, tb, m, n, k) in [(0, 0, 16384, 16384, 16384), (0, 0, 32768, 16384, 4096), (1, 0, 16384, 16384, 16384),
                          (0, 1, 16384, 16384, 16384), (1, 1, 16384, 16384, 16384), (0, 0, 32768, 32768, 8192),
                          (0, 0, 8200, 8192, 4100)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    lda = k if ta else m; ldb = n if tb else k
    A = torch.rand(lda * (m if ta else k), dtype=tdt, device="cuda", generator=g) - 0.5
    B = torch.rand(ldb * (k if tb else n), dtype=tdt, device="cuda", generator=g) - 0.5
    C = torch.zeros(m * n, dtype=tdt, device="cuda")
    go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 0.0, C.data_ptr(), m, None))
    go(); L.call("elx_device_synchronize")
    best = 1e9
    for _ in range(3):
        t = time.perf_counter(); go(); go(); L.call("elx_device_synchronize"); best = min(best, (time.perf_counter() - t) / 2)
    At = A.view(m if ta else k, lda); Bt = B.view(k if tb else n, ldb)
    ref = (At if ta else At.t()) @ (Bt if tb else Bt.t())          # m x n
    got = C.view(n, m).t()
    r = ((got - ref).norm() / (A.norm() * B.norm() * k * eps)).item()
    print(f"{dt} {kind} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}: {2*m*n*k/best/1e12:.2f} TFLOP/s  resid {r:.2e}", flush=True)
    del A, B, C, ref
'''
dt = "f32" if "--f32" in sys.argv else "f64"
for kind in [a for a in sys.argv[1:] if not a.startswith("--")] or ["reg", "dma"]:
    env = dict(os.environ, ELX_F64_KERNEL=kind, ELX_F32_KERNEL=kind)
    subprocess.run([sys.executable, "-c", code % (ROOT, kind, dt)], env=env, check=True)
