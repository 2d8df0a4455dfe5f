"""BLAS-1 / data-movement kernels against the HBM roofline (config C5 local block).

  python tools/blas1_bench.py [m n]      (default 16384 x 8192 = one rank's [MC,MR]
                                          block of an n = 32768 matrix on a 2x4 grid)

Algorithmic bytes per element: axpy 3s (read X, Y; write Y),
hadamard 3s, scale 2s, copy 2s, transpose 2s, fill 1s, map 2s.  Each kernel is
timed with HIP events on its own stream over 20 launches after a warm-up.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L

HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md (6.29 TB/s measured float4 copy)
m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
DT = [("f64", L.F64, torch.float64, 8), ("f32", L.F32, torch.float32, 4), ("bf16", L.BF16, torch.bfloat16, 2),
      ("f16", L.F16, torch.float16, 2)]
stream = torch.cuda.Stream()
sp = stream.cuda_stream


def timed(fn, reps=20):
    with torch.cuda.stream(stream):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


for name, dt, tdt, es in DT:
    X = torch.rand(m * n, dtype=torch.float32, device="cuda").to(tdt)
    Y = torch.rand(m * n, dtype=torch.float32, device="cuda").to(tdt)
    Z = torch.empty(m * n, dtype=tdt, device="cuda")
    torch.cuda.synchronize()
    x, y, z = X.data_ptr(), Y.data_ptr(), Z.data_ptr()
    ops = {
        "axpy": (3, lambda: L.check(L.lib().elx_axpy2d(dt, m, n, 0.5, x, 1, m, y, 1, m, sp))),
        "hadamard": (3, lambda: L.check(L.lib().elx_hadamard2d(dt, m, n, x, m, y, m, z, m, sp))),
        "scale": (2, lambda: L.check(L.lib().elx_scale2d(dt, m, n, 1.0, y, m, sp))),
        "copy": (2, lambda: L.check(L.lib().elx_copy2d(dt, m, n, x, 1, m, z, 1, m, sp))),
        "transpose": (2, lambda: L.check(L.lib().elx_transpose(dt, m, n, x, m, z, n, sp))),
        "fill": (1, lambda: L.check(L.lib().elx_fill2d(dt, m, n, 0.25, z, m, sp))),
        "map(relu)": (2, lambda: L.check(L.lib().elx_entrywise_map(dt, 7, m, n, x, m, z, m, sp))),
    }
    for op, (mult, fn) in ops.items():
        t = timed(fn)
        gbs = mult * es * m * n / t
        print(f"{name:5s} {op:10s} {m}x{n}: {t*1e3:8.3f} ms  {gbs/1e9:8.1f} GB/s  {100*gbs/HBM_PEAK:5.1f}% of 8 TB/s",
              flush=True)
    # vendor reference point: torch's own elementwise kernels on the same buffers
    with torch.cuda.stream(stream):
        t = timed(lambda: Y.add_(X, alpha=0.5))
    print(f"{name:5s} {'torch.add_':10s} {m}x{n}: {t*1e3:8.3f} ms  {3*es*m*n/t/1e9:8.1f} GB/s  (vendor reference)",
          flush=True)
    del X, Y, Z
