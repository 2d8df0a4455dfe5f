"""Why does f16 run slower than bf16 through the same four-wave kernel?

In one process, interleaved (clock drift hits all arms alike), NN n^3 through
elx_gemm_{bf16,f16} with Uniform(-0.1, 0.1) operands (the bench's range):
  bf16          random bf16 operands (7 stored mantissa bits)
  f16           random f16 operands (10 stored mantissa bits)
  f16_bf16vals  f16 operands holding bf16-representable values (the low three
                mantissa bits zero): the f16 instruction on bf16-like data
  bf16_zero     all-zero bf16 operands (no toggling at all)
MI355X_MICROARCH.md "DVFS give-back": under load the clock follows the energy
per MFMA, which depends on the operand bits; the two MFMA forms take the same
cycles.  If f16_bf16vals runs at bf16's speed, the gap is the data's switching
energy, not the kernel.

  python tools/h16_dtype_ab.py [n] [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5


def operands(kind):
    g = torch.Generator(device="cuda").manual_seed(7)
    mk = lambda: (torch.rand(n * n, generator=g, device="cuda") * 0.2 - 0.1)  # noqa: E731
    if kind == "bf16":
        return [mk().to(torch.bfloat16) for _ in range(3)], L.lib().elx_gemm_bf16
    if kind == "f16":
        return [mk().to(torch.float16) for _ in range(3)], L.lib().elx_gemm_f16
    if kind == "f16_bf16vals":
        return [mk().to(torch.bfloat16).to(torch.float16) for _ in range(3)], L.lib().elx_gemm_f16
    return [torch.zeros(n * n, dtype=torch.bfloat16, device="cuda") for _ in range(3)], L.lib().elx_gemm_bf16


def sustained(go, warm_s=0.5, run_s=1.5):
    """seconds per call over ~run_s of back-to-back calls after warm_s of them
    (the clock under sustained load, as in a long GEMM)"""
    import time
    t = time.perf_counter()
    while time.perf_counter() - t < warm_s:
        go()
        L.call("elx_device_synchronize")
    calls, t = 0, time.perf_counter()
    while time.perf_counter() - t < run_s:
        for _ in range(4):
            go()
        calls += 4
        L.call("elx_device_synchronize")
    return (time.perf_counter() - t) / calls


arms = ["bf16", "f16", "f16_bf16vals", "bf16_zero"]
ops = {a: operands(a) for a in arms}
res = {a: [] for a in arms}
for _ in range(reps):
    for a in arms:
        (A, B, C), fn = ops[a]
        go = lambda: L.check(fn(0, 0, n, n, n, 1.0, A.data_ptr(), n, B.data_ptr(), n, 0.0, C.data_ptr(), n, None))  # noqa: E731
        res[a].append(2.0 * n ** 3 / sustained(go) / 1e12)
line = f"NN {n}^3 beta=0:"
for a in arms:
    line += f"  {a} best {max(res[a]):7.1f} mean {sum(res[a]) / reps:7.1f}"
print(line + " TF", flush=True)
