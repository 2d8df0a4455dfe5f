"""Does the operands' leading dimension move the 16-bit kernel?  NT / TT read
twice NN's fabric bytes at 16384^3 ("Unit order"); if that is an
address-mapping effect of power-of-two strides, padding ld changes it.

In one process, interleaved: bf16 <orient> n^3 with lda = ldb = n + pad for each
pad, beta = 0, sustained timing (1.5 s per arm after 0.5 s of warm-up).

  python tools/h16_ld_ab.py [n] [reps] [orients] [pads]
  e.g. python tools/h16_ld_ab.py 16384 3 NN,NT,TN,TT 0,64,256
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
orients = (sys.argv[3] if len(sys.argv) > 3 else "NN,NT,TN,TT").split(",")
pads = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "0,64,256").split(",")]
fn = L.lib().elx_gemm_bf16


def sustained(go, warm_s=0.5, run_s=1.5):
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


ld_max = n + max(pads)
A = (torch.rand(ld_max * n, device="cuda") * 0.2 - 0.1).to(torch.bfloat16)
B = (torch.rand(ld_max * n, device="cuda") * 0.2 - 0.1).to(torch.bfloat16)
C = torch.zeros(n * n, dtype=torch.bfloat16, device="cuda")
res = {(o, p): [] for o in orients for p in pads}
for _ in range(reps):
    for o in orients:
        ta, tb = int(o[0] == "T"), int(o[1] == "T")
        for p in pads:
            ld = n + p
            go = lambda: L.check(fn(ta, tb, n, n, n, 1.0, A.data_ptr(), ld, B.data_ptr(), ld, 0.0,  # noqa: E731
                                    C.data_ptr(), n, None))
            res[(o, p)].append(2.0 * n ** 3 / sustained(go) / 1e12)
for o in orients:
    print(f"bf16 {o} {n}^3 beta=0: " + "  ".join(f"ld+{p} best {max(res[(o, p)]):7.1f} mean "
                                               f"{sum(res[(o, p)]) / reps:7.1f}" for p in pads) + " TF", flush=True)
