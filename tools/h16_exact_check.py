"""Exact-integer check of a (variant) library's 16-bit GEMM, for A/B builds that
the test suite cannot import (tools/variant_build.sh trees):

  python tools/h16_exact_check.py <package root> [m,n,k ...]

Integer operands in [-2, 2]: every partial sum is exact in f32, so the result
must equal numpy's rounding of the exact value bit for bit (as
tests/test_gpu_kernels.py::test_local_gemm_16bit_exact), all four orientations,
bf16 and f16.  Prints one line per case and exits non-zero on any mismatch.
Exact for every k whose tail the kernel takes itself (k % 8 == 0, or both
operands rows-contiguous); otherwise a second pass adds the tail to the
already rounded C ("Exactness and the k tail").
"""
import os
import sys

root = sys.argv[1]
sys.path.insert(0, root)
sys.path.insert(1, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from elemental_amd import _lib as L  # noqa: E402

print("library:", L.LIB_PATH, flush=True)
shapes = [tuple(int(x) for x in s.split(",")) for s in sys.argv[2:]] or [(2048, 2312, 2112), (4096, 4096, 640)]
bad_total = 0
for m, n, k in shapes:
    for ta in "NT":
        for tb in "NT":
            for kind in ("bf16", "f16"):
                rng = np.random.default_rng(m + n + k)
                A = rng.integers(-2, 3, (m, k) if ta == "N" else (k, m)).astype(np.float32)
                B = rng.integers(-2, 3, (k, n) if tb == "N" else (n, k)).astype(np.float32)
                C = rng.integers(-64, 65, (m, n)).astype(np.float32)
                opA = A if ta == "N" else A.T
                opB = B if tb == "N" else B.T
                exact = (opA.astype(np.float64) @ opB.astype(np.float64)) - 2.0 * C
                if kind == "f16":
                    enc = lambda x: x.astype(np.float16).view(np.uint16)  # noqa: E731
                    fn, want = L.lib().elx_gemm_f16, exact.astype(np.float16).view(np.uint16)
                else:
                    enc = lambda x: oracle.f32_to_bf16_bits(x)  # noqa: E731
                    fn, want = L.lib().elx_gemm_bf16, oracle.f32_to_bf16_bits(exact.astype(np.float32))
                # column-major bytes on the device (as tests/test_gpu_kernels.py dev / host)
                dev = lambda x: torch.from_numpy(np.ravel(np.asfortranarray(x), order="F").view(np.int16).copy()).cuda()  # noqa: E731
                dA, dB, dC = dev(enc(A)), dev(enc(B)), dev(enc(C))
                torch.cuda.synchronize()
                L.check(fn(int(ta == "T"), int(tb == "T"), m, n, k, 1.0, dA.data_ptr(), A.shape[0], dB.data_ptr(),
                           B.shape[0], -2.0, dC.data_ptr(), m, None))
                L.call("elx_device_synchronize")
                got = dC.cpu().numpy().view(np.uint16).reshape((m, n), order="F")
                bad = int(np.count_nonzero(got != want))
                bad_total += bad
                print(f"{kind} {ta}{tb} {m}x{n}x{k}: {bad} mismatches", flush=True)
sys.exit(1 if bad_total else 0)
