"""Per-workgroup timeline of the 16-bit four-wave kernel from a diagnostic
build (tools/variant_build.sh stamps ...: s_memrealtime at entry, after the
prologue's first wait, after the K-tile loop, after the epilogue's stores).

  python tools/h16_stamps.py <package root> dt,ta,tb,m,n,k [...]

Prints, per shape, the kernel's span and the distributions (min / median /
max, microseconds) of each phase and of the start and end offsets."""
import ctypes
import os
import sys

import numpy as np

root = sys.argv[1]
sys.path.insert(0, root)
import torch  # noqa: E402
from elemental_amd import _lib as L  # noqa: E402

TD = {"f16": torch.float16, "bf16": torch.bfloat16}
lib = L.lib()
buf = np.zeros((4, 8192), np.uint64)
for spec in sys.argv[2:]:
    dt, ta, tb, m, n, k = spec.split(",")
    ta, tb, m, n, k = int(ta), int(tb), int(m), int(n), int(k)
    lda, ldb = (k if ta else m), (n if tb else k)
    A = torch.rand(lda * (m if ta else k), device="cuda").sub_(0.5).to(TD[dt])
    B = torch.rand(ldb * (k if tb else n), device="cuda").sub_(0.5).to(TD[dt])
    C = torch.zeros(m * n, device="cuda").to(TD[dt])
    fn = lib.elx_gemm_bf16 if dt == "bf16" else lib.elx_gemm_f16
    for _ in range(200):
        L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 0.0, C.data_ptr(), m, None))
    torch.cuda.synchronize()
    lib.elx_h16_stamps(buf.ctypes.data_as(ctypes.c_void_p), 8192)
    nwg = ((m + 255) // 256) * ((n + 255) // 256)
    s = buf[:, :nwg].astype(np.int64)
    t0 = s[0].min()
    us = lambda x: x / 100.0  # noqa: E731  (100 MHz)
    def d(x):
        return f"{us(np.min(x)):7.2f} {us(np.median(x)):7.2f} {us(np.max(x)):7.2f}"
    print(f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}: {nwg} wgs, span {us(s[3].max() - t0):.2f} us", flush=True)
    print("   start offset   ", d(s[0] - t0))
    print("   prologue       ", d(s[1] - s[0]))
    print("   K-tile loop    ", d(s[2] - s[1]))
    print("   epilogue       ", d(s[3] - s[2]))
    print("   end offset     ", d(s[3] - t0))
    xcd = np.arange(nwg) % 8
    print("   end by XCD     ", " ".join(f"{us(np.median(s[3][xcd == x] - t0)):.1f}" for x in range(8)))
    print("   loop by XCD    ", " ".join(f"{us(np.median(s[2][xcd == x] - s[1][xcd == x])):.1f}" for x in range(8)))
