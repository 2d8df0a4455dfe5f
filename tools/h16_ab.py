"""Interleaved in-process A/B of 16-bit GEMM kernel variants (cdna_hip_programming.md
§5.4 rule 24: one process, variants alternated over rounds, median and min).

  python tools/h16_ab.py [--rounds R] [--variants name=KERNEL[:FLAGS],...] dt,ta,tb,m,n,k ...

A variant KERNEL[:FLAGS[:GROUP]] sets ELX_H16_KERNEL / ELX_H16_FLAGS / ELX_H16_GROUP
(read by the library on every call).
Operands are random Uniform(-0.5, 0.5), column-major, beta = 1; every timing is
`inner` back-to-back launches between two syncs after ~0.5 s of warm-up on the
first round.
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from elemental_amd import _lib as L

TD = {"f16": torch.float16, "bf16": torch.bfloat16}


def main():
    args = sys.argv[1:]
    rounds, variants, shapes = 5, "d=d,w=w", []
    while args:
        a = args.pop(0)
        if a == "--rounds":
            rounds = int(args.pop(0))
        elif a == "--variants":
            variants = args.pop(0)
        else:
            shapes.append(a)
    vs = []
    for v in variants.split(","):
        name, spec = v.split("=")
        parts = spec.split(":")
        kern = parts[0]
        fl = parts[1] if len(parts) > 1 and parts[1] else "0"
        grp = parts[2] if len(parts) > 2 and parts[2] else ""   # "" = the library's default
        assert grp == "" or int(grp) >= 1, f"group height must be >= 1: {v}"
        vs.append((name, kern, fl, grp))
    for spec in shapes or ["bf16,1,0,16384,16384,16384"]:
        dt, ta, tb, m, n, k = spec.split(",")
        ta, tb, m, n, k = int(ta), int(tb), int(m), int(n), int(k)
        lda, ldb = (k if ta else m), (n if tb else k)
        A = torch.rand(lda * (m if ta else k), device="cuda").sub_(0.5).to(TD[dt])
        B = torch.rand(ldb * (k if tb else n), device="cuda").sub_(0.5).to(TD[dt])
        C = torch.rand(m * n, device="cuda").sub_(0.5).to(TD[dt])
        fn = L.lib().elx_gemm_bf16 if dt == "bf16" else L.lib().elx_gemm_f16
        go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 1.0, C.data_ptr(), m, None))
        flop = 2.0 * m * n * k
        inner = max(1, int(0.05 / (flop / 1.4e15)))
        res = {v[0]: [] for v in vs}
        for r in range(rounds):
            for name, kern, fl, grp in vs:
                os.environ["ELX_H16_KERNEL"], os.environ["ELX_H16_FLAGS"] = kern, fl
                if grp:
                    os.environ["ELX_H16_GROUP"] = grp
                else:
                    os.environ.pop("ELX_H16_GROUP", None)
                if r == 0:
                    t0 = time.perf_counter()
                    while time.perf_counter() - t0 < 0.5:
                        go()
                        L.call("elx_device_synchronize")
                L.call("elx_device_synchronize")
                t = time.perf_counter()
                for _ in range(inner):
                    go()
                L.call("elx_device_synchronize")
                res[name].append(flop * inner / (time.perf_counter() - t) / 1e12)
        line = f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}:"
        for v in vs:
            name, x = v[0], res[v[0]]
            line += f"  {name} {statistics.median(x):7.1f} (max {max(x):7.1f})"
        print(line, flush=True)
        del A, B, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
