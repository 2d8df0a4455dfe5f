"""In-process A/B of the 16-bit kernel's workgroup -> tile order: the grouped
order (ELX_H16_MAP=0) against super-block orders (ELX_H16_MAP=1 with
ELX_H16_SB = "xr,pr" geometries), interleaved so that clock drift hits all alike.

  python tools/h16_map_ab.py [dt,ta,tb,m,n,k ...] [--reps 4] [--sb 2,8 1,8 ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402
from gemm_bench import timeit  # noqa: E402

SHAPES = ["bf16,0,0,32768,32768,32768", "bf16,1,0,16384,16384,16384", "bf16,0,0,16384,16384,16384",
          "f16,0,0,32768,32768,32768"]
TD = {"f16": torch.float16, "bf16": torch.bfloat16}


def run(spec, reps, maps):
    dt, ta, tb, m, n, k = spec.split(",")
    ta, tb, m, n, k = int(ta), int(tb), int(m), int(n), int(k)
    tdt = TD[dt]
    lda = k if ta else m
    ldb = n if tb else k
    A = torch.rand(lda * (m if ta else k), device="cuda").sub_(0.5).to(tdt)
    B = torch.rand(ldb * (k if tb else n), device="cuda").sub_(0.5).to(tdt)
    C = torch.rand(m * n, device="cuda").sub_(0.5).to(tdt)
    fn = L.lib().elx_gemm_bf16 if dt == "bf16" else L.lib().elx_gemm_f16
    go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, 1.0, C.data_ptr(), m, None))
    res = {mp: [] for mp in maps}
    for _ in range(reps):
        for mp in maps:
            if mp == "0":
                os.environ["ELX_H16_MAP"] = mp
            else:
                os.environ["ELX_H16_MAP"] = "1"
                os.environ["ELX_H16_SB"] = mp
            res[mp].append(2 * m * n * k / timeit(go, 2) / 1e12)
    os.environ.pop("ELX_H16_MAP")
    os.environ.pop("ELX_H16_SB", None)
    line = f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}:"
    for mp in maps:
        v = res[mp]
        line += f"  map{mp} best {max(v):7.1f} mean {sum(v) / len(v):7.1f}"
    print(line, flush=True)
    del A, B, C
    torch.cuda.empty_cache()


if __name__ == "__main__":
    reps = 4
    args, sbs = [], []
    it = iter(sys.argv[1:])
    for a in it:
        if a == "--reps":
            reps = int(next(it))
        elif a == "--sb":
            sbs = next(it).split(":")
        else:
            args.append(a)
    for spec in args or SHAPES:
        run(spec, reps, ["0"] + (sbs or ["2,8"]))
