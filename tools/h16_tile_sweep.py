"""16-bit local GEMM: the four-wave kernel's 256 x 256 and 128 x 128 tiles (and
split-k caps) on the same shapes in one process, beside hipBLASLt (torch.matmul).

  python tools/h16_tile_sweep.py [dt,ta,tb,m,n,k ...] [--splits 1,2,4] [--tiles 256,192,128,192m0] [--beta 0]

(an empty tile entry, e.g. --tiles ,256: the library's own choice; --beta: ours
at that beta, default 1; the vendor call C = op(A) op(B) reads no C, so --beta 0
is the like-for-like comparison)

Each line: the shape, TFLOP/s per variant (ELX_H16_TILE = 256 / 192 / 128, read
per call by the library, a suffix m0 / m1 forcing the grouped / super-block tile
order through ELX_H16_MAP; ELX_H16_SPLIT caps the split-k chunks), and the
vendor's.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402
from gemm_bench import timeit  # noqa: E402

SHAPES = ["bf16,0,0,2048,2048,2048", "bf16,1,0,2048,2048,2048", "bf16,0,1,2048,2048,2048",
          "bf16,0,0,1024,1024,8192", "bf16,0,0,2048,2048,8192", "bf16,0,0,3072,3072,3072",
          "bf16,0,0,2560,2560,2560", "bf16,0,0,4096,4096,4096", "bf16,0,0,1536,2048,2048",
          "bf16,0,0,1024,1024,1024", "f16,0,0,2048,2048,2048"]
TD = {"f16": torch.float16, "bf16": torch.bfloat16}


def run(spec, variants, beta=1.0):
    dt, ta, tb, m, n, k = spec.split(",")
    ta, tb, m, n, k = int(ta), int(tb), int(m), int(n), int(k)
    tdt = TD[dt]
    lda = k if ta else m
    ldb = n if tb else k
    A = torch.rand(lda * (m if ta else k), device="cuda").sub_(0.5).to(tdt)
    B = torch.rand(ldb * (k if tb else n), device="cuda").sub_(0.5).to(tdt)
    C = torch.rand(m * n, device="cuda").sub_(0.5).to(tdt)
    fn = L.lib().elx_gemm_bf16 if dt == "bf16" else L.lib().elx_gemm_f16
    go = lambda: L.check(fn(ta, tb, m, n, k, 1.0, A.data_ptr(), lda, B.data_ptr(), ldb, beta, C.data_ptr(), m, None))
    out = []
    for tile, split in variants:
        os.environ["ELX_H16_TILE"] = tile[:3]
        os.environ["ELX_H16_SPLIT"] = split
        if len(tile) > 3:
            os.environ["ELX_H16_MAP"] = tile[4:]
        t = timeit(go, 3)
        os.environ.pop("ELX_H16_MAP", None)
        out.append(f"tile{tile}/split{split} {2 * m * n * k / t / 1e12:7.1f}")
    os.environ.pop("ELX_H16_TILE")
    os.environ.pop("ELX_H16_SPLIT")
    At = A.view(m if ta else k, lda)
    Bt = B.view(k if tb else n, ldb)
    opA = At if ta else At.t()
    opB = Bt if tb else Bt.t()
    Cv = torch.empty(m, n, dtype=tdt, device="cuda")
    tv = timeit(lambda: torch.matmul(opA, opB, out=Cv), 3)
    print(f"{dt} {'T' if ta else 'N'}{'T' if tb else 'N'} {m}x{n}x{k}: " + "  ".join(out) +
          f"  vendor {2 * m * n * k / tv / 1e12:7.1f}", flush=True)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    splits, tiles, beta = ["64"], ["256", "192", "128"], 1.0
    for i, a in enumerate(sys.argv):
        if a in ("--splits", "--tiles", "--beta"):
            vals = sys.argv[i + 1].split(",")
            if a == "--splits":
                splits = vals
            elif a == "--tiles":
                tiles = vals
            else:
                beta = float(vals[0])
            args = [x for x in args if x != sys.argv[i + 1]]
    variants = [(t, s) for t in tiles for s in splits]
    for spec in args or SHAPES:
        run(spec, variants, beta)
