"""16-bit tile-order group height (ELX_H16_GROUP, read per call) A/B in one
process, interleaved rounds so clock drift hits both values alike."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_bench

groups = [int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "4,8").split(",")]
for rnd in range(3):
    for g in groups:
        os.environ["ELX_H16_GROUP"] = str(g)
        print(f"round {rnd} group={g}", flush=True)
        gemm_bench.run("bf16", 0, 0, 32768, 32768, 32768, False)
        gemm_bench.run("bf16", 1, 0, 16384, 16384, 16384, False)
        gemm_bench.run("f16", 0, 0, 32768, 32768, 32768, False)
