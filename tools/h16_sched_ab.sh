#!/bin/bash
# Round-4 A/B: the one-barrier four-wave loop (ELX_H16_SCHED=1, default) vs the
# two-barrier loop (=2), interleaved in one process per shape pair (tools/gemm_bench.py lines)
R=$GRAFT_REPO_ROOT
SH="bf16,1,0,16384,16384,16384 bf16,0,0,16384,16384,16384 bf16,0,1,16384,16384,16384 bf16,1,1,16384,16384,16384 bf16,0,0,32768,32768,32768 f16,0,0,16384,16384,16384"
for rep in 1 2; do
  for v in 1 2; do
    echo "== rep $rep ELX_H16_SCHED=$v"; ELX_H16_SCHED=$v timeout -k 5 200 python3 $R/tools/gemm_bench.py $SH 2>&1 | grep TFLOP || exit 1
  done
done
