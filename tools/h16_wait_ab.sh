#!/bin/bash
# Round-4 A/B: 16-bit loop waits as inline asm (ELX_H16_WAIT=asm, round 3) vs
# the builtin (default), and the two-barrier loop (ELX_H16_SCHED=2), in turn
R=$GRAFT_REPO_ROOT
SH="bf16,1,0,16384,16384,16384 bf16,0,0,16384,16384,16384 bf16,0,1,16384,16384,16384 bf16,1,1,16384,16384,16384 bf16,0,0,32768,32768,32768 f16,0,0,16384,16384,16384"
for rep in 1 2; do
  for v in "ELX_H16_WAIT=asm" "ELX_H16_WAIT=builtin" "ELX_H16_SCHED=2"; do
    echo "== rep $rep $v"; env $v timeout -k 5 200 python3 $R/tools/gemm_bench.py $SH 2>&1 | grep TFLOP || exit 1
  done
done
