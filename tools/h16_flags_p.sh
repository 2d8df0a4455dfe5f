#!/bin/bash
# phased 16-bit kernel ablations, bf16 TN (ELX_H16_FLAGS, timing only): 0 base, 1 no staging, 2 no vmcnt waits, 3 both, 4 no setprio
for f in ${FLAGS:-0 1 2 3 4}; do
  ELX_H16_FLAGS=$f timeout -k 10 120 python tools/gemm_bench.py bf16,1,0,8192,8192,8192 bf16,1,0,16384,16384,16384 2>&1 | grep TFLOP | sed "s/^/flags=$f /"
done
