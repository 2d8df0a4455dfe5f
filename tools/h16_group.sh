#!/bin/bash
# 16-bit kernel tile-order group height (ELX_H16_GROUP) vs time
for g in 1 2 4 8; do
  ELX_H16_GROUP=$g timeout -k 10 120 python tools/gemm_bench.py bf16,0,0,16384,16384,16384 bf16,0,0,32768,32768,8192 bf16,1,0,16384,16384,16384 bf16,0,0,32768,32768,32768 2>&1 | grep TFLOP | sed "s/^/group=$g /" || exit 1
done
