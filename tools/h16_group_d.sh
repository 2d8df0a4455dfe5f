#!/bin/bash
# tile-order group height sweep for the deep-prefetch 16-bit kernel (ELX_H16_GROUP)
set -e
for rep in 1 2; do
for g in 4 8 16; do
  ELX_H16_GROUP=$g timeout -k 10 120 python tools/gemm_bench.py bf16,0,0,32768,32768,32768 bf16,0,0,16384,16384,16384 bf16,1,0,16384,16384,16384 2>&1 | grep TFLOP | sed "s/^/group=$g /"
done
done
