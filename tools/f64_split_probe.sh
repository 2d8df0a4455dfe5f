#!/bin/bash
# split-k chunk count for grids below two workgroups per CU: with k = 2048 the
# min-chunk knob sets z = min(ceil(1024 / tiles), 2048 / chunk): 1024 -> 2,
# 683 -> 3, 512 -> 4, 342 -> 6 (capped by the first term), 256 -> 8; 0 = rule
set -e
cd "$(dirname "$0")/.."
S="f64,0,0,1024,1024,2048 f64,0,0,1536,1536,2048 f64,0,0,1536,2048,2048 f64,0,0,1920,2048,2048 f64,0,0,1536,2048,4096 f32,0,0,1536,2048,2048 f32,0,0,1024,1024,2048"
for c in ${CHUNKS:-0 1024 683 512 342 256}; do
echo "== min chunk $c"
ELX_DMA_MIN_CHUNK=$c timeout -k 10 200 python -u tools/gemm_bench.py $S
done
timeout -k 10 200 python -u tools/gemm_bench.py $S --vendor
