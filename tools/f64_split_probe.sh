#!/bin/bash
# f64 one-workgroup-per-CU grids (2048^3: 256 tiles): split-k in 2 chunks
# (ELX_DMA_MIN_CHUNK=1024) vs none (default) vs 4 chunks (512)
set -e
cd "$(dirname "$0")/.."
S="f64,0,0,2048,2048,2048 f64,1,0,2048,2048,2048 f64,0,0,2048,2048,4096 f64,0,0,1536,2048,2048 f32,0,0,2048,2048,2048"
for r in 1 2; do
for c in 0 1024 512; do
echo "== min chunk $c"
ELX_DMA_MIN_CHUNK=$c timeout -k 10 200 python -u tools/gemm_bench.py $S
done
done
timeout -k 10 200 python -u tools/gemm_bench.py $S --vendor
