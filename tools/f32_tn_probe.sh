#!/bin/bash
# f32 wave-tile probe: WTM = 32 (8 waves of 32x64) vs 64 (4 waves of 64x64)
# over k and layout; the C4 shapes are TN with k = 524288.
set -e
cd "$(dirname "$0")/.."
S="f32,1,0,8192,8192,524288 f32,1,0,8192,8192,131072 f32,1,0,8192,8192,65536 f32,1,0,8192,8192,16384 f32,1,0,2048,2048,524288 f32,0,0,8192,8192,524288 f32,0,1,8192,8192,65536 f32,1,1,8192,8192,65536 f32,0,0,16384,16384,16384 f32,1,0,16384,16384,16384 f32,0,0,4096,4096,4096"
for r in 1 2; do
for w in 32 64; do
echo "== WTM $w"
ELX_F32G_WTM=$w timeout -k 10 300 python -u tools/gemm_bench.py $S
done
done
