#!/bin/bash
# fp32 LDS-DMA kernel: wave tile 32x64 (8 waves) vs 64x64 (4 waves)
for w in 32 64; do
  echo "# WTM=$w"
  ELX_F32G_WTM=$w timeout -k 10 150 python tools/f64_ab.py --f32 dma || exit 1
  ELX_F32G_WTM=$w timeout -k 10 100 python tools/gemm_bench.py f32,1,0,2048,2048,524288 f32,0,0,32768,16384,4096 || exit 1
done
