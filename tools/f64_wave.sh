#!/bin/bash
# fp64 LDS-DMA kernel: wave tile 32x64 (8 waves) vs 64x64 (4 waves), BM 128 / 256
for cfg in "128 32" "128 64" "256 64"; do
  set -- $cfg
  echo "# BM=$1 WTM=$2"
  ELX_F64G_BM=$1 ELX_F64G_WTM=$2 timeout -k 10 150 python tools/f64_ab.py dma || exit 1
done
