#!/bin/bash
# C4 (SUMMA_DOT) on one GPU vs the Dot block (ELX_DOT_BLOCK), interleaved
set -e
for rep in 1 2; do
  for b in 2048 4096 8192; do
    ELX_DOT_BLOCK=$b timeout -k 10 200 python bench.py --config c4 --steps 2 --no-cpu-baseline 2>&1 | grep -o '"value": [0-9.]*' | head -1 | sed "s/^/dot_block=$b C4 /"
  done
done
