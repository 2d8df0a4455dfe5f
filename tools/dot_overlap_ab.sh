#!/bin/bash
# C4 (SUMMA_DOT) with the two-slot contraction overlap (default) vs serial (ELX_DOT_OVERLAP=0), interleaved
set -e
for rep in 1 2; do
  for ov in 1 0; do
    ELX_DOT_OVERLAP=$ov timeout -k 10 200 python bench.py --config c4 --steps 3 2>&1 | grep -o '"value": [0-9.]*' | head -1 | sed "s/^/overlap=$ov C4 [VC,STAR] /"
  done
done
