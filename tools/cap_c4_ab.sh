#!/bin/bash
# C4 / C2 with the comm-stream copy cap at its default vs uncapped (ELX_COMM_COPY_WGS=0), interleaved
set -e
for rep in 1 2; do
  for cap in 256 0; do
    ELX_COMM_COPY_WGS=$cap timeout -k 10 200 python bench.py --config c4 --steps 2 --no-cpu-baseline 2>&1 | grep -o '"value": [0-9.]*' | head -1 | sed "s/^/cap=$cap C4 /"
  done
done
