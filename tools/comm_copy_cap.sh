#!/bin/bash
# C3 on one GPU with every panel copied through the comm stream (ELX_SUMMA_COPY=1,
# the N>1 pipeline's HBM pattern) vs the cap on comm-stream copy workgroups
set -e
for cap in ${CAPS:-0 64 32 16}; do
  ELX_SUMMA_COPY=1 ELX_COMM_COPY_WGS=$cap timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra-configs --c3-steps 2 2>&1 | grep '^{"metric"' | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['c3_1gpu']
print('cap=$cap c3_1gpu (copied panels)', c['value'], 'TFLOP/s, GEMM launch', c['roofline']['avg_launch_ms'], 'ms, exposed gap', c['exposed_compute_gap_ms_per_step'], 'ms/step')"
done
