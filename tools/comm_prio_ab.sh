#!/bin/bash
# comm-stream priority (high, default, vs the compute stream's: ELX_COMM_PRIORITY=0) with the
# copy cap, on C3 with every panel copied (ELX_SUMMA_COPY=1), interleaved
set -e
for rep in 1 2; do
  for pr in 1 0; do
    ELX_COMM_PRIORITY=$pr ELX_SUMMA_COPY=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra-configs --c3-steps 2 2>&1 | grep '^{"metric"' | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['c3_1gpu']
print('priority=$pr c3_1gpu (copied panels)', c['value'], 'TF, launch', c['roofline']['avg_launch_ms'], 'ms, gap', c['exposed_compute_gap_ms_per_step'])"
  done
done
