#!/bin/bash
# C4 (TN fp32 8192^2 x 524288, SUMMA_DOT) vs the GPU Dot block size, and the local kernel on the block shapes
for b in 2000 2048 4096 8192; do
  ELX_DOT_BLOCK=$b timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/dot_$b.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/dot_$b.json'));print('block $b', d['value'], d['pct_of_mfma_peak'])"
done
timeout -k 10 200 python tools/gemm_bench.py f32,1,0,2000,2000,524288 f32,1,0,2048,2048,524288 f32,1,0,4096,4096,524288 f32,1,0,8192,8192,524288 f32,1,0,8192,8192,65536
