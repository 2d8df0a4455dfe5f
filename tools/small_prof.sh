#!/bin/bash
# Kernel-level durations of the small / mid-grid shapes (split-k partial GEMM vs
# splitk_reduce vs the no-split kernel): rocprofv3 kernel trace of gemm_bench.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for sh in f64,0,0,2048,2048,2048 f64,0,0,1536,2048,2048 f32,0,0,1024,1024,2048; do
  tag=$(echo $sh | tr ',' '_')
  timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/small_prof_$tag -o k -- python3 $R/tools/gemm_bench.py $sh > $R/gpurun_out/small_prof_$tag.log 2>&1 || exit $?
  echo "== $sh"; grep -h "gemm\|splitk\|Name" $(find $R/gpurun_out/small_prof_$tag -name "*kernel_stats.csv") | cut -d, -f1-6 | head -8
done
