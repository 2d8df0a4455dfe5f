#!/bin/bash
# The cpu_baseline leg's placement on the GPU box's host cores: the box's CPU,
# then C1 (SUMMA_NNC f64 4096^3, nb 128, 2x2 ranks, pinned) at 1/2/4 MKL threads
# per rank, with MKL's AVX-512 kernels (default) and with MKL's own vendor
# dispatch (CPU_SUMMA_MKL_VENDOR=1: AVX2 kernels on AMD); ~8 s each.
R=$GRAFT_REPO_ROOT
lscpu | grep -E "Model name|^CPU\(s\)|Thread|Core|Socket|NUMA|MHz|Flags" | cut -c1-300
echo "nproc=$(nproc) allowed=$(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
for t in 2 1 4; do
  for vend in 0 1; do
    echo "threads/rank=$t mkl_vendor_dispatch=$vend: $(CPU_SUMMA_MKL_VENDOR=$vend timeout -k 5 60 $R/oracle/_build/cpu_summa 4096 128 2 2 $t 8 /opt/conda/lib/libmkl_rt.so)"
  done
done
