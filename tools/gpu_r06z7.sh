#!/bin/bash
# round-6 call z7: time vs k on one round of 256-tiles (4096^2 x k, TN and NN,
# beta 0), ours and hipBLASLt: the per-K-tile cost and the fixed cost per launch
R=$GRAFT_REPO_ROOT
cd $R
S=""
for k in 512 1024 2048 4096 8192 16384; do S="$S bf16,1,0,4096,4096,$k bf16,0,0,4096,4096,$k"; done
timeout -k 10 400 python3 tools/gemm_bench.py $S --vendor > gpurun_out/r06z7_k_sweep.log 2>&1 || exit $?
exit 0
