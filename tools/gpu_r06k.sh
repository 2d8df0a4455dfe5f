#!/bin/bash
# round-6 call k: tail split at a quarter round, plan's picks vs vendor
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "tail_split or 16bit_exact" > gpurun_out/r06k_tests.log 2>&1 || exit $?
S="bf16,0,0,6144,6144,6144 bf16,1,0,6144,6144,6144 bf16,0,0,7168,7168,7168 bf16,0,0,10240,10240,10240 bf16,0,0,6144,4096,4096 bf16,0,0,4608,4608,4608 bf16,0,0,3072,3072,3072 bf16,0,0,4096,4096,4096 bf16,0,0,32768,32768,32768 f16,0,0,6144,6144,6144"
timeout -k 10 600 python3 tools/h16_tile_sweep.py $S --tiles ,256 --splits 64 --beta 0 > gpurun_out/r06k_plan_vs_vendor.log 2>&1 || exit $?
exit 0
