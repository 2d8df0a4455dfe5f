#!/bin/bash
# round-6 call z2: 64 x 64 tiles (WM = 2, four workgroups per CU) for the
# 16-bit four-wave kernel: exact tests forced to them, then timing against
# the plan's tile on small grids
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit_exact and 64" > gpurun_out/r06z2_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TILE "0;64;128" --beta 1 --reps 3 bf16,0,0,2048,2048,2048 bf16,0,0,1536,2048,2048 bf16,0,0,1024,1024,1024 bf16,0,0,1024,2048,1024 bf16,0,0,2048,1024,4096 bf16,1,0,2048,2048,2048 bf16,0,1,2048,2048,2048 f16,0,0,2048,2048,2048 bf16,0,0,1024,1024,8192 bf16,0,0,2560,2560,2560 bf16,0,0,1536,1536,1536 bf16,0,0,2048,2048,512 > gpurun_out/r06z2_t64_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/gemm_bench.py bf16,0,0,2048,2048,2048 bf16,0,0,1536,2048,2048 bf16,0,0,1024,1024,1024 bf16,0,0,1536,1536,1536 bf16,0,0,2048,2048,512 --vendor > gpurun_out/r06z2_vendor.log 2>&1 || exit $?
exit 0
