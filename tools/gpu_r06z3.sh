#!/bin/bash
# round-6 call z3: the plan with 64-tiles: the 16-bit kernel tests, the plan
# against forced 128-tiles on small grids (every orientation), hipBLASLt beside
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or tail_split or ktail" > gpurun_out/r06z3_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TILE "0;128" --beta 1 --reps 3 bf16,0,0,1024,1024,1024 bf16,1,0,1024,1024,1024 bf16,0,1,1024,1024,1024 bf16,1,1,1024,1024,1024 bf16,1,0,1536,1536,1536 bf16,0,1,1536,1536,1536 f16,0,0,1536,2048,2048 bf16,1,0,1536,2048,2048 bf16,0,0,1024,3072,2048 bf16,0,0,2048,1536,1024 > gpurun_out/r06z3_t64_plan_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/gemm_bench.py bf16,0,0,1024,1024,1024 bf16,1,0,1024,1024,1024 bf16,0,0,1536,1536,1536 bf16,0,0,1536,2048,2048 bf16,1,0,1536,2048,2048 bf16,0,0,1024,2048,1024 --vendor > gpurun_out/r06z3_vendor.log 2>&1 || exit $?
exit 0
