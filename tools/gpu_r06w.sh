#!/bin/bash
# round-6 call w: the split-k tail on by default (a quarter to a third of a
# round of 256-tiles, not TN): the 16-bit kernel tests, and the plan with and
# without it (ELX_H16_TAILSK) beside hipBLASLt
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or tail_split or ktail" > gpurun_out/r06w_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TAILSK 1,0 --beta 1 --reps 3 bf16,0,0,4608,4608,4608 bf16,0,1,4608,4608,4608 bf16,1,1,4608,4608,4608 bf16,1,0,4608,4608,4608 f16,0,0,4608,4608,4608 bf16,0,0,8448,8448,8448 bf16,0,0,3328,6656,4096 bf16,0,0,7168,7168,7168 bf16,0,0,10240,10240,10240 > gpurun_out/r06w_tailsk_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/gemm_bench.py bf16,0,0,4608,4608,4608 bf16,0,1,4608,4608,4608 bf16,1,1,4608,4608,4608 f16,0,0,4608,4608,4608 bf16,0,0,8448,8448,8448 bf16,0,0,3328,6656,4096 --vendor > gpurun_out/r06w_vendor.log 2>&1 || exit $?
exit 0
