#!/bin/bash
# round-6 call l: the 16-B epilogue (permlane16_swap pairs): exact tests, A/B
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or tail_split" > gpurun_out/r06l_tests.log 2>&1 || exit $?
S="bf16,0,0,4096,4096,4096 bf16,0,0,3072,3072,3072 bf16,1,0,3584,3584,3584 bf16,0,0,2048,2048,2048 bf16,0,0,6144,6144,6144 bf16,0,0,16384,16384,16384 bf16,0,0,16384,8192,8192 bf16,0,0,32768,32768,32768"
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_EPI16 1,0 --beta 1 $S > gpurun_out/r06l_epi_ab.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_EPI16 1,0 --beta 0 bf16,0,0,4096,4096,4096 bf16,0,0,3072,3072,3072 bf16,0,0,32768,32768,32768 >> gpurun_out/r06l_epi_ab.log 2>&1 || exit $?
exit 0
