#!/bin/bash
# round-6 call za: non-temporal C stores in the interior epilogue
# (ELX_H16_NTC=1) vs plain stores, at beta 0 and 1; then the 16-bit tests
R=$GRAFT_REPO_ROOT
cd $R
S="bf16,1,0,4096,4096,4096 bf16,0,0,4096,4096,4096 bf16,0,0,4096,4096,1024 bf16,0,1,3072,3072,3072 bf16,0,0,2048,2048,2048 f16,0,0,6144,6144,6144 bf16,0,0,16384,16384,16384 bf16,0,0,32768,32768,32768"
timeout -k 10 900 python3 tools/h16_env_ab.py ELX_H16_NTC 1,0 --beta 0 --reps 3 $S > gpurun_out/r06za_ntc_ab.log 2>&1 || exit $?
timeout -k 10 900 python3 tools/h16_env_ab.py ELX_H16_NTC 1,0 --beta 1 --reps 3 $S >> gpurun_out/r06za_ntc_ab.log 2>&1 || exit $?
ELX_H16_NTC=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit_exact" > gpurun_out/r06za_tests.log 2>&1 || exit $?
exit 0
