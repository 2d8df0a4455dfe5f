#!/bin/bash
# round-6 call z9: the epilogue through LDS (whole tile columns per store
# instruction) vs the accumulator-order one (ELX_H16_EPILDS=0): the 16-bit
# kernel tests, then the A/B at beta 0 and 1 on one-round, mid-size and C5 grids
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or tail_split or ktail" > gpurun_out/r06z9_tests.log 2>&1 || exit $?
S="bf16,1,0,4096,4096,4096 bf16,0,0,4096,4096,4096 bf16,0,0,4096,4096,1024 bf16,0,1,3072,3072,3072 bf16,1,1,4608,4608,4608 f16,0,0,6144,6144,6144 bf16,0,0,2048,2048,2048 bf16,0,0,1024,1024,1024 bf16,0,0,16384,16384,16384 bf16,0,0,32768,32768,32768"
timeout -k 10 900 python3 tools/h16_env_ab.py ELX_H16_EPILDS 1,0 --beta 0 --reps 3 $S > gpurun_out/r06z9_epi_ab.log 2>&1 || exit $?
timeout -k 10 900 python3 tools/h16_env_ab.py ELX_H16_EPILDS 1,0 --beta 1 --reps 3 $S >> gpurun_out/r06z9_epi_ab.log 2>&1 || exit $?
exit 0
