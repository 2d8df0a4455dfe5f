#!/bin/bash
# round-6 call x: the vectorised split-k reduce (h16_splitk_reduce4) against
# the grid-stride one (ELX_H16_RED=0), tests, and a kernel trace of 4608^3
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or tail_split or ktail or split" > gpurun_out/r06x_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_RED 1,0 --beta 1 --reps 3 bf16,0,0,4608,4608,4608 bf16,0,0,3328,6656,4096 bf16,0,0,8448,8448,8448 bf16,0,0,1024,1024,8192 bf16,0,0,2048,2048,16384 bf16,1,0,1536,1536,32768 f16,0,0,1024,2048,16384 > gpurun_out/r06x_red_ab.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06x -o t -- python3 $R/tools/prof_gemm.py bf16 4608 0 0 10 > $R/gpurun_out/prof_r06x.log 2>&1 || exit $?
exit 0
