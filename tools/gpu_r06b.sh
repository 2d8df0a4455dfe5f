#!/bin/bash
# round-6 call b: bench self-launch / stage-hang / pool release tests, f16 vs bf16
# (sustained A/B + counters), fp32 ring vs slab for NN/NT on 257..511-tile grids
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_kernels.py \
  -k "bench_stage_hang or bench_launches or release_off" > gpurun_out/r06b_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/h16_dtype_ab.py 32768 3 > gpurun_out/r06b_dtype_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/h16_dtype_ab.py 16384 3 >> gpurun_out/r06b_dtype_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/ring_ab.py f32,0,0,3072,2560,4096 f32,0,1,3072,2560,4096 f32,0,0,2560,2560,8192 \
  f32,0,1,2560,2560,8192 f32,1,0,3072,2560,4096 --modes 0,1,8 --reps 3 > gpurun_out/r06b_f32_ring_ab.log 2>&1 || exit $?
IMPLS=ours bash tools/h16_vs_vendor.sh r06b_bf16 bf16 32768 0 0 || exit $?
IMPLS=ours bash tools/h16_vs_vendor.sh r06b_f16 f16 32768 0 0 || exit $?
exit 0
