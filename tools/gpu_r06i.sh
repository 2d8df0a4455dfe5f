#!/bin/bash
# round-6 call i: the 16-bit tests on the final tile rule, the ld-padding A/B
# (NT / TT fabric question), and the plan's choices beside the vendor
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or vendor_blas" > gpurun_out/r06i_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/h16_ld_ab.py 16384 2 NN,NT,TN,TT 0,64,256 > gpurun_out/r06i_ld_ab.log 2>&1 || exit $?
S="bf16,0,0,2560,2560,2560 bf16,0,0,3072,3072,3072 bf16,0,0,4608,4608,4608 bf16,0,0,6144,6144,6144 bf16,0,0,4096,2048,4096 bf16,1,0,3584,3584,3584 bf16,1,0,2560,2560,2560 bf16,1,0,3072,3072,3072 bf16,0,0,32768,32768,32768"
timeout -k 10 600 python3 tools/h16_tile_sweep.py $S --tiles ,256 --splits 64 --beta 0 > gpurun_out/r06i_plan_vs_vendor.log 2>&1 || exit $?
exit 0
