#!/bin/bash
# round-6 call e: 16-bit exact + local GEMM tests on the new plan; the mid-size
# map at beta = 0 (like-for-like with the vendor) with the library's own tile
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "16bit or vendor_blas or matches_mkl" > gpurun_out/r06e_tests.log 2>&1 || exit $?
S=""
for n in 1536 2048 2560 3072 3584 4096 4608 5120 6144 8192; do S="$S bf16,0,0,$n,$n,$n"; done
S="$S bf16,0,0,1536,2048,2048 bf16,0,0,2560,2560,8192 bf16,1,0,3072,3072,3072 bf16,0,1,3072,3072,3072 bf16,1,1,3072,3072,3072 f16,0,0,3072,3072,3072 bf16,1,0,4096,4096,4096 bf16,1,0,16384,16384,16384"
timeout -k 10 900 python3 tools/h16_tile_sweep.py $S --tiles ,256,192,128 --splits 64 --beta 0 > gpurun_out/r06e_sweep_b0.log 2>&1 || exit $?
exit 0
