#!/bin/bash
# round-6 call c: the 192 x 192 16-bit tile (WM = 6): exact-integer tests, then
# the mid-size sweep beside hipBLASLt
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "test_local_gemm_16bit_exact and (192 or 3072)" > gpurun_out/r06c_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_tile_sweep.py bf16,0,0,3072,3072,3072 bf16,0,0,2560,2560,2560 bf16,0,0,3584,3584,3584 \
  bf16,0,0,4096,4096,4096 bf16,0,0,1536,2048,2048 bf16,1,0,3072,3072,3072 bf16,0,1,3072,3072,3072 bf16,1,1,3072,3072,3072 \
  f16,0,0,3072,3072,3072 bf16,0,0,6144,6144,6144 bf16,0,0,3072,3072,12288 \
  --tiles 256,192,128,192m0 --splits 64 > gpurun_out/r06c_sweep.log 2>&1 || exit $?
exit 0
