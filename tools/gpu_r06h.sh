#!/bin/bash
# round-6 call h: 160 / 224 tiles (WM 5 / 7): exact tests, then the tile map
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "test_local_gemm_16bit_exact and (160 or 224 or 2560 or 3584)" > gpurun_out/r06h_tests.log 2>&1 || exit $?
S=""
for n in 2048 2560 3072 3584 4096 4608 5120 5632 6144 6656 7168 8192; do S="$S bf16,0,0,$n,$n,$n"; done
S="$S bf16,0,0,1536,2048,2048 bf16,0,0,2560,2560,8192 bf16,1,0,3584,3584,3584 bf16,1,0,2560,2560,2560 bf16,0,1,2560,2560,2560 bf16,0,0,4096,2048,4096 bf16,0,0,8192,4096,2048"
timeout -k 10 900 python3 tools/h16_tile_sweep.py $S --tiles ,256,224,192,160,128 --splits 64 --beta 0 > gpurun_out/r06h_sweep.log 2>&1 || exit $?
exit 0
