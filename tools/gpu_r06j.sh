#!/bin/bash
# round-6 call j: data-parallel rounds + tail: exact tests, then the affected
# shapes with the tail split on / off beside hipBLASLt
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "tail_split or (16bit_exact and 3072)" > gpurun_out/r06j_tests.log 2>&1 || exit $?
S="bf16,0,0,6144,6144,6144 bf16,0,0,4608,4608,4608 bf16,0,0,7168,7168,7168 bf16,0,0,10240,10240,10240 bf16,1,0,6144,6144,6144 bf16,0,0,6144,4096,4096 bf16,0,0,3072,3072,4096"
for t in 1 0; do
  echo "ELX_H16_TAIL=$t" >> gpurun_out/r06j_sweep.log
  ELX_H16_TAIL=$t timeout -k 10 600 python3 tools/h16_tile_sweep.py $S --tiles ,256,192,128 --splits 64 --beta 0 >> gpurun_out/r06j_sweep.log 2>&1 || exit $?
done
exit 0
