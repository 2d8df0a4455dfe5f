#!/bin/bash
# round-6 call d: which of the 256 / 192 / 128 tiles wins where (square and
# rectangular bf16 shapes, NN), beside hipBLASLt, for h16_plan's rule
R=$GRAFT_REPO_ROOT
cd $R
S=""
for n in 1024 1536 2048 2560 3072 3584 4096 4608 5120 5632 6144 6656 7168 8192 10240 12288; do S="$S bf16,0,0,$n,$n,$n"; done
S="$S bf16,0,0,2048,2048,8192 bf16,0,0,4096,4096,1024 bf16,0,0,4096,2048,4096 bf16,0,0,8192,4096,2048 bf16,0,0,1536,2048,2048 bf16,0,0,2560,2560,8192 bf16,0,0,16384,8192,8192"
timeout -k 10 900 python3 tools/h16_tile_sweep.py $S --tiles 256,192,128 --splits 64 > gpurun_out/r06d_sweep.log 2>&1 || exit $?
exit 0
