#!/bin/bash
# round-6 call y: grids of 1.5 rounds of 256-tiles (t8 = 384): 256 vs 128
# tiles (the plan takes 128 at utilisation 0.75); 3328 x 6656 x 4096 by tile
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TILE "256;128;192" --beta 1 --reps 3 bf16,0,0,6144,4096,4096 bf16,0,0,3072,8192,4096 bf16,0,0,2048,12288,4096 bf16,0,1,6144,4096,4096 bf16,1,1,6144,4096,4096 f16,0,0,6144,4096,4096 bf16,0,0,6144,4096,8192 bf16,0,0,3328,6656,4096 > gpurun_out/r06y_t384_ab.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TILE "256;128" --beta 0 --reps 3 bf16,0,0,6144,4096,4096 bf16,0,0,3072,8192,4096 >> gpurun_out/r06y_t384_ab.log 2>&1 || exit $?
exit 0
