#!/bin/bash
# round-6 call p: tile-order group height at C5's shape, one process, interleaved
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_GROUP 8,4,16,32 --beta -0.5 --reps 4 bf16,0,0,32768,32768,32768 bf16,0,0,16384,8192,8192 > gpurun_out/r06p_group_ab.log 2>&1 || exit $?
exit 0
