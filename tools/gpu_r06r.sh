#!/bin/bash
# round-6 call r: NT / TT at 16384^3 under the super-block geometries and the
# grouped order (is NT's extra L2 traffic a tile-order effect?)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_SB "2,8;2,4;4,8;4,4;1,8;8,4" --beta 0 --reps 2 bf16,0,1,16384,16384,16384 bf16,1,1,16384,16384,16384 bf16,0,0,16384,16384,16384 > gpurun_out/r06r_sb_ab.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_MAP 1,0 --beta 0 --reps 2 bf16,0,1,16384,16384,16384 bf16,1,1,16384,16384,16384 >> gpurun_out/r06r_sb_ab.log 2>&1 || exit $?
exit 0
