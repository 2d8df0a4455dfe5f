#!/bin/bash
# round-6 call q: the plan counting 192- / 128-tile tails too (4608^3 -> 192-tiles + tail)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 tools/h16_exact_check.py . 4608,4608,1024 4608,2304,1088 > gpurun_out/r06q_exact.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TAIL 1,0 --beta 0 --reps 3 bf16,0,0,4608,4608,4608 bf16,1,0,4608,4608,4608 bf16,0,1,4608,4608,4608 f16,0,0,4608,4608,4608 bf16,0,0,4608,4608,2048 > gpurun_out/r06q_tail_ab.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_tile_sweep.py bf16,0,0,4608,4608,4608 --tiles ,256,192,128 --splits 64 --beta 0 >> gpurun_out/r06q_tail_ab.log 2>&1 || exit $?
exit 0
