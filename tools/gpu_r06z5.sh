#!/bin/bash
# round-6 call z5: TN single-round grids (4096^3, 4096 x 4096 x 8192) against
# the knobs that shape them: tile order (ELX_H16_MAP), unit order (ELX_H16_SWAP),
# group height; hipBLASLt beside
R=$GRAFT_REPO_ROOT
cd $R
S="bf16,1,0,4096,4096,4096 bf16,1,0,4096,4096,8192 bf16,1,0,8192,4096,4096"
timeout -k 10 300 python3 tools/h16_env_ab.py ELX_H16_MAP 1,0 --beta 0 --reps 3 $S > gpurun_out/r06z5_tn_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/h16_env_ab.py ELX_H16_SWAP 1,0 --beta 0 --reps 3 $S >> gpurun_out/r06z5_tn_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/h16_env_ab.py ELX_H16_SB "2,8;1,8;4,8;2,4;2,16" --beta 0 --reps 3 $S >> gpurun_out/r06z5_tn_ab.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/gemm_bench.py $S --vendor >> gpurun_out/r06z5_tn_ab.log 2>&1 || exit $?
exit 0
