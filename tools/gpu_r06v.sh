#!/bin/bash
# round-6 call v: split-k tail round (ELX_H16_TAILSK=1: a last round of at most
# half the 256-tile slots runs as split-k over the same tiles): exactness at
# 256-tiles, then timing against the plain 256-tile grid and the default plan
R=$GRAFT_REPO_ROOT
cd $R
ELX_H16_TAILSK=1 ELX_H16_TILE=256 timeout -k 10 600 python3 tools/h16_exact_check.py . 4608,4608,4608 6144,4096,4096 2560,5120,2088 > gpurun_out/r06v_exact.log 2>&1 || exit $?
ELX_H16_TILE=256 timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TAILSK 1,0 --beta 0 --reps 3 bf16,0,0,6144,4096,4096 bf16,0,0,4608,4608,4608 bf16,1,0,4608,4608,4608 bf16,0,1,4608,4608,4608 bf16,0,0,7168,7168,7168 bf16,0,0,10240,10240,10240 bf16,0,0,6144,6144,6144 bf16,1,0,6144,6144,6144 bf16,0,0,9216,9216,9216 f16,0,0,4608,4608,4608 > gpurun_out/r06v_tailsk_ab.log 2>&1 || exit $?
timeout -k 10 600 python3 tools/h16_env_ab.py ELX_H16_TILE "0" --beta 0 --reps 3 bf16,0,0,6144,4096,4096 bf16,0,0,4608,4608,4608 bf16,1,0,4608,4608,4608 bf16,0,1,4608,4608,4608 bf16,0,0,7168,7168,7168 bf16,0,0,10240,10240,10240 bf16,0,0,6144,6144,6144 bf16,1,0,6144,6144,6144 bf16,0,0,9216,9216,9216 f16,0,0,4608,4608,4608 > gpurun_out/r06v_plan.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/gemm_bench.py bf16,0,0,6144,4096,4096 bf16,0,0,4608,4608,4608 bf16,1,0,4608,4608,4608 bf16,0,1,4608,4608,4608 --vendor > gpurun_out/r06v_vendor.log 2>&1 || exit $?
exit 0
