#!/bin/bash
# Round-3 evidence at HEAD: rocprofv3 kernel stats + PMC passes for the N=1 bench
# line's C2 and C5 points, then the back-to-back comparison against hipBLASLt.
cd $GRAFT_REPO_ROOT
bash tools/collect_profiles.sh r03e --no-extra-configs || exit $?
bash tools/collect_profiles.sh r03e_c5 --config c5 --no-extra-configs || exit $?
timeout -k 10 400 python -u tools/gemm_bench.py --vendor f64,0,0,32768,32768,32768 f64,0,0,4096,4096,4096 f64,0,0,2048,2048,2048 f32,0,0,16384,16384,16384 f32,1,0,8192,8192,524288 bf16,0,0,32768,32768,32768 bf16,1,0,16384,16384,16384 bf16,0,0,16384,16384,16384 bf16,0,1,16384,16384,16384 bf16,1,1,16384,16384,16384 f16,0,0,16384,16384,16384 > gpurun_out/r03e_vendor.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r03e_vendor.log
