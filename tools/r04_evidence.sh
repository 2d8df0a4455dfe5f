#!/bin/bash
# Round-4 evidence at HEAD: rocprofv3 kernel stats + PMC passes (FETCH, WRITE,
# L2 hit, MOPS-based MFMA utilisation) of the N=1 bench line's C2 and C5
# points, the C5 kernel beside hipBLASLt's (NN and TN bf16 16384^3), then the
# back-to-back comparison against the vendor library.
cd $GRAFT_REPO_ROOT
bash tools/collect_profiles.sh r04e --no-extra-configs || exit $?
bash tools/collect_profiles.sh r04e_c5 --config c5 --no-extra-configs || exit $?
bash tools/h16_vs_vendor.sh r04_tn bf16 16384 1 0 || exit $?
bash tools/h16_vs_vendor.sh r04_nn bf16 16384 0 0 || exit $?
timeout -k 10 400 python -u tools/gemm_bench.py --vendor f64,0,0,32768,32768,32768 f64,0,0,4096,4096,4096 f64,0,0,2048,2048,2048 f64,0,0,1536,2048,2048 f32,0,0,16384,16384,16384 f32,0,0,1024,1024,2048 f32,1,0,8192,8192,524288 bf16,0,0,32768,32768,32768 bf16,1,0,16384,16384,16384 bf16,0,0,16384,16384,16384 bf16,0,1,16384,16384,16384 bf16,1,1,16384,16384,16384 f16,0,0,16384,16384,16384 > gpurun_out/r04e_vendor.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r04e_vendor.log
