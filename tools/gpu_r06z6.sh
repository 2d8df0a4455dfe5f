#!/bin/bash
# round-6 call z6: kernel trace of TN 4096^3 back to back (kernel time vs the
# wall time per call: launch and host gaps) and of hipBLASLt on the same
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06z6_ours -o t -- python3 $R/tools/prof_gemm.py bf16 4096 1 0 50 > $R/gpurun_out/prof_r06z6_ours.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06z6_vendor -o t -- python3 $R/tools/prof_gemm.py bf16 4096 1 0 50 --vendor > $R/gpurun_out/prof_r06z6_vendor.log 2>&1 || exit $?
exit 0
