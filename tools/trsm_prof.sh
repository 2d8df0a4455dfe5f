#!/bin/bash
# rocprofv3 kernel stats of El::Trsm LEFT f64 m=n=16384 (tools/trsm_bench.py) at the current defaults
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_trsm -o trsm -- python3 $R/tools/trsm_bench.py 16384 16384 f64 > $R/gpurun_out/prof_trsm.log 2>&1
echo "rc=$?"
