#!/bin/bash
# round-6 call v5: the final tree (rebuilt after the reverted store experiment): the GPU suite, smoke, the default bench
# line, its rocprofv3 kernel trace
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06v5_gputests.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06v5_smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/r06v5_bench.json 2> gpurun_out/r06v5_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06v5 -o bench -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3-1gpu > $R/gpurun_out/prof_r06v5_bench.log 2>&1 || exit $?
cd $R
exit 0
