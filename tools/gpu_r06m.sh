#!/bin/bash
# round-6 call m: the final library: the GPU suite, smoke, the default bench
# line, its rocprofv3 kernel trace, and the driver-pool probe on this box
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06m_gputests.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06m_smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/r06m_bench.json 2> gpurun_out/r06m_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r06m -o bench -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c3-1gpu > $R/gpurun_out/prof_r06m_bench.log 2>&1 || exit $?
cd $R
for f in kernel h2d; do timeout -k 10 240 ./tools/_build_pool_trim_probe 300 $f >> gpurun_out/r06m_pool_trim_probe.log 2>&1 || exit $?; done
exit 0
