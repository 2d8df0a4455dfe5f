#!/bin/bash
# round-6 call f: the whole GPU suite, smoke, then the default bench line
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f_gputests.log 2>&1 || exit $?
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06f_smoke.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/r06f_bench.json 2> gpurun_out/r06f_bench.err || exit $?
exit 0
