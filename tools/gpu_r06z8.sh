#!/bin/bash
# round-6 call z8: per-workgroup timeline (diagnostic build with s_memrealtime
# stamps) of one-round grids, to place the fixed cost per launch
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 tools/h16_stamps.py tools/_build_probe/stamps bf16,1,0,4096,4096,4096 bf16,1,0,4096,4096,1024 bf16,0,0,4096,4096,4096 bf16,1,0,4096,4096,8192 > gpurun_out/r06z8_stamps.log 2>&1 || exit $?
exit 0
