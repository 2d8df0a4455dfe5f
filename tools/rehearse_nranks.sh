#!/bin/bash
# Rehearsal of bench.py's N>1 line on a one-GPU box: N ranks on device 0 with the
# host-staged (gloo) comm (ELX_BENCH_COMM=host), small n.  Checks the line's
# control flow (self-launch, residual, transfer stats, max over ranks), not RCCL
# or xGMI.  bench.py starts its own N rank processes (launch_ranks).
# usage: tools/rehearse_nranks.sh N [bench args...]
N=$1; shift
export ELX_BENCH_COMM=host
python3 bench.py --gpus "$N" "$@"
