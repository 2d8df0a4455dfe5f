#!/bin/bash
# Rehearsal of bench.py's N>1 line on a one-GPU box: N ranks on device 0 with the
# host-staged (gloo) comm (ELX_BENCH_COMM=host), small n.  Checks the line's
# control flow (residual, transfer stats, max over ranks), not RCCL or xGMI.
# usage: tools/rehearse_nranks.sh N [bench args...]
N=$1; shift
export ELX_BENCH_COMM=host
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
  --master-port $((29500 + N)) bench.py --gpus "$N" "$@"
