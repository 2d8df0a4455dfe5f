#!/bin/bash
# 16-bit grids of few 256 x 256 tiles: split-k (default) vs none (ELX_H16_SPLIT=0),
# own processes, alternating
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SH="bf16,0,0,2048,2048,2048 bf16,1,0,2048,2048,2048 bf16,0,0,1024,1024,8192 bf16,0,0,1024,1024,1024 bf16,0,0,2048,2048,8192 bf16,0,0,2560,2560,2560 bf16,0,0,3072,3072,3072"
for r in 1 2; do
  echo "== default"; timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
  echo "== ELX_H16_SPLIT=0"; ELX_H16_SPLIT=0 timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
done
