#!/bin/bash
# 16-bit grids of few 256 x 256 tiles: split-k chunk cap (ELX_H16_SPLIT = 64
# default, 4, 2, 0 = none), own processes, alternating
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SH="bf16,0,0,2048,2048,2048 bf16,1,0,2048,2048,2048 bf16,0,0,1024,1024,8192 bf16,0,0,1024,1024,1024 bf16,0,0,2048,2048,8192 bf16,0,0,1024,1024,2048"
for r in 1 2; do
  for z in 64 4 2 0; do
    echo "== ELX_H16_SPLIT=$z"; ELX_H16_SPLIT=$z timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
  done
done
