#!/bin/bash
# 16-bit grids of fewer 256 x 256 tiles than CUs: split-k (default) vs none
# (ELX_H16_SPLIT=0), own processes, vendor beside the default
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SH="bf16,0,0,1024,1024,8192 bf16,1,0,1024,1024,8192 bf16,0,0,1024,1024,1024 bf16,0,0,2048,2048,2048 bf16,1,0,2048,2048,2048 bf16,0,0,3072,3072,3072 bf16,0,0,4096,4096,4096 bf16,0,0,2048,2048,8192 f16,0,0,2048,2048,2048"
echo "== default (+ vendor)"; timeout -k 5 150 python3 $R/tools/gemm_bench.py $SH --vendor || exit $?
echo "== ELX_H16_SPLIT=0"; ELX_H16_SPLIT=0 timeout -k 5 150 python3 $R/tools/gemm_bench.py $SH || exit $?
