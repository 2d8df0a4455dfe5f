#!/bin/bash
# fp64 64 x 64 tiles forced (ELX_F64G_T64=2): four waves of 32 x 32 vs eight of
# 32 x 16 (ELX_F64G_T64W=4 / 8), with the default dispatch beside them; own
# processes, alternating
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SH="f64,0,0,2048,2048,2048 f64,1,0,2048,2048,2048 f64,0,1,2048,2048,2048 f64,1,1,2048,2048,2048 f64,0,0,1536,2048,2048 f64,0,0,3072,3072,3072 f64,0,0,1024,1024,2048"
for r in 1 2; do
  for w in 4 8; do
    echo "== ELX_F64G_T64W=$w ELX_F64G_T64=2"; ELX_F64G_T64W=$w ELX_F64G_T64=2 timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
  done
  echo "== default"; timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
done
