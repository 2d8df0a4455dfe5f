#!/bin/bash
# 64 x 64 tiles forced (ELX_F64G_T64=2 / ELX_F32G_T64=2) vs never (0) on shapes
# around the selection rule's edges, own processes, alternating
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SH="2048,2048,2048 1536,2048,2048 2560,2560,2560 3072,3072,3072 3584,3584,3584 2048,4096,2048 4096,4096,4096 1024,1024,2048"
for dt in f64 f32; do
  K=ELX_$(echo $dt | tr a-z A-Z)G_T64
  L=""; for s in $SH; do L="$L $dt,0,0,$s"; done
  for v in 2 0 2 0; do
    echo "== $dt $K=$v"; env $K=$v timeout -k 5 150 python3 $R/tools/gemm_bench.py $L || exit $?
  done
done
