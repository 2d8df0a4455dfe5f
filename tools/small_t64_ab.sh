#!/bin/bash
# Grids of fewer than 256 128 x 128 tiles: 128 x 128 tiles split k ways (default)
# vs 64 x 64 tiles (ELX_F*G_T64=2) unsplit up to k = 2048 or split at k >= 2048
# (ELX_DMA_MIN_CHUNK=1024), own processes, alternating
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for dt in f32 f64; do
  K=ELX_$(echo $dt | tr a-z A-Z)G_T64
  SH="$dt,0,0,1024,1024,2048 $dt,1,0,1024,1024,2048 $dt,0,0,1024,1024,1024 $dt,0,0,1024,1024,4096 $dt,0,0,768,1024,2048 $dt,0,0,1536,1536,1024 $dt,0,0,512,512,2048"
  for r in 1 2; do
    echo "== $dt default"; timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
    echo "== $dt $K=2"; env $K=2 timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
    echo "== $dt $K=2 ELX_DMA_MIN_CHUNK=1024"; env $K=2 ELX_DMA_MIN_CHUNK=1024 timeout -k 5 100 python3 $R/tools/gemm_bench.py $SH || exit $?
  done
done
