#!/bin/bash
# Round-4 A/B of the fp64 / f32 small- and mid-grid paths (<= 512 tiles):
# default vs 64-row fp64 tiles (ELX_F64G_BM64 = max 128-row workgroups), each
# beside the vendor library (torch.matmul), tools/gemm_bench.py lines.
R=$GRAFT_REPO_ROOT
SH="f64,0,0,2048,2048,2048 f64,1,0,2048,2048,2048 f64,0,0,1536,2048,2048 f64,0,0,1024,1024,2048 f64,0,0,2048,2048,4096 f64,0,0,3072,3072,3072 f64,0,0,4096,4096,4096 f32,0,0,1024,1024,2048 f32,0,0,2048,2048,2048 f32,0,0,1536,2048,2048"
echo "== default (+ vendor)"; timeout -k 5 200 python3 $R/tools/gemm_bench.py $SH --vendor || exit $?
for w in 256 512; do
  echo "== ELX_F64G_BM64=$w"; ELX_F64G_BM64=$w timeout -k 5 120 python3 $R/tools/gemm_bench.py $SH || exit $?
done
