#!/bin/bash
# fp32 mid-size shapes: default vs ELX_F32G_T64=0 (no 64 x 64 tiles), own
# processes (the knob is read once), the vendor beside the default
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
SH="f32,0,0,2048,2048,2048 f32,1,0,2048,2048,2048 f32,0,1,2048,2048,2048 f32,0,0,1536,2048,2048 f32,0,0,1024,1024,2048 f32,0,0,2560,2560,2560 f32,0,0,3072,3072,3072 f32,0,0,4096,4096,4096"
echo "== default (+ vendor)"; timeout -k 5 200 python3 $R/tools/gemm_bench.py $SH --vendor || exit $?
echo "== ELX_F32G_T64=0"; ELX_F32G_T64=0 timeout -k 5 120 python3 $R/tools/gemm_bench.py $SH || exit $?
echo "== default"; timeout -k 5 120 python3 $R/tools/gemm_bench.py $SH || exit $?
