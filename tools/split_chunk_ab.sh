#!/bin/bash
# few-tile split-k minimum chunk (ELX_SPLIT_CHUNK) at mid sizes, two repetitions
set -e
for rep in 1 2; do
for c in 0 1024 512; do
  ELX_SPLIT_CHUNK=$c timeout -k 10 120 python tools/gemm_bench.py f64,0,0,2048,2048,2048 f64,0,0,3072,3072,3072 f64,0,0,1536,1536,1536 f32,0,0,2048,2048,2048 f32,1,0,2048,2048,8192 2>&1 | grep TFLOP | sed "s/^/chunk=$c /"
done
done
