#!/bin/bash
# 16-bit tile order A/B: grouped (default) vs XCD-grid (ELX_H16_MAP=xcd); parity with xcd, then times, then FETCH_SIZE
set -e
ELX_H16_MAP=xcd timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "16bit" 2>&1 | tail -1 | sed "s/^/map=xcd parity: /"
for rep in 1 2; do
for mp in g xcd; do
  ELX_H16_MAP=$mp timeout -k 10 120 python tools/gemm_bench.py bf16,0,0,32768,32768,32768 bf16,0,0,16384,16384,16384 bf16,1,0,16384,16384,16384 f16,0,0,16384,16384,16384 2>&1 | grep TFLOP | sed "s/^/map=$mp /"
done
done
