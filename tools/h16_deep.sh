#!/bin/bash
# 16-bit kernel A/B: deep-prefetch two-phase kernel (ELX_H16_KERNEL=d) vs the balanced-read phased default (b)
set -e
ELX_H16_KERNEL=d timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "16bit" 2>&1 | tail -1 | sed "s/^/kernel=d parity: /"
for rep in 1 2; do
for kk in d b; do
  for o in "0,0" "1,0" "0,1" "1,1"; do
    ELX_H16_KERNEL=$kk timeout -k 10 120 python tools/gemm_bench.py bf16,$o,8192,8192,8192 bf16,$o,16384,16384,16384 2>&1 | grep TFLOP | sed "s/^/kernel=$kk /"
  done
  ELX_H16_KERNEL=$kk timeout -k 10 120 python tools/gemm_bench.py f16,0,0,16384,16384,16384 bf16,0,0,32768,32768,32768 2>&1 | grep TFLOP | sed "s/^/kernel=$kk /"
done
done
