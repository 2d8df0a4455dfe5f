#!/bin/bash
# 16-bit kernel A/B: two-stage (ELX_H16_KERNEL=s) vs phased ping-pong (default), parity then timing
set -e
ELX_H16_KERNEL=s timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k 16bit
for kern in s p; do
  for o in "0,0" "1,0" "0,1" "1,1"; do
    ELX_H16_KERNEL=$kern timeout -k 10 120 python tools/gemm_bench.py bf16,$o,8192,8192,8192 bf16,$o,16384,16384,16384 2>&1 | grep TFLOP | sed "s/^/kernel=$kern /"
  done
done
