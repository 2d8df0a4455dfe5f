#!/bin/bash
# A/B of the 16-bit kernels (ELX_H16_KERNEL=dbuf|ring), same shapes, vendor beside.
for k in dbuf ring; do
  ELX_H16_KERNEL=$k python tools/gemm_bench.py bf16,0,0,8192,8192,8192 bf16,1,0,8192,8192,8192 bf16,0,1,8192,8192,8192 \
      f16,0,0,8192,8192,8192 bf16,0,0,16384,8192,4096 bf16,0,0,32768,32768,32768 2>&1 | grep TFLOP | sed "s/^/$k /"
done
