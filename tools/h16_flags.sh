#!/bin/bash
# bf16 NN kernel ablations (ELX_H16_FLAGS, timing only): 0 base, 1 no staging, 2 no barrier, 3 both, 8 no DMA wait
for f in ${FLAGS:-0 1 2 3 8}; do
  ELX_H16_KERNEL=s ELX_H16_FLAGS=$f python tools/gemm_bench.py bf16,0,0,8192,8192,8192 bf16,0,0,16384,16384,16384 2>&1 | grep TFLOP | sed "s/^/flags=$f /"
done
