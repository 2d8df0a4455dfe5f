#!/bin/bash
# LDS-DMA staging source A/B: global_load_lds (ELX_*_STAGE=g) vs buffer descriptors (default)
S="f64,0,0,16384,16384,16384 f64,0,0,32768,16384,4096 f64,1,0,16384,16384,16384 f32,0,0,16384,16384,16384 f32,1,0,2048,2048,524288 bf16,0,0,16384,16384,16384 bf16,1,0,16384,16384,16384 bf16,0,1,8192,8192,8192"
for rep in 1 2; do
  for st in g b; do
    ELX_F64G_STAGE=$st ELX_F32G_STAGE=$st ELX_H16_STAGE=$st timeout -k 10 300 python tools/gemm_bench.py $S 2>&1 | grep TFLOP | sed "s/^/stage=$st /" || exit $?
  done
done
