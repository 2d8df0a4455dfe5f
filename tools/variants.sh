#!/bin/bash
for r in 1 2; do for v in ${TILES:-128 1288 1289}; do echo "tile $v"; ELX_GEMM_TILE=$v python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids; done; done
