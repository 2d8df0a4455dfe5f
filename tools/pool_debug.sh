#!/bin/bash
# gemm_suite repeated under the allocator's debug knobs (round-4 residual hunt:
# intermittent wrong results on the second warm-up with threshold-0 pools)
S=tests/cpp/_build/gemm_suite
for v in "" "ELX_POOL_POISON=1" "ELX_POOL_CACHE=0"; do
  for rep in 1 2 3; do
    for f in tools/suite_pool_exp.txt tools/suite_pool_exp2.txt; do
      echo "=== env [$v] rep $rep exp $f"
      env $v timeout -k 5 60 $S --f $f --o /tmp/res.txt --warmup 3 --runs 1 --check 2>&1 | grep -E "residual" || echo "ok"
    done
  done
done
