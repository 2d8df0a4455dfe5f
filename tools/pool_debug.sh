#!/bin/bash
# gemm_suite repeated under the allocator's debug knobs: the round-4
# wrong-result hunt (intermittent associativity residuals 0.05-5 on the second
# warm-up, with the cache off too).  Usage: tools/pool_debug.sh [reps]
S=tests/cpp/_build/gemm_suite
REPS=${1:-3}
fails=0
for v in "ELX_POOL_CACHE=1" "ELX_POOL_CACHE=0" "ELX_POOL_POISON=1"; do
  for rep in $(seq 1 "$REPS"); do
    for f in tools/suite_pool_exp.txt tools/suite_pool_exp2.txt; do
      echo "=== env [$v] rep $rep exp $f"
      out=$(env $v timeout -k 5 60 $S --f $f --o /tmp/res.txt --warmup 3 --runs 1 --check 2>&1)
      rc=$?
      echo "$out" | grep -E "Testing|residual|error" || true
      echo "rc=$rc"
      if [ $rc -ge 124 ]; then echo "timeout/abort: stopping"; exit $rc; fi
      [ $rc -ne 0 ] && fails=$((fails + 1))
    done
  done
done
echo "failing runs: $fails"
