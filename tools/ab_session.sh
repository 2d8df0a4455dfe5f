#!/bin/bash
# One GPU session: a pytest selection (TESTS, pytest -k expression), then
# gemm_bench lines (SH) under each environment variant in VARIANTS
# ("name=ENV1=v1,ENV2=v2;name2=..."), all in order, into gpurun_out/ab_bench.log.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "$TESTS" -m gpu > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
rm -f gpurun_out/ab_bench.log
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
  name=${v%%=*}; envs=${v#*=}
  echo "== $name ($envs)" >> gpurun_out/ab_bench.log
  ( IFS=',' read -ra ES <<< "$envs"; for e in "${ES[@]}"; do export "$e"; done; timeout -k 10 250 python -u tools/gemm_bench.py $SH ) >> gpurun_out/ab_bench.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/ab_bench.log
