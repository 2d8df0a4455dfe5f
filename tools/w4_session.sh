#!/bin/bash
# Four-wave 16-bit kernel: exact/parity tests, A/B timings against the default
# kernel, and (PMC=1) its counters on bf16 TN 16384^3.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ELX_H16_KERNEL=w timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "16bit" -m gpu > gpurun_out/w4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/w4_tests.log; [ $rc -ne 0 ] && exit $rc
SH=${SH:-"bf16,1,0,16384,16384,16384 bf16,0,0,16384,16384,16384 bf16,0,0,32768,32768,32768 bf16,0,1,16384,16384,16384 bf16,1,1,16384,16384,16384"}
rm -f gpurun_out/w4_bench.log
for KF in ${KS:-d w}; do   # kernel[:flags]
  K=${KF%%:*}; F=0; [ "$KF" != "$K" ] && F=${KF#*:}
  echo "== $K flags $F" >> gpurun_out/w4_bench.log
  ELX_H16_KERNEL=$K ELX_H16_FLAGS=$F timeout -k 10 200 python -u tools/gemm_bench.py $SH >> gpurun_out/w4_bench.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/w4_bench.log
if [ "$PMC" = 1 ]; then
  ELX_H16_KERNEL=w ELX_H16_FLAGS=${PMCF:-0} IMPLS=ours bash tools/h16_vs_vendor.sh wtn bf16 16384 1 0 > gpurun_out/vv_wtn.log 2>&1 || exit $?
  python3 tools/pmc_compare.py wtn 8.796e12 > gpurun_out/vv_wtn.json
  python3 -c "import json; r=json.load(open('gpurun_out/vv_wtn.json'))['ours']; c=r['counters']; print('TF %.0f clk %.3f busy %.3f waitany %.3g wavecyc %.3g valu %.3g salu %.3g' % (r['tflops'], r['effective_clock_ghz'], r['mfma_busy_frac'], c['SQ_WAIT_ANY'], c['SQ_WAVE_CYCLES'], c['SQ_INSTS_VALU'], c['SQ_INSTS_SALU']))"
fi
