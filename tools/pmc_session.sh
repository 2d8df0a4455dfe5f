#!/bin/bash
# Counter passes on the local GEMM kernel (one rocprofv3 run per pass; no tracing domains mixed in).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $pmc --output-format csv -d $R/gpurun_out/pmc$i -o pmc -- python3 $R/tools/prof_gemm.py "$@" > $R/gpurun_out/pmc$i.log 2>&1
  rc=$?; echo "pass $i ($pmc): rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
