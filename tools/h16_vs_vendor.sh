#!/bin/bash
# Side-by-side counters of our GEMM kernel and hipBLASLt's on one shape (any dtype):
#   [IMPLS="ours vendor"] tools/h16_vs_vendor.sh <tag> <dt> <n> <ta> <tb>
# kernel-trace stats, then separate PMC passes (clock/MFMA/LDS, FETCH_SIZE, L2 hit).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
MOPS=SQ_INSTS_VALU_MFMA_MOPS_$(echo $1 | tr a-z A-Z)
mkdir -p $R/gpurun_out
for impl in ${IMPLS:-ours vendor}; do
  V=""; [ $impl = vendor ] && V="--vendor"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${impl}_trace -o t -- python3 $R/tools/prof_gemm.py "$@" 10 $V > $R/gpurun_out/${TAG}_${impl}_trace.log 2>&1
  rc=$?; echo "$impl trace rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
  i=0
  # MFMA utilisation from the MOPS counters, cross-checked by the busy cycles
  # (both calibrated: tools/pmc_metrics.py, profiles/r04_mfma_calib.log)
  for pmc in "$MOPS SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
             "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $R/gpurun_out/${TAG}_${impl}_pmc$i -o pmc -- python3 $R/tools/prof_gemm.py "$@" 3 $V > $R/gpurun_out/${TAG}_${impl}_pmc$i.log 2>&1
    rc=$?; echo "$impl pmc $i rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
  done
done
exit 0
