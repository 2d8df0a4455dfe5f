#!/bin/bash
# Counter passes on the phased bf16 TN kernel: base vs no-staging ablation (ELX_H16_FLAGS=1).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true

for fl in 0 1; do
  i=0
  for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS GRBM_COUNT"; do
    i=$((i+1))
    ELX_H16_FLAGS=$fl timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $R/gpurun_out/h16pmc_f${fl}_$i -o pmc -- python3 $R/tools/prof_gemm.py bf16 16384 1 0 > $R/gpurun_out/h16pmc_f${fl}_$i.log 2>&1
    rc=$?; echo "flags $fl pass $i: rc=$rc"
    case $rc in 124|137|134|139) exit $rc;; esac
  done
done
exit 0
