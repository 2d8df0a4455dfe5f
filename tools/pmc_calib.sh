#!/bin/bash
# rocprofv3 PMC passes over tools/mfma_calib.hip (known MFMA counts per
# dispatch): is SQ_VALU_MFMA_BUSY_CYCLES usable on gfx950, and do the MOPS
# counters give FLOPs / 512?  Outputs: gpurun_out/calib_pmc<i>/, calib.log.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 5 60 $R/tools/_build_mfma_calib 1000 > $R/gpurun_out/calib.log 2>&1 || exit $?
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_BF16" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pmc --output-format csv -d $R/gpurun_out/calib_pmc$i -o pmc -- $R/tools/_build_mfma_calib 1000 > $R/gpurun_out/calib_pmc$i.log 2>&1
  rc=$?; echo "calib pass $i ($pmc) rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
