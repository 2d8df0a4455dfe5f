#!/bin/bash
# rocprofv3 evidence for bench.py (round tag $1): kernel-trace stats of the bench
# command, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) on the
# same command.  Outputs under gpurun_out/prof_<tag>*; copy summaries to profiles/.
TAG=${1:-r01}; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-c3-1gpu $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG} -o bench -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $R/gpurun_out/prof_${TAG}_pmc$i -o pmc -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_pmc$i.log 2>&1
  rc=$?; echo "pmc $i ($pmc) rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
