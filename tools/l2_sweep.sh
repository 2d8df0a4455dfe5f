#!/bin/bash
# L2 locality sweep of the fp64 LDS-DMA kernel: tile-group height x XCD remap,
# time (tools/prof_gemm.py timing via rocprofv3 kernel trace) and TCC hit/miss.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "8 1" "4 1" "16 1" "8 0" "2 1"; do
  set -- $cfg
  export ELX_F64G_GROUP=$1 ELX_F64G_REMAP=$2
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/l2_$1_$2 -o pmc -- python3 $R/tools/prof_gemm.py f64 16384 > $R/gpurun_out/l2_$1_$2.log 2>&1
  rc=$?; echo "group=$1 remap=$2 rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
