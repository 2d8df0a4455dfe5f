#!/bin/bash
# kernel traces of C4 (SUMMA_DOT) with and without the contraction overlap
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for ov in 1 0; do
  ELX_DOT_OVERLAP=$ov timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/dot_tr$ov -o tr -- python3 $R/bench.py --config c4 --steps 1 --warmup 1 > $R/gpurun_out/dot_tr$ov.log 2>&1
  rc=$?; echo "trace ov=$ov rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
done
