#!/bin/bash
# Which fp64 kernel shape ran at 2048^3 with ELX_F64G_BM64=256 (kernel trace)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
ELX_F64G_BM64=256 timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bm64_prof -o k -- python3 $R/tools/gemm_bench.py f64,0,0,2048,2048,2048 f64,0,0,1024,1024,2048 > $R/gpurun_out/bm64_prof.log 2>&1 || exit $?
python3 - <<PY
import csv, glob
for f in glob.glob("$R/gpurun_out/bm64_prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:110], r["Calls"], r["AverageNs"])
PY
grep TFLOP $R/gpurun_out/bm64_prof.log
