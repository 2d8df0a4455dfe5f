#!/bin/bash
# Which hipBLASLt kernels torch.matmul runs on the small fp64 / fp32 shapes (names
# carry the macro tile, depth and stream-k mode) and their durations beside ours
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 5 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vendor_small -o k -- python3 $R/tools/gemm_bench.py f64,0,0,2048,2048,2048 f64,0,0,1536,2048,2048 f32,0,0,1024,1024,2048 --vendor > $R/gpurun_out/vendor_small.log 2>&1 || exit $?
python3 - <<PY
import csv, glob
for f in glob.glob("$R/gpurun_out/vendor_small/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:200], r["Calls"], r["AverageNs"])
PY
grep TFLOP $R/gpurun_out/vendor_small.log
