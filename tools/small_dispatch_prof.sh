#!/bin/bash
# Which kernel instantiations the small / mid-size shapes dispatch to (rocprofv3
# kernel-trace stats of tools/gemm_bench.py): 64 x 64 fp64 / fp32 tiles, the
# fp32 ring, the 16-bit split-k partial kernel and its reduce
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 5 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/small_dispatch -o k -- python3 $R/tools/gemm_bench.py f64,0,0,2048,2048,2048 f64,1,0,2048,2048,2048 f64,0,0,3072,3072,3072 f32,0,1,1024,1024,2048 f32,0,0,3072,3072,3072 bf16,0,0,1024,1024,8192 bf16,0,0,2048,2048,2048 > $R/gpurun_out/small_dispatch.log 2>&1 || exit $?
python3 - <<PY
import csv, glob
for f in glob.glob("$R/gpurun_out/small_dispatch/**/*kernel_stats.csv", recursive=True):
    for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"])):
        if "elx" in r["Name"]:
            print(r["Name"][:170], r["Calls"], r["AverageNs"])
PY
grep TFLOP $R/gpurun_out/small_dispatch.log
