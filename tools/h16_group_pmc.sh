#!/bin/bash
# 16-bit tile-order group height (ELX_H16_GROUP) at C5's shape: time, then fabric
# bytes and L2 hit rate per value (rocprofv3 PMC passes on tools/prof_gemm.py)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for g in 2 4 8 16; do
  echo "group=$g $(ELX_H16_GROUP=$g timeout -k 5 120 python3 $R/tools/gemm_bench.py bf16,0,0,32768,32768,32768 bf16,1,0,16384,16384,16384 2>&1 | grep TFLOP | tr '\n' ' ')"
done
for g in 4 8; do
  for pmc in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    ELX_H16_GROUP=$g timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $R/gpurun_out/h16g${g}_$(echo $pmc | cut -c1-5) -o p -- python3 $R/tools/prof_gemm.py bf16 32768 0 0 2 > /dev/null 2>&1 || exit $?
  done
done
python3 - <<PY
import csv, glob
for g in (4, 8):
    out = {}
    for f in glob.glob(f"$R/gpurun_out/h16g{g}_*/**/*counter_collection.csv", recursive=True):
        disp = {}
        for r in csv.DictReader(open(f)):
            if "h4w" not in r["Kernel_Name"]: continue
            disp.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
            disp[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d in disp.values():
            for k, v in d.items(): out.setdefault(k, []).append(v)
    m = {k: sum(v) / len(v) for k, v in out.items()}
    fab = 2 * m.get("FETCH_SIZE", 0) * 1024 / 1e9
    hit = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]) if "TCC_HIT_sum" in m else None
    print(f"group={g} fabric_read_GB={fab:.1f} l2_hit={hit}")
PY
