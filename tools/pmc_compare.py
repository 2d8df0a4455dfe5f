"""Summarise tools/h16_vs_vendor.sh output: per implementation, the dominant
kernel's average duration, effective clock, MFMA-busy fraction, LDS traffic,
fabric bytes and L2 hit rate (per launch, counters summed over XCDs/SEs).

  python tools/pmc_compare.py <tag> <flops_per_launch>
"""
import csv, glob, json, os, sys
tag, flops = sys.argv[1], float(sys.argv[2])
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
out = {}
for impl in ("ours", "vendor"):
    stats = glob.glob(os.path.join(root, f"{tag}_{impl}_trace", "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        continue
    rows = sorted(csv.DictReader(open(stats[0])), key=lambda r: -float(r["TotalDurationNs"]))
    top = rows[0]
    name, avg = top["Name"], float(top["AverageNs"]) * 1e-9
    c = {}
    for d in sorted(glob.glob(os.path.join(root, f"{tag}_{impl}_pmc*"))):
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            disp = {}
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"] != name:
                    continue
                disp.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
                disp[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            for nm in {k for v in disp.values() for k in v}:
                vals = [v[nm] for v in disp.values() if nm in v]
                c[nm] = sum(vals) / len(vals)
    res = {"kernel": name[:120], "avg_ms": avg * 1e3, "tflops": flops / avg / 1e12, "counters": c}
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        res["effective_clock_ghz"] = cyc / avg / 1e9
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            res["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc)
    if "FETCH_SIZE" in c:
        res["fabric_read_GB"] = 2.0 * c["FETCH_SIZE"] * 1024 / 1e9
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        res["l2_hit"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    out[impl] = res
print(json.dumps(out, indent=1))
