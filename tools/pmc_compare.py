"""Summarise tools/h16_vs_vendor.sh output: per implementation, the dominant
kernel's average duration, effective clock, MFMA utilisation (from the
calibrated MOPS counter, tools/pmc_metrics.py), fabric bytes and L2 hit rate
(per launch, counters summed over XCDs/SEs).

  python tools/pmc_compare.py <tag> <flops_per_launch> [dtype]
"""
import csv, glob, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_metrics  # noqa: E402
tag, flops = sys.argv[1], float(sys.argv[2])
dtype = sys.argv[3] if len(sys.argv) > 3 else "bf16"
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
    res.update(pmc_metrics.derive(c, avg, dtype, flops))
    out[impl] = res
print(json.dumps(out, indent=1))
