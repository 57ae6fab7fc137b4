"""Summarise rocprofv3 --pmc / --kernel-trace CSVs of one pmc_pass.sh run."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "pb_"
out = {"dir": d, "kernel_filter": kern, "counters": {}, "trace": {}}
for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    waves = None
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"] and "len" not in r["Kernel_Name"] and "scan" not in r["Kernel_Name"]:
            agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (kn, cn), v in agg.items():
        out["counters"].setdefault(kn, {})[cn] = sum(v) / len(v)
for f in glob.glob(os.path.join(d, "trace", "run_kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        out["trace"][r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                   "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]), "pct": float(r["Percentage"])}
for kn, c in out["counters"].items():
    w = c.get("SQ_WAVES")
    print(kn)
    for k, v in sorted(c.items()):
        print(f"   {k:26s} {v:16.0f}" + (f"   per-wave {v / w:10.1f}" if w else ""))
for kn, t in out["trace"].items():
    print(f"trace {kn}: {t}")
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
