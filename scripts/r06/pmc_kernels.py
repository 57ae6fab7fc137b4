"""Per-kernel mean PMC values from rocprofv3 --pmc --output-format csv runs (tool only).
python3 scripts/r06/pmc_kernels.py <run_counter_collection.csv>... [--match substr]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in args:
    if path == match:
        continue
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        if match and match not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.0f}  (n={len(v)})")
