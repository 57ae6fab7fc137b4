"""Per-buffer PMC counters of scripts/place_probe.py run under rocprofv3 --pmc: the last
ROUNDS x NBUF x K dispatches of the build kernel, in place_probe's order (round, buffer,
launch), averaged per buffer.  python3 pmc_place.py counter_collection.csv NBUF K [ROUNDS] [KERNEL]"""
import collections
import csv
import json
import sys

path, nbuf, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
kern = sys.argv[5] if len(sys.argv) > 5 else "pb_vline_kernel"
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    if kern in r["Kernel_Name"]:
        vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(vals)[-rounds * nbuf * k:]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for n, d in enumerate(ids):
    buf = (n // k) % nbuf
    for c, v in vals[d].items():
        per[buf][c].append(v)
for b in range(nbuf):
    print(json.dumps({"buf": b, **{c: round(sum(v) / len(v)) for c, v in sorted(per[b].items())}}))
