"""Per-(kernel, grid) dispatch statistics from a rocprofv3 --kernel-trace CSV,
so the average duration can be matched against bench.py's HIP-event timing
(same kernel, same grid = same launch shape)."""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
g = collections.defaultdict(list)
for r in rows:
    g[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = []
for (k, grid), v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    out.append({"kernel": k, "grid_threads": grid, "calls": len(v), "avg_ms": sum(v) / len(v) / 1e6,
                "median_ms": v[len(v) // 2] / 1e6, "min_ms": v[0] / 1e6, "max_ms": v[-1] / 1e6})
json.dump(out, open(sys.argv[2], "w"), indent=1)
for e in out:
    print(f"{e['kernel'][:60]:60s} grid={e['grid_threads']:>10d} n={e['calls']:3d} avg={e['avg_ms']:.4f} ms")
