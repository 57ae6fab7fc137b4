"""Per-(kernel, grid) dispatch statistics from a rocprofv3 --kernel-trace CSV,
so the average duration can be matched against bench.py's HIP-event timing
(same kernel, same grid = same launch shape).  bench.py's timed region is the
run of STEPS launches before the LAUNCH_REPS per-launch-timed ones that precede its first
write-probe (pb_fill_kernel) launch; "timed_window" reports those alone (the all-launch average includes the
clock-ramp launches).  python3 trace_summary.py trace.csv out.json [STEPS [LAUNCH_REPS]]"""
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
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20  # bench.py run_configs(launch_reps=20)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first_fill = next((i for i, r in enumerate(rows) if "pb_fill_kernel" in r["Kernel_Name"]), None)
if first_fill is not None and out:
    # the frame-build launches (the busiest kernel shape before the probe), runtime copies skipped
    pre = collections.Counter()
    for r in rows[:first_fill]:
        pre[(r["Kernel_Name"], int(r["Grid_Size_X"]))] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    k, grid = pre.most_common(1)[0][0]
    runs = [r for r in rows[:first_fill] if r["Kernel_Name"] == k and int(r["Grid_Size_X"]) == grid]
    # the timed window: the `steps` launches before bench.py's per-launch pass (its last
    # LAUNCH_REPS launches, with an event pair and so an L2 write-back between launches)
    win = runs[len(runs) - steps - reps:len(runs) - reps] if len(runs) >= steps + reps else []
    if len(win) == steps:
        d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
        out.insert(0, {"timed_window": True, "kernel": k, "grid_threads": grid, "calls": len(d),
                       "avg_ms": sum(d) / len(d) / 1e6, "median_ms": d[len(d) // 2] / 1e6,
                       "min_ms": d[0] / 1e6, "max_ms": d[-1] / 1e6})
json.dump(out, open(sys.argv[2], "w"), indent=1)
for e in out:
    tag = " (timed window)" if e.get("timed_window") else ""
    print(f"{e['kernel'][:60]:60s} grid={e['grid_threads']:>10d} n={e['calls']:3d} avg={e['avg_ms']:.4f} ms{tag}")
