"""Inter-launch gaps of back-to-back build launches from a rocprofv3 --kernel-trace CSV.

For each kernel (name, grid) with >= MIN launches: launch duration, the gap from a
launch's end to the next launch's start (negative = the launches overlap), and the
per-launch span of each run of back-to-back launches (runs split at gaps > 200 us,
i.e. at the host-side pauses between reps).  python3 gaps.py trace.csv [out.json]"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    by[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
out = []
for (k, grid), v in by.items():
    if len(v) < 8:
        continue
    v.sort()
    dur = [e - s for s, e in v]
    gaps = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
    runs, cur = [], [v[0]]
    for i in range(1, len(v)):
        if v[i][0] - v[i - 1][1] > 200_000:
            runs.append(cur)
            cur = []
        cur.append(v[i])
    runs.append(cur)
    spans = [((r[-1][1] - r[0][0]) / len(r)) / 1e6 for r in runs if len(r) >= 8]
    med = lambda x: sorted(x)[len(x) // 2] if x else None  # noqa: E731
    inrun = [g for g in gaps if g <= 200_000]
    out.append({"kernel": k, "grid_threads": grid, "launches": len(v), "dur_ms_med": med(dur) / 1e6,
                "dur_ms_avg": sum(dur) / len(dur) / 1e6,
                "gap_us_med": med(inrun) / 1e3 if inrun else None,
                "gap_us_min": min(inrun) / 1e3 if inrun else None, "gap_us_max": max(inrun) / 1e3 if inrun else None,
                "overlapping_pairs": sum(1 for g in inrun if g < 0), "runs": len(spans),
                "span_ms_per_launch_runs": [round(x, 5) for x in spans]})
out.sort(key=lambda e: -e["launches"] * e["dur_ms_avg"])
for e in out:
    print(json.dumps(e))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
