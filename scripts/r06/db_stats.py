"""Per-kernel statistics from a rocprofv3 rocpd database (--kernel-trace; ROCm 7.2's default
output): name, dispatches, average / min / max duration (ms), grid, VGPRs, LDS.
python3 scripts/r06/db_stats.py <run_results.db> [--json out.json]"""
import json
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute(
    "select name, count(*), avg(duration) / 1e6, min(duration) / 1e6, max(duration) / 1e6, max(grid_x), "
    "max(vgpr_count), max(lds_size) from kernels group by name, grid_x order by sum(duration) desc").fetchall()
out = []
for r in rows:
    d = {"kernel": r[0], "dispatches": r[1], "avg_ms": round(r[2], 5), "min_ms": round(r[3], 5),
         "max_ms": round(r[4], 5), "grid_x": r[5], "vgpr": r[6], "lds": r[7]}
    out.append(d)
    print(f"{r[0][:80]:80s} n={r[1]:4d} avg={r[2]:.4f} min={r[3]:.4f} max={r[4]:.4f} grid={r[5]} vgpr={r[6]} lds={r[7]}")
if "--json" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
