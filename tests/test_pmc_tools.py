"""The profile tools' PMC aggregation keeps the build launches only (CPU): a configs[4]-style
run also dispatches pb_xpage_kernel once at load for pb_ximg_body's image pages, a small grid
under a build kernel's name, which must not enter the per-launch averages
(scripts/pmc_collect.py -> profiles/pmc_r05.json, the bench line's roofline.traffic)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _csv(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(FIELDS, r)))


def test_setup_dispatches_are_excluded(tmp_path):
    k = "void pb_xpage_kernel<32, 1, false, 512, false>(pb_kargs)"
    rows = [(1, 3072, k, "WRITE_SIZE", 196.0)] + [(i, 45671424, k, "WRITE_SIZE", 3212000.0) for i in range(2, 9)]
    _csv(str(tmp_path / "pmc_c5_icmp_echo_write_size" / "run_counter_collection.csv"), rows)
    _csv(str(tmp_path / "pmc_c5_icmp_echo_fetch_size" / "run_counter_collection.csv"),
         [(1, 3072, k, "FETCH_SIZE", 38.0)] + [(i, 45671424, k, "FETCH_SIZE", 50.0) for i in range(2, 9)])
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_collect.py"), str(tmp_path)], check=True,
                   capture_output=True)
    d = json.load(open(tmp_path / "pmc_summary.json"))
    assert d["per_launch_hbm_bytes"]["c5_icmp_echo"] == int(3212000.0 * 1024 + 2 * 50.0 * 1024)
