"""bench.py keeps the driver's contract: one JSON line with the BASELINE metric,
the roofline and CPU-baseline objects, and numbers that add up.  A short run of
the real script (small launches) on the MI355X box."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "1", "--packets",
           str(1 << 20), "--ramp-seconds", "0.05", "--cpu-seconds", "0.4"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["vs_baseline"] is None
    # value = packets per second of the timed launches (Mpps), ms_per_step their wall time
    assert abs(d["value"] - (1 << 20) / (d["ms_per_step"] * 1e-3) / 1e6) < 0.01 * d["value"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["algorithmic_bytes_per_launch"] == (1 << 20) * 64
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert 0.05 < r["frac"] < 1.0
    assert d["config"]["workload"].startswith("c2_udp_64")
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    assert d["udp_1500"]["kernel"].startswith("pb_fstage_kernel")
