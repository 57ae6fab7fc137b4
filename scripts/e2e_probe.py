"""End-to-end host pipeline rate of pcktbatch-gpu with the in-memory TX ring
(build on the GPU -> land in pinned UMEM slots -> TX descriptors -> completions),
no pcap.  Each case runs at N and 4N frames: the steady-state rate is the slope
3N / (t(4N) - t(N)), which cancels process start and GPU initialisation; the
whole-run rate of the 4N run is reported beside it.  One JSON line per case.
Environment: E2E_CASES (comma list of case names), E2E_THREADS (comma list), E2E_ARGS (extra
pcktbatch-gpu options, e.g. "--umemslot 64"), E2E_BATCHES (comma list of --gpubatch values),
E2E_SCALE (multiplies every case's N)."""
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "pb-af-xdp_amd", "bin", "pcktbatch-gpu")
BASE = ["-z", "--interface", "pbnodev0", "--smac", "52:54:00:59:29:cc", "--dmac", "52:54:00:d5:50:54",
        "--dip", "10.60.0.195", "--sip", "10.20.0.0/16", "--protocol", "udp", "--udport", "27015",
        "--delay", "0", "--track", "1"]
CASES = [("udp64", 22, 22, 1 << 24), ("udp1500", 1458, 1458, 1 << 21), ("var64-1500", 64, 1500, 1 << 22)]
env = dict(os.environ, PB_SEQ_GAP_MS="0")
EXTRA = os.environ.get("E2E_ARGS", "").split()
if os.environ.get("E2E_CASES"):
    CASES = [c for c in CASES if c[0] in os.environ["E2E_CASES"].split(",")]
CASES = [(c[0], c[1], c[2], c[3] * int(os.environ.get("E2E_SCALE", "1"))) for c in CASES]
THREADS = [int(t) for t in os.environ.get("E2E_THREADS", "1,2,4").split(",")]
BATCHES = [int(b, 0) for b in os.environ["E2E_BATCHES"].split(",")] if os.environ.get("E2E_BATCHES") else None


def run(lo, hi, n, threads, batch):
    cmd = [BIN] + BASE + ["--pmin", str(lo), "--pmax", str(hi), "--maxpckts", str(n), "--threads", str(threads),
                          "--gpubatch", str(batch)] + EXTRA
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    dt = time.perf_counter() - t0
    if r.returncode:
        print(r.stderr[-2000:], file=sys.stderr)
        sys.exit(1)
    m = re.search(r"total of (\d+) packets and (\d+) bytes", r.stdout)
    return int(m.group(1)), int(m.group(2)), dt


for name, lo, hi, n in CASES:
    for threads in THREADS:
        for batch in BATCHES or ([1 << 18, 1 << 20] if threads == 1 else [1 << 18]):
            p1, b1, t1 = run(lo, hi, n, threads, batch)
            p4, b4, t4 = run(lo, hi, 4 * n, threads, batch)
            slope = t4 - t1
            print(json.dumps({"case": name, "args": " ".join(EXTRA), "threads": threads, "gpubatch": batch,
                              "packets": [p1, p4],
                              "wall_s": [round(t1, 3), round(t4, 3)],
                              "steady_mpps": round((p4 - p1) / slope / 1e6, 1),
                              "steady_frame_gbps": round((b4 - b1) / slope / 1e9, 2),
                              "whole_run_mpps": round(p4 / t4 / 1e6, 1)}), flush=True)
