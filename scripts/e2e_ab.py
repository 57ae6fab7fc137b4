"""Host-pipeline A/B: pcktbatch-gpu (build -> land in pinned UMEM slots -> TX
descriptors on the in-memory ring, no pcap) for one case under several
environment variants (landing chunk / landings in flight / spin waits, or any
library switch).  Steady rate = 3N / (t(4N) - t(N)), as scripts/e2e_probe.py.
python3 e2e_ab.py CASE THREADS 'tag:VAR=a,VAR2=b' ...   CASE: udp64 | udp1500 | var
(ARGS=... in a variant appends command-line arguments.)"""
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
        "--delay", "0", "--track", "1", "--seed", "1"]
CASES = {"udp64": (22, 22, 1 << 24), "udp1500": (1458, 1458, 1 << 21), "var": (64, 1500, 1 << 22)}


def run(env, lo, hi, n, threads, batch, extra=()):
    cmd = [BIN] + BASE + ["--pmin", str(lo), "--pmax", str(hi), "--maxpckts", str(n), "--threads", str(threads),
                          "--gpubatch", str(batch)] + list(extra)
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    dt = time.perf_counter() - t0
    if r.returncode:
        print(r.stderr[-2000:], file=sys.stderr)
        sys.exit(1)
    m = re.search(r"total of (\d+) packets and (\d+) bytes", r.stdout)
    return int(m.group(1)), int(m.group(2)), dt


case, threads = sys.argv[1], int(sys.argv[2])
lo, hi, n = CASES[case]
variants = []
for v in sys.argv[3:]:
    tag, _, envs = v.partition(":")
    variants.append((tag, dict(e.split("=", 1) for e in envs.split(",") if e)))
for rep in range(int(os.environ.get("REPS", "2"))):
    for tag, extra in variants:
        env = dict(os.environ, PB_SEQ_GAP_MS="0", **extra)
        batch = int(extra.get("GPUBATCH", 1 << 18))
        nn = int(extra.get("N", n))  # frames of the short run (the long one sends 4x)
        args = extra.get("ARGS", "").split()  # extra command-line arguments ('ARGS=--umemframes 16384')
        p1, b1, t1 = run(env, lo, hi, nn, threads, batch, args)
        p4, b4, t4 = run(env, lo, hi, 4 * nn, threads, batch, args)
        slope = t4 - t1
        print(json.dumps({"case": case, "tag": tag, "env": extra, "threads": threads, "rep": rep,
                          "steady_mpps": round((p4 - p1) / slope / 1e6, 1),
                          "steady_frame_gbps": round((b4 - b1) / slope / 1e9, 2),
                          "wall_s": [round(t1, 3), round(t4, 3)]}), flush=True)
