"""End-to-end host pipeline rate of pcktbatch-gpu with the in-memory TX ring
(build on the GPU -> land in pinned UMEM slots -> TX descriptors -> completions),
no pcap: frames per second over the whole process run (startup included) and
over the sequence (its own Average PPS line).  One JSON line per case."""
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
CASES = [("udp64", 22, 22, 1 << 25), ("udp1500", 1458, 1458, 1 << 22), ("var64-1500", 64, 1500, 1 << 23)]
env = dict(os.environ, PB_SEQ_GAP_MS="0")
for name, lo, hi, n in CASES:
    for threads in (1, 2, 4):
        for batch in ([1 << 18, 1 << 20] if threads == 1 else [1 << 18]):
            cmd = [BIN] + BASE + ["--pmin", str(lo), "--pmax", str(hi), "--maxpckts", str(n), "--threads",
                                  str(threads), "--gpubatch", str(batch)]
            t0 = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
            dt = time.perf_counter() - t0
            if r.returncode:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            m = re.search(r"total of (\d+) packets and (\d+) bytes", r.stdout)
            pk, by = int(m.group(1)), int(m.group(2))
            print(json.dumps({"case": name, "threads": threads, "gpubatch": batch, "packets": pk, "bytes": by,
                              "wall_s": round(dt, 3), "mpps": round(pk / dt / 1e6, 1),
                              "frame_gbps": round(by / dt / 1e9, 2)}), flush=True)
