"""Diagnostic: pcktbatch-gpu variable TCP capture vs the oracle, first mismatches."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pb-af-xdp_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import oracle_binding as ob  # noqa: E402
import pb_configs as pc  # noqa: E402
from pbgpu import Sequence  # noqa: E402
from test_gpu_host import BIN, read_pcap  # noqa: E402

pcap = "/tmp/diag_tcp.pcap"
cmd = [BIN, "-z", "--interface", "eth0", "--dip", pc.DIP, "--sip", "172.16.0.0/12", "--protocol", "tcp",
       "--tdport", "80", "--syn", "1", "--pmin", "0", "--pmax", "900", "--maxpckts", "3000", "--delay", "0",
       "--gpubatch", sys.argv[1] if len(sys.argv) > 1 else "1000", "--seed", "7", "--pcap", pcap, "-v"]
r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
print("rc", r.returncode, r.stdout[-600:], r.stderr[-600:])
got = read_pcap(pcap)
cfg = {"eth": {}, "ip": {"dip": pc.DIP, "ranges": ["172.16.0.0/12"], "protocol": "tcp"},
       "tcp": {"dport": 80, "syn": 1}, "payloads": [{"length": {"min": 0, "max": 900}}]}
want = ob.frames(Sequence.from_config(cfg), 0, 0, 3000, 7)
print("got", len(got), "want", len(want))
n = 0
for i in range(min(len(got), len(want))):
    if got[i] != want[i]:
        n += 1
        if n < 8:
            g, w = got[i], want[i]
            d = next((j for j in range(min(len(g), len(w))) if g[j] != w[j]), None)
            print(f"frame {i}: len {len(g)} want {len(w)} first diff byte {d}")
print("mismatches", n)
