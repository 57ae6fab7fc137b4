"""Same-box A/B of two builds of libpbgpu.so (tool only): each rep runs every library in a fresh
child process that times `steps` span-mode builds of one config after a 0.5-s ramp.
python3 scripts/r05/lib_ab.py CONFIG REPS LIB_A LIB_B ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import sys, time
sys.path[:0] = [%r, %r]
import pb_configs as pc
from pbgpu import GpuContext, Sequence
cfg, lib = sys.argv[1], sys.argv[2]
ctx = GpuContext(0, lib_path=lib)
names = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"] if cfg == "c5_mix" else [cfg]
n = 1 << 24 if cfg == "c5_mix" else 1 << 25
for i, nm in enumerate(names):
    ctx.load_sequence(i, Sequence.from_config(pc.get(nm)), pc.SEED_BASE)
bufs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(len(names))]
ctx.set_timing(ctx.TIMING_SPAN)
def step(s):
    if len(names) > 1:
        ctx.build_batch([(i, s * n, n, bufs[i]) for i in range(len(names))])
    else:
        ctx.build(0, s * n, n, bufs[0])
t = time.perf_counter()
while time.perf_counter() - t < 0.5:
    for s in range(8):
        step(s)
    ctx.sync()
ctx.kernel_time()
for s in range(50):
    step(s)
ctx.sync()
ms, k = ctx.kernel_time()
print(ms / k)
''' % (ROOT, os.path.join(ROOT, "pb-af-xdp_amd"))

cfg, reps, libs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for r in range(reps):
    row = {"config": cfg, "rep": r}
    for lib in libs:
        out = subprocess.run([sys.executable, "-c", CHILD, cfg, lib], capture_output=True, text=True, timeout=240)
        if out.returncode:
            raise SystemExit(out.stderr[-2000:])
        row[os.path.basename(os.path.dirname(lib)) + "/" + os.path.basename(lib)] = round(float(out.stdout.split()[-1]), 5)
    print(json.dumps(row), flush=True)
