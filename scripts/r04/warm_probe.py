"""Clock / power ramp probe: back-to-back launches of one config for SECONDS, the span time of
each batch of K launches printed with its start time — how long until the rate settles?

python3 scripts/r04/warm_probe.py CONFIG PACKETS SECONDS [K]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg, n, secs = sys.argv[1], int(sys.argv[2]), float(sys.argv[3])
k = int(sys.argv[4]) if len(sys.argv) > 4 else 50
ctx = GpuContext(0)
ctx.load_sequence(0, Sequence.from_config(pc.get(cfg)), pc.SEED_BASE)
ctx.set_timing(ctx.TIMING_SPAN)
fb = ctx.alloc_frames(*ctx.build_size(0, n))
t0 = time.perf_counter()
rows = []
s = 0
while time.perf_counter() - t0 < secs:
    t = time.perf_counter() - t0
    for _ in range(k):
        ctx.build(0, s * n, n, fb)
        s += 1
    ctx.sync()
    ms, cnt = ctx.kernel_time()
    rows.append((round(t, 2), round(ms / cnt, 4)))
print(json.dumps({"config": cfg, "packets": n, "k": k, "t_s_ms": rows}))
fb.free()
ctx.close()
