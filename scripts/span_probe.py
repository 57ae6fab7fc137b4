"""Per-launch event pairs vs span timing: wall time per back-to-back build launch
(and what each mode's kernel_time reports), alternating modes to cancel drift.
python3 span_probe.py CONFIG PACKETS"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg, n = sys.argv[1], int(sys.argv[2])
steps = 100
ctx = GpuContext(0)
ctx.load_sequence(0, Sequence.from_config(pc.get(cfg)), pc.SEED_BASE)
fb = ctx.alloc_frames(*ctx.build_size(0, n))
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    for s in range(8):
        ctx.build(0, s * n, n, fb)
    ctx.sync()
res = {0: [], 1: []}
for rep in range(4):
    for mode in (0, 1):
        ctx.set_timing(mode)
        for s in range(5):
            ctx.build(0, s * n, n, fb)
        ctx.sync()
        ctx.kernel_time()
        t0 = time.perf_counter()
        for s in range(steps):
            ctx.build(0, s * n, n, fb)
        ctx.sync()
        wall = (time.perf_counter() - t0) / steps * 1e3
        ms, k = ctx.kernel_time()
        res[mode].append((round(wall, 4), round(ms / k, 4)))
for mode, v in res.items():
    print(json.dumps({"config": cfg, "mode": ["launch", "span"][mode], "wall_ms_per_step,kernel_time_ms": v}))
fb.free()
ctx.close()
