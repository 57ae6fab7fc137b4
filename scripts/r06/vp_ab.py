"""configs[2] kernels (or VP_CFG's) side by side in one process on the same buffers (tool only):
python3 scripts/r06/vp_ab.py [reps] [nbuf] [variants...]
variants: PBGPU_KERNEL values, or VAR=val[,VAR2=val2] load-time settings, to load (default: "" = the
library default, and "vpage"); each is
loaded into its own slot, then every buffer is built by every variant, reps rounds, 10 launches per
timing (TIMING_LAUNCH medians).  One JSON line per (buffer, variant)."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
NBUF = int(sys.argv[2]) if len(sys.argv) > 2 else 2
VARS = sys.argv[3:] or ["", "vpage"]
n = 1 << 25
ctx = GpuContext(0)
seq = Sequence.from_config(pc.get(os.environ.get("VP_CFG", "c3_udp_var")))  # VP_CFG: another BASELINE config
names = {}
ENV_KEYS = {"PBGPU_KERNEL"}
for i, v in enumerate(VARS):
    # (the round-6 forms vpage:512 and vpage:pool selected kernels since removed)
    env = dict(e.split("=", 1) for e in v.split(",")) if "=" in v else {"PBGPU_KERNEL": v} if v else {}
    for key in set(ENV_KEYS) | set(env):
        os.environ.pop(key, None)
    os.environ.update(env)
    ENV_KEYS.update(env)
    ctx.load_sequence(i, seq, pc.SEED_BASE)
    names[i] = ctx.kernel_name(i)
for key in ENV_KEYS:
    os.environ.pop(key, None)
bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(NBUF)]
ctx.set_timing(ctx.TIMING_LAUNCH)
t0 = time.perf_counter()
while time.perf_counter() - t0 < float(os.environ.get("VP_RAMP", "0.6")):
    ctx.build(0, 0, n, bufs[0])
ctx.sync()
ctx.kernel_times()
res = {}
for r in range(REPS):
    for b, fb in enumerate(bufs):
        for i in range(len(VARS)):
            for k in range(int(os.environ.get("VP_LAUNCHES", "10"))):
                ctx.build(i, k * n, n, fb)
            ctx.sync()
            t = ctx.kernel_times()
            res.setdefault((b, i), []).append(float(statistics.median(t)))
for (b, i), v in sorted(res.items()):
    print(json.dumps({"buf": b, "variant": VARS[i] or "default", "kernel": names[i], "ms_med": round(statistics.median(v), 4),
                      "ms_min": round(min(v), 4), "all": [round(x, 4) for x in v]}), flush=True)
