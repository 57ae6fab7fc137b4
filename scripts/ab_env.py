"""In-process A/B of library env switches (read per build call), alternating
variants to cancel box drift.  python3 ab_env.py CONFIG PACKETS 'tag:VAR=a,VAR2=b' ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg, n = sys.argv[1], int(sys.argv[2])
variants = []
for v in sys.argv[3:]:
    tag, _, envs = v.partition(":")
    variants.append((tag, dict(e.split("=", 1) for e in envs.split(",") if e)))
keys = {k for _, e in variants for k in e}
ctx = GpuContext(0)
if os.environ.get("SPAN"):  # one event pair around all of a rep's builds: pre-passes included
    ctx.set_timing(ctx.TIMING_SPAN)
seq = Sequence.from_config(pc.get(cfg))
res = {t: [] for t, _ in variants}
# clock ramp: ~0.5 s of untimed launches (bench.py run_config)
import time  # noqa: E402
ctx.load_sequence(0, seq, pc.SEED_BASE)
fb = ctx.alloc_frames(*ctx.build_size(0, n))
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    for s in range(8):
        ctx.build(0, s * n, n, fb)
    ctx.sync()
fb.free()
ctx.kernel_time()
names = {}
for rep in range(int(os.environ.get("REPS", "5"))):
    for tag, env in variants:
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env)
        ctx.load_sequence(0, seq, pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(0, n))
        for s in range(2):
            ctx.build(0, s * n, n, fb)
        ctx.sync()
        ctx.kernel_time()
        for s in range(10):
            ctx.build(0, (2 + s) * n, n, fb)
        ctx.sync()
        ms, k = ctx.kernel_time()
        nbytes = fb.total_bytes() if hasattr(fb, "total_bytes") else None
        fb.free()
        names[tag] = ctx.kernel_name(0)
        res[tag].append(ms / k)
bpl = ctx.build_size(0, n)[1]
ctx.close()
for tag, v in res.items():
    v = sorted(v)
    print(json.dumps({"tag": tag, "kernel": names[tag], "ms_med": round(v[len(v) // 2], 5), "ms_min": round(v[0], 5),
                      "ms_all": [round(x, 4) for x in res[tag]]}))
