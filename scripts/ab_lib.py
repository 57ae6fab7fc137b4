"""In-process A/B of compile-time variants of libpbgpu.so (each loaded side by side
from its own path), alternating variants to cancel box drift.
python3 ab_lib.py CONFIG PACKETS tag:path[:VAR=a,VAR2=b] ..."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg, n = sys.argv[1], int(sys.argv[2])
variants = []
for v in sys.argv[3:]:
    parts = v.split(":")
    env = dict(e.split("=", 1) for e in (parts[2] if len(parts) > 2 else "").split(",") if e)
    variants.append((parts[0], os.path.join(ROOT, parts[1]), env))
keys = {k for _, _, e in variants for k in e}
seq = Sequence.from_config(pc.get(cfg))
ctxs = {t: GpuContext(0, lib_path=p) for t, p, _ in variants}
if os.environ.get("SPAN"):  # one event pair around all of a rep's builds (no per-launch L2 write-back)
    for c in ctxs.values():
        c.set_timing(c.TIMING_SPAN)
res = {t: [] for t, _, _ in variants}
names = {}


def run(tag, env, steps):
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(env)
    ctx = ctxs[tag]
    ctx.load_sequence(0, seq, pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(0, n))
    for s in range(2):
        ctx.build(0, s * n, n, fb)
    ctx.sync()
    ctx.kernel_time()
    for s in range(steps):
        ctx.build(0, (2 + s) * n, n, fb)
    ctx.sync()
    ms, k = ctx.kernel_time()
    fb.free()
    names[tag] = ctx.kernel_name(0)
    return ms / k


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:  # clock ramp
    run(variants[0][0], variants[0][2], 8)
for rep in range(int(os.environ.get("REPS", "5"))):
    for tag, _, env in variants:
        res[tag].append(run(tag, env, 10))
for c in ctxs.values():
    c.close()
for tag, v in res.items():
    v = sorted(v)
    print(json.dumps({"tag": tag, "kernel": names[tag], "ms_med": round(v[len(v) // 2], 5), "ms_min": round(v[0], 5),
                      "ms_all": [round(x, 4) for x in res[tag]]}), flush=True)
