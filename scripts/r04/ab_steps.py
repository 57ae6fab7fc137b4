"""In-process A/B of bench-shaped step loops (span timing, back-to-back launches),
alternating variants rep by rep to cancel box drift.

python3 scripts/r04/ab_steps.py CONFIG PACKETS tag:lib[:nbufs[:VAR=a,VAR2=b]] ...
  lib    : libpbgpu.so path relative to the repo ('-' = the in-tree library)
  nbufs  : output buffers per sequence the steps alternate between (default 1)
Env: REPS (default 6), STEPS (default 40).  CONFIG may be c5_mix (three sequences); a variant
with AB_BATCH=1 builds them with one pbgpu_build_batch call per step."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg, n = sys.argv[1], int(sys.argv[2])
names = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"] if cfg == "c5_mix" else [cfg]
variants = []
for v in sys.argv[3:]:
    parts = v.split(":")
    lib = None if parts[1] == "-" else os.path.join(ROOT, parts[1])
    nb = int(parts[2]) if len(parts) > 2 and parts[2] else 1
    env = dict(e.split("=", 1) for e in (parts[3] if len(parts) > 3 else "").split(",") if e)
    variants.append((parts[0], lib, nb, env))
keys = {k for *_, e in variants for k in e}
ctxs = {}
for tag, lib, nb, env in variants:
    c = GpuContext(0, lib_path=lib) if lib else GpuContext(0)
    c.set_timing(c.TIMING_SPAN)
    for i, nm in enumerate(names):
        c.load_sequence(i, Sequence.from_config(pc.get(nm)), pc.SEED_BASE)
    ctxs[tag] = c
res = {t: [] for t, *_ in variants}
knames = {}
steps = int(os.environ.get("STEPS", "40"))


def run(tag, nb, env, k):
    for key in keys:
        os.environ.pop(key, None)
    os.environ.update(env)
    ctx = ctxs[tag]
    for i, nm in enumerate(names):  # load-time switches (PBGPU_FST_G and the other shapes) take effect
        ctx.load_sequence(i, Sequence.from_config(pc.get(nm)), pc.SEED_BASE)
    bufs = [[ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(len(names))] for _ in range(nb)]
    def step(first, row):
        if os.environ.get("AB_BATCH") == "1":
            ctx.build_batch([(i, first, n, row[i]) for i in range(len(names))])
        else:
            for i in range(len(names)):
                ctx.build(i, first, n, row[i])

    for s in range(2 * nb):
        step(s * n, bufs[s % nb])
    ctx.sync()
    ctx.kernel_time()
    for s in range(k):
        step((2 * nb + s) * n, bufs[s % nb])
    ctx.sync()
    ms, _ = ctx.kernel_time()
    for row in bufs:
        for fb in row:
            fb.free()
    knames[tag] = [ctx.kernel_name(i) for i in range(len(names))]
    return ms / k


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:  # clock ramp
    run(variants[0][0], variants[0][2], variants[0][3], 8)
for rep in range(int(os.environ.get("REPS", "6"))):
    for tag, _, nb, env in variants:
        res[tag].append(run(tag, nb, env, steps))
for c in ctxs.values():
    c.close()
for tag, _, nb, env in variants:
    v = sorted(res[tag])
    print(json.dumps({"config": cfg, "tag": tag, "nbufs": nb, "env": env, "kernels": knames[tag],
                      "ms_per_step_med": round(v[len(v) // 2], 5), "ms_min": round(v[0], 5),
                      "ms_all": [round(x, 4) for x in res[tag]]}), flush=True)
