"""Store-shape variants across buffer placements: NBUF frame buffers alive at once (each keeps
its own physical placement, and with it its rate: profiles/r04/place_*.jsonl), every variant
timed on every buffer, K back-to-back launches each (span timing), alternating.

python3 scripts/r04/place_ab.py CONFIG PACKETS NBUF K tag:VAR=a,VAR2=b ..."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg, n, nbuf, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
variants = []
for v in sys.argv[5:]:
    tag, _, envs = v.partition(":")
    variants.append((tag, dict(e.split("=", 1) for e in envs.split(",") if e)))
keys = {key for _, e in variants for key in e}
ctx = GpuContext(0)
seq = Sequence.from_config(pc.get(cfg))
ctx.load_sequence(0, seq, pc.SEED_BASE)
ctx.set_timing(ctx.TIMING_SPAN)
bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    ctx.build(0, 0, n, bufs[0])
    ctx.sync()
ctx.kernel_time()
res = {}
for rnd in range(int(os.environ.get("ROUNDS", "2"))):
    for i, fb in enumerate(bufs):
        for tag, env in variants:
            for key in keys:
                os.environ.pop(key, None)
            os.environ.update(env)
            ctx.load_sequence(0, seq, pc.SEED_BASE)  # load-time switches (PBGPU_FST_G, PBGPU_XP_IMG) take effect
            for s in range(k):
                ctx.build(0, s * n, n, fb)
            ctx.sync()
            ms, cnt = ctx.kernel_time()
            res.setdefault((tag, i), []).append(ms / cnt)
addr = [hex(C.cast(fb.ptr.contents.data, C.c_void_p).value or 0) for fb in bufs]
if os.environ.get("FILL"):  # the plain fill shapes over each buffer's own memory (GB/s)
    for key in keys:
        os.environ.pop(key, None)
    # the bytes one build writes (configs[2] writes ~27.6 of its 51.7-GB capacity)
    nb = (min(fb.total_bytes() for fb in bufs) // 65536) * 65536 if not os.environ.get("FILL_CAP") else \
        (bufs[0].f.capacity_bytes // 65536) * 65536
    for i, fb in enumerate(bufs):
        shapes = ctx.fill_probe_at(fb, nb, 5)
        print(json.dumps({"config": cfg, "buf": i, "addr": addr[i], "fill_gbps": {k: round(nb / (v * 1e-3) / 1e9, 1)
                                                                                  for k, v in shapes.items()}}),
              flush=True)
for tag, _ in variants:
    per = [round(min(res[(tag, i)]), 4) for i in range(nbuf)]
    print(json.dumps({"config": cfg, "tag": tag, "kernel": ctx.kernel_name(0), "ms_min_per_buffer": per,
                      "ms_all": {i: [round(x, 4) for x in res[(tag, i)]] for i in range(nbuf)},
                      "addr": addr}), flush=True)
for fb in bufs:
    fb.free()
ctx.close()
