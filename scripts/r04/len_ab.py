"""Small-frame kernel shapes by frame length: for each length, NBUF buffers alive at once and
every variant timed on every buffer (span timing, K launches), load-time switches applied by
reloading the sequence.  python3 len_ab.py PROTO NBUF K LEN,LEN,... tag:VAR=a,VAR2=b ...
PROTO: icmp (static payload, as configs[4]'s ICMP) or udp (random payload, as configs[1])."""
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

proto, nbuf, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
lens = [int(x) for x in sys.argv[4].split(",")]
variants = []
for v in sys.argv[5:]:
    tag, _, envs = v.partition(":")
    variants.append((tag, dict(e.split("=", 1) for e in envs.split(",") if e)))
keys = {key for _, e in variants for key in e}
n = 1 << 25
ctx = GpuContext(0)
ctx.set_timing(ctx.TIMING_SPAN)
for flen in lens:
    if proto == "icmp":
        cfg = copy.deepcopy(pc.get("c5_icmp_echo"))
        cfg["payloads"] = [{"exact": " ".join("%02X" % (i * 7 & 255) for i in range(flen - 42))}]
    else:
        cfg = copy.deepcopy(pc.get("c2_udp_64"))
        cfg["payloads"] = [{"length": {"min": flen - 42, "max": flen - 42}}]
    seq = Sequence.from_config(cfg)
    ctx.load_sequence(0, seq, pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        ctx.build(0, 0, n, bufs[0])
        ctx.sync()
    ctx.kernel_time()
    res = {}
    for rnd in range(2):
        for i, fb in enumerate(bufs):
            for tag, env in variants:
                for key in keys:
                    os.environ.pop(key, None)
                os.environ.update(env)
                ctx.load_sequence(0, seq, pc.SEED_BASE)
                for s in range(k):
                    ctx.build(0, s * n, n, fb)
                ctx.sync()
                ms, cnt = ctx.kernel_time()
                res.setdefault(tag, {}).setdefault(i, []).append(ms / cnt)
                res.setdefault("_k", {})[tag] = ctx.kernel_name(0)
    for tag, _ in variants:
        print(json.dumps({"proto": proto, "flen": flen, "tag": tag, "kernel": res["_k"][tag],
                          "ms_min_per_buffer": [round(min(res[tag][i]), 4) for i in range(nbuf)]}), flush=True)
    for fb in bufs:
        fb.free()
ctx.close()
