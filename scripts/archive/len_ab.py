"""pb_xpage_kernel (forced) vs the linear small kernel over frame lengths, in process.
python3 len_ab.py [udp|small]"""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

ctx = GpuContext(0)
ctx.set_timing(ctx.TIMING_SPAN)
CASES = [(p, f, r) for p, f, r in (
    ("udp", 60, 1), ("udp", 60, 4), ("udp", 100, 4), ("udp", 120, 4),
    ("tcp", 60, 4), ("tcp", 60, 1), ("tcp", 72, 4), ("tcp", 100, 4), ("tcp", 120, 4))]
if len(sys.argv) > 1 and sys.argv[1] == "udp":
    CASES = [("udp", f, 1) for f in (44, 48, 60, 72, 100, 120, 124)]
if len(sys.argv) > 1 and sys.argv[1] == "small":
    CASES = [("udp", f, 1) for f in (44, 48, 52, 56, 60)] + [("udp", 60, 4), ("tcp", 56, 4), ("tcp", 60, 4)]
for proto, flen, nr in CASES:
    cfg = copy.deepcopy(pc.get("c4_tcp_syn" if proto == "tcp" else "c2_udp_64"))
    hl = 54 if proto == "tcp" else 42
    cfg["payloads"] = [{"length": {"min": flen - hl, "max": flen - hl}}]
    cfg["ip"]["ranges"] = pc.get("c4_tcp_syn")["ip"]["ranges"][:nr]
    n = (2 << 30) // flen
    res = {}
    for rep in range(3):
        for tag, env in (("xpage", None), ("linear", "nopage")):
            if env:
                os.environ["PBGPU_KERNEL"] = env
                os.environ.pop("PBGPU_XP_FORCE", None)
            else:
                os.environ.pop("PBGPU_KERNEL", None)
                os.environ["PBGPU_XP_FORCE"] = "1"
            ctx.load_sequence(0, Sequence.from_config(cfg), pc.SEED_BASE)
            fb = ctx.alloc_frames(*ctx.build_size(0, n))
            for s in range(3):
                ctx.build(0, s * n, n, fb)
            ctx.sync()
            ctx.kernel_time()
            for s in range(10):
                ctx.build(0, s * n, n, fb)
            ctx.sync()
            ms, k = ctx.kernel_time()
            fb.free()
            res.setdefault(tag, []).append(round(ms / k, 4))
            res[tag + "_kernel"] = ctx.kernel_name(0)
    print(json.dumps({"proto": proto, "flen": flen, "ranges": nr, **res}))
ctx.close()
