"""pb_xpage_kernel (forced, 256- and 512-thread workgroups) vs the linear small
kernel over frame lengths and payload kinds, in process (span timing).  Lengths
not a multiple of 4 were measured with a byte-phase xpage instance since
reverted (profiles/r01/xpage/len_gt64.txt); without it they fall to the linear kernel.
python3 xp_len_ab.py"""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
import pbgpu  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

if os.environ.get("PBGPU_LIB_AB"):  # A/B against another build of the library
    pbgpu.load_library(os.environ["PBGPU_LIB_AB"])

VARIANTS = [("linear", {"PBGPU_KERNEL": "nopage"}), ("xp256", {"PBGPU_XP_FORCE": "1"}),
            ("xp512", {"PBGPU_XP_FORCE": "1", "PBGPU_XP_WGT": "512"})]
EXTRA = os.environ.get("XP_EXTRA")  # e.g. "xp512np4:PBGPU_XP_FORCE=1,PBGPU_XP_WGT=512,PBGPU_XP_NP=4"
if EXTRA:
    for v in EXTRA.split():
        tag, kv = v.split(":", 1)
        VARIANTS.append((tag, dict(x.split("=") for x in kv.split(","))))
KEYS = {k for _, e in VARIANTS for k in e}


def case(name, flen=None):
    cfg = copy.deepcopy(pc.get(name))
    if flen is not None:
        hl = 54 if "tcp" in cfg else 42
        cfg["payloads"] = [{"length": {"min": flen - hl, "max": flen - hl}}]
    return cfg


CASES = [("c5_icmp_echo", None), ("c1_udp_static_106", None), ("c2_udp_64", 98), ("c2_udp_64", 100),
         ("c2_udp_64", 72), ("c2_udp_64", 124), ("c4_tcp_syn", 120), ("c2_udp_64", 44), ("c4_tcp_syn", None)]
if os.environ.get("XP_CASES"):
    CASES = [(c.split(":")[0], int(c.split(":")[1]) if ":" in c else None) for c in os.environ["XP_CASES"].split()]

ctx = GpuContext(0)
ctx.set_timing(ctx.TIMING_SPAN)
for name, flen in CASES:
    cfg = case(name, flen)
    seq = Sequence.from_config(cfg)
    res = {}
    for rep in range(int(os.environ.get("REPS", "3"))):
        for tag, env in VARIANTS:
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            ctx.load_sequence(0, seq, pc.SEED_BASE)
            n = 1 << 25
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
    for k in KEYS:
        os.environ.pop(k, None)
    print(json.dumps({"case": name, "flen": flen, "n": n, **res}), flush=True)
ctx.close()
