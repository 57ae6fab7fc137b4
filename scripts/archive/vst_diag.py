"""Diagnose a vstage parity failure: per-frame mismatch summary for configs[2] under env variants."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd"), os.path.join(ROOT, "tests")]
import oracle_binding as ob  # noqa: E402
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

ctx = GpuContext(0)
seq = Sequence.from_config(pc.get("c3_udp_var"))
n = int(os.environ.get("N", "4000"))
o_data, o_off = ob.build(seq, 5, 7, n, pc.SEED_BASE)
for tag in sys.argv[1:]:
    os.environ.pop("PBGPU_FST_DBG", None)
    if tag != "-":
        os.environ["PBGPU_FST_DBG"] = tag
    ctx.load_sequence(5, seq, pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(5, n))
    ctx.build(5, 7, n, fb)
    ctx.sync()
    g = fb.packed()
    fb.free()
    bad = np.nonzero(g != o_data)[0]
    print(tag, ctx.kernel_name(5), "bad bytes", bad.size, "of", g.size)
    if bad.size:
        fr = np.searchsorted(o_off, bad, side="right") - 1
        uf = np.unique(fr)
        print(" bad frames", uf.size, "first", uf[:20].tolist())
        for f in uf[:6]:
            b = bad[fr == f] - o_off[f]
            ln = o_off[f + 1] - o_off[f]
            print("  frame", int(f), "len", int(ln), "start%16", int(o_off[f] % 16), "nbad", b.size, "offs", b[:12].tolist(), "...", b[-4:].tolist())
        lens = np.diff(o_off)
        print("  first 40 frames: len / bad", [(int(lens[i]), int(i in set(uf.tolist()))) for i in range(40)])
        f = int(uf[0])
        s = int(o_off[f])
        print("  got ", g[s:s + 48].tobytes().hex())
        print("  want", o_data[s:s + 48].tobytes().hex())
ctx.close()
