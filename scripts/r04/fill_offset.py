"""Store-shape alignment probe: the write-probe shapes over NBUF configs[2]-sized buffers (each
keeps its own placement), at byte offsets OFFS from each buffer's start, alongside the packed
kernel's own time on that buffer — do region stores off the 4-KiB grid lose in a slow placement?

python3 scripts/r04/fill_offset.py NBUF NBYTES OFF[,OFF...]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

nbuf, nbytes, offs = int(sys.argv[1]), int(sys.argv[2]), [int(x) for x in sys.argv[3].split(",")]
ctx = GpuContext(0)
ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
ctx.set_timing(ctx.TIMING_SPAN)
n = 1 << 25
bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
names = [ctx.lib.pbgpu_fill_shape_name(i).decode() for i in range(ctx.FILL_SHAPES)]
keep = [i for i, nm in enumerate(names) if "region" in nm or "XCD" in nm]
for i, fb in enumerate(bufs):
    for s in range(10):
        ctx.build(0, s * n, n, fb)
    ctx.sync()
    ms, cnt = ctx.kernel_time()
    row = {"buf": i, "vline_ms": round(ms / cnt, 4)}
    d = fb.f.data
    base = d if isinstance(d, int) else C.cast(d, C.c_void_p).value
    for off in offs:
        out = (C.c_double * ctx.FILL_SHAPES)()
        rc = ctx.lib.pbgpu_fill_probe_at(ctx.h, C.c_void_p(base + off), nbytes, 5, out)
        assert rc == 0, rc
        row[f"off{off}"] = {names[k]: round(nbytes / (out[k] * 1e-3) / 1e9, 1) for k in keep}
    print(json.dumps(row), flush=True)
for fb in bufs:
    fb.free()
ctx.close()
