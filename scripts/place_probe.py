"""Does the frames buffer's placement set the 1500-B rate?  Several buffers alive at once,
each built into K times in a row (span timing), per-launch ms per buffer with its device
address.  python3 place_probe.py [CONFIG] [PACKETS] [NBUF] [K]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2_udp_1500"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 25
nbuf = int(sys.argv[3]) if len(sys.argv) > 3 else 4
k = int(sys.argv[4]) if len(sys.argv) > 4 else 6
ctx = GpuContext(0)
ctx.load_sequence(0, Sequence.from_config(pc.get(cfg)), pc.SEED_BASE)
ctx.set_timing(ctx.TIMING_SPAN)
bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    ctx.build(0, 0, n, bufs[0])
    ctx.sync()
ctx.kernel_time()
for rnd in range(3):
    for i, fb in enumerate(bufs):
        for s in range(k):
            ctx.build(0, s * n, n, fb)
        ctx.sync()
        ms, cnt = ctx.kernel_time()
        print(json.dumps({"round": rnd, "buf": i, "addr": hex(C.cast(fb.ptr.contents.data, C.c_void_p).value or 0),
                          "ms_per_launch": round(ms / cnt, 4)}), flush=True)
for fb in bufs:
    fb.free()
ctx.close()
