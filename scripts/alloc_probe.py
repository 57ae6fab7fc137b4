"""Does the kernel time depend on which allocation the frames land in?
Allocates several frame buffers, builds into each in turn (same launch), prints
per-buffer kernel ms and the buffer's device address."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg, n, nbuf = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
ctx = GpuContext(0)
seq = Sequence.from_config(pc.get(cfg))
ctx.load_sequence(0, seq, pc.SEED_BASE)
bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
for rep in range(3):
    row = []
    for fb in bufs:
        for s in range(2):
            ctx.build(0, s * n, n, fb)
        ctx.sync()
        ctx.kernel_time()
        for s in range(10):
            ctx.build(0, s * n, n, fb)
        ctx.sync()
        ms, k = ctx.kernel_time()
        row.append(f"{ms / k:.4f}@{fb.f.data:#x}" if hasattr(fb, "f") else f"{ms / k:.4f}")
    print(rep, " ".join(row), flush=True)
