"""Host-side timing of bench.run_configs' phases between the warm-up and the timed steps (tool
only): where does the multi-millisecond idle gap before configs[4]'s first timed launch come
from?  python3 scripts/r05/gap_probe.py [config ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
import pb_dist  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

MIX = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"]


def run(cfg):
    ctx = GpuContext(0)
    names = MIX if cfg == "c5_mix" else [cfg]
    n = 1 << 24 if cfg == "c5_mix" else 1 << 25
    bufs = []
    for i, nm in enumerate(names):
        ctx.load_sequence(i, Sequence.from_config(pc.get(nm)), pc.SEED_BASE)
        bufs.append(ctx.alloc_frames(*ctx.build_size(i, n)))
    ctx.set_timing(ctx.TIMING_SPAN)

    def step(s):
        first = pb_dist.step_first_iter(s, 0, 1, n)
        if len(names) > 1:
            ctx.build_batch([(i, first, n, bufs[i]) for i in range(len(names))])
        else:
            ctx.build(0, first, n, bufs[0])

    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        for s in range(8):
            step(s)
        ctx.sync()
    for rep in range(3):
        T = [("start", time.perf_counter())]
        for s in range(10):
            step(s)
        T.append(("warm-up launched", time.perf_counter()))
        ctx.sync()
        T.append(("sync", time.perf_counter()))
        ctx.kernel_time()
        T.append(("kernel_time", time.perf_counter()))
        ctx.counters(len(names))
        T.append(("counters", time.perf_counter()))
        step(10)
        T.append(("first timed launch call", time.perf_counter()))
        for s in range(11, 60):
            step(s)
        T.append(("49 more launched", time.perf_counter()))
        ctx.sync()
        T.append(("sync", time.perf_counter()))
        ms, k = ctx.kernel_time()
        print(cfg, "rep", rep, " ".join(f"{a}={1e3 * (b - T[i][1]):.3f}ms" for i, (a, b) in enumerate(T[1:])),
              f"span/launch={ms / k:.4f}", flush=True)
    for b in bufs:
        b.free()


for c in sys.argv[1:] or ["c5_mix", "c2_udp_64"]:
    run(c)
