"""Where the D2H-inclusive rate of configs[1] is bound (tool only; DESIGN.md 6, verdict r05 item 5).
python3 scripts/r06/d2h_probe.py [reps]
For 64-B and 1500-B frames, 2^18 per batch (bench.py's d2h_rate size), landing only (the frames are
built once), into pinned registered host memory:
  scatter-4K  the library's landing: pb_scatter_fixed stores each frame into its 4-KiB UMEM slot
              over the host link (af_xdp.c:200-214 geometry)
  dma-4K      the same slots by one hipMemcpy2DAsync (PBGPU_UMEM_DMA=1)
  scatter-dense / dma-dense   the same bytes into back-to-back slots (slot = frame length)
  scatter-<S>  power-of-two slots of S bytes between the two (a UMEM with several frames per 4 KiB)
  dma1d-dense  the dense case as one contiguous copy (pbgpu_copy_packed: hipMemcpyAsync)
and the build alone.  One JSON line per measurement: ms per batch, Mpps, frame GB/s."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = 1 << 18


def run(mode):
    if mode == "dma":
        os.environ["PBGPU_UMEM_DMA"] = "1"
    else:
        os.environ.pop("PBGPU_UMEM_DMA", None)
    ctx = GpuContext(0)
    out = []
    for i, name in enumerate(("c2_udp_64", "c2_udp_1500")):
        ctx.load_sequence(i, Sequence.from_config(pc.get(name)), pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(i, N))
        ctx.build(i, 0, N, fb)
        ctx.sync()
        flen = fb.total_bytes() // N
        t0 = time.perf_counter()
        for r in range(REPS):
            ctx.build(i, r * N, N, fb)
        ctx.sync()
        out.append({"frame": flen, "what": "build only", "ms": (time.perf_counter() - t0) / REPS * 1e3})
        slots = [4096, flen] + ([128, 256] if flen == 64 else [2048] if flen == 1500 else [])
        for slot in slots:
            if mode == "dma" and slot not in (4096, flen):
                continue
            umem = np.zeros(N * slot + 4096, dtype=np.uint8)
            assert ctx.lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes) == 0
            fb.to_umem(umem, slot, 0, N)  # first landing: mappings, staging
            t0 = time.perf_counter()
            for r in range(REPS):
                fb.to_umem(umem, slot, 0, N)
            dt = (time.perf_counter() - t0) / REPS
            ok = bytes(umem[:flen]) == fb.frames()[0] if slot == 4096 else True
            ctx.lib.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
            what = {4096: "4K", flen: "dense"}.get(slot, str(slot))
            out.append({"frame": flen, "what": f"{mode}-{what}", "ms": dt * 1e3, "first_frame_ok": ok})
            if slot == flen and mode == "scatter":
                t0 = time.perf_counter()
                for r in range(REPS):
                    assert ctx.lib.pbgpu_copy_packed(ctx.h, fb.ptr, umem.ctypes.data, 0, N * flen) == 0
                dt = (time.perf_counter() - t0) / REPS
                out.append({"frame": flen, "what": "dma1d-dense", "ms": dt * 1e3,
                            "first_frame_ok": bytes(umem[:flen]) == fb.frames()[0]})
        fb.free()
    ctx.close()
    for o in out:
        o["mpps"] = round(N / (o["ms"] / 1e3) / 1e6, 1)
        o["frame_gbps"] = round(N * o["frame"] / (o["ms"] / 1e3) / 1e9, 2)
        o["ms"] = round(o["ms"], 4)
        print(json.dumps(o), flush=True)


run("scatter")
run("dma")
