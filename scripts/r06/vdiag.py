"""pb_vline_kernel decomposition (libpbprobe6v.so from probes/r06_vdiag.hip; tool only).
python3 scripts/r06/vdiag.py [reps] [nbuf] [diag,diag,...]
configs[2] (2^25 frames) into nbuf buffers alive at once; per buffer, round after round: the product
build (pr6_build: pb_vline_kernel), its copy with compile-time cuts (DIAG 0 uncut, 1 no payload
bytes, 2 no chunk work, 4 no orbit sums, 5 = 1 + 4, 6 = 2 + 4) and the write-roofline fills over
the same bytes (4 KiB per workgroup; 208-KiB regions in 16-KiB steps, the kernel's geometry); VD_CAPS=4,5,...
adds the product build with its workgroups capped per CU by dynamic LDS.
One JSON line per (buffer, variant): medians over the rounds of 10-launch means."""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
NBUF = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ctx = GpuContext(0, lib_path=os.path.join(ROOT, "pb-af-xdp_amd", "lib", "libpbprobe6v.so"))
L = ctx.lib
D, U64 = C.c_double, C.c_uint64
L.pr6v_run.argtypes = [C.c_void_p, C.c_uint16, U64, U64, C.c_void_p, C.c_int, C.c_int, C.POINTER(D)]
L.pr6_build.argtypes = [C.c_void_p, C.c_uint16, U64, U64, C.c_void_p, C.c_int, C.POINTER(D)]
L.pr6_fill.argtypes = [C.c_void_p, C.c_void_p, U64, C.c_int, C.c_int, C.POINTER(D)]
L.pr6v_build_cap.argtypes = [C.c_void_p, C.c_uint16, U64, U64, C.c_void_p, C.c_uint32, C.c_int, C.POINTER(D)]
CAPS = [int(x) for x in os.environ.get("VD_CAPS", "").split(",") if x]  # product build, workgroups per CU


def ok(rc, what):
    if rc != 0:
        raise SystemExit(f"{what}: rc {rc}")


DIAGS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 2, 4, 5, 6]
ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
# the cuts that keep the bytes (0, 16, 32, 48) must build exactly the product's frames: 2^20 frames
m = 1 << 20
a = ctx.alloc_frames(*ctx.build_size(0, m))
b = ctx.alloc_frames(*ctx.build_size(0, m))
ctx.build(0, 12345, m, a)
ctx.sync()
want, want_off = a.packed().copy(), a.offsets().copy()
for dg in DIAGS:
    if dg & 7:
        continue
    ok(L.pr6v_run(ctx.h, 0, 12345, m, b.ptr, dg, 1, C.byref(D())), f"check {dg}")
    ctx.sync()
    same = bool((b.packed() == want).all()) and bool((b.offsets() == want_off).all())
    print(json.dumps({"check": dg, "frames": m, "bit_exact": same}), flush=True)
    if not same:
        raise SystemExit(f"diag {dg} differs from the product build")
a.free()
b.free()
n = 1 << 25
bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(NBUF)]
for fb in bufs:
    ctx.build(0, 0, n, fb)
ctx.sync()
total = bufs[0].total_bytes()
ms = D()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.6:  # clock ramp
    ok(L.pr6_build(ctx.h, 0, 0, n, bufs[0].ptr, 10, C.byref(ms)), "ramp")
res = {}
for r in range(REPS):
    for b, fb in enumerate(bufs):
        ok(L.pr6_build(ctx.h, 0, 0, n, fb.ptr, 10, C.byref(ms)), "build")
        res.setdefault((b, "product"), []).append(ms.value)
        for cap in CAPS:
            ok(L.pr6v_build_cap(ctx.h, 0, 0, n, fb.ptr, cap, 10, C.byref(ms)), f"cap {cap}")
            res.setdefault((b, f"product cap {cap}/CU"), []).append(ms.value)
        for dg in DIAGS:
            ok(L.pr6v_run(ctx.h, 0, 0, n, fb.ptr, dg, 10, C.byref(ms)), f"diag {dg}")
            res.setdefault((b, f"diag{dg}"), []).append(ms.value)
        for name, mode in (("fill 4KiB/wg", 2), ("fill 4KiB/wg 4/CU", 5), ("fill 208KiB regions", 12)):
            ok(L.pr6_fill(ctx.h, C.c_void_p(fb.f.data), total, mode, 10, C.byref(ms)), name)
            res.setdefault((b, name), []).append(ms.value)
for (b, k), v in res.items():
    print(json.dumps({"buf": b, "variant": k, "ms_med": round(statistics.median(v), 4), "ms_min": round(min(v), 4),
                      "all": [round(x, 4) for x in v]}), flush=True)
