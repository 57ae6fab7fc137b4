"""pb_fstage_kernel decomposition (libpbprobe6v.so from probes/r06_vdiag.hip; tool only).
python3 scripts/r06/fdiag.py [reps] [nbuf] [diag,diag,...]
configs[1]'s 1500-B frames (2^25) into nbuf buffers alive at once; per buffer, round after round:
the product build, its copy with compile-time cuts (0 uncut, 1 no payload bytes, 2 no payload pass,
8 no checksum accumulation, 9 = 1 + 8, 16 the L4 sums from the orbit prefix sums in a second wave, 32 the chunk loop unrolled by two) and the write-roofline fills over the same bytes.
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
DIAGS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 2, 8, 9]
ctx = GpuContext(0, lib_path=os.path.join(ROOT, "pb-af-xdp_amd", "lib", "libpbprobe6v.so"))
L = ctx.lib
D, U64 = C.c_double, C.c_uint64
L.pr6v_fst.argtypes = [C.c_void_p, C.c_uint16, U64, U64, C.c_void_p, C.c_int, C.c_int, C.POINTER(D)]
L.pr6_build.argtypes = [C.c_void_p, C.c_uint16, U64, U64, C.c_void_p, C.c_int, C.POINTER(D)]
L.pr6_fill.argtypes = [C.c_void_p, C.c_void_p, U64, C.c_int, C.c_int, C.POINTER(D)]


def ok(rc, what):
    if rc != 0:
        raise SystemExit(f"{what}: rc {rc}")


ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
# a packed-frame sequence in another slot: the library builds the orbit table (pb_orbit_sum's
# prefix sums) for it, which DIAG 16 reads (the probe refuses DIAG 16 without it)
ctx.load_sequence(1, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
m = 1 << 18
a = ctx.alloc_frames(*ctx.build_size(0, m))
b = ctx.alloc_frames(*ctx.build_size(0, m))
ctx.build(0, 777, m, a)
ctx.sync()
want = a.packed().copy()
for dg in DIAGS:
    if dg not in (0, 16, 32):  # the cuts that keep the bytes
        continue
    ok(L.pr6v_fst(ctx.h, 0, 777, m, b.ptr, dg, 1, C.byref(D())), f"check {dg}")
    ctx.sync()
    same = bool((b.packed() == want).all())
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
    ok(L.pr6_build(ctx.h, 0, 0, n, bufs[0].ptr, 4, C.byref(ms)), "ramp")
res = {}
for r in range(REPS):
    for bi, fb in enumerate(bufs):
        ok(L.pr6_build(ctx.h, 0, 0, n, fb.ptr, 10, C.byref(ms)), "build")
        res.setdefault((bi, "product"), []).append(ms.value)
        for dg in DIAGS:
            ok(L.pr6v_fst(ctx.h, 0, 0, n, fb.ptr, dg, 10, C.byref(ms)), f"diag {dg}")
            res.setdefault((bi, f"diag{dg}"), []).append(ms.value)
        for name, mode in (("fill 4KiB/wg", 2), ("fill 4KiB/wg 4/CU", 5), ("fill 16KiB/wg XCD-contig", 9)):
            ok(L.pr6_fill(ctx.h, C.c_void_p(fb.f.data), total, mode, 10, C.byref(ms)), name)
            res.setdefault((bi, name), []).append(ms.value)
for (bi, k), v in res.items():
    print(json.dumps({"buf": bi, "variant": k, "ms_med": round(statistics.median(v), 4), "ms_min": round(min(v), 4),
                      "all": [round(x, 4) for x in v]}), flush=True)
