"""Round-6 gate probe driver (pb-af-xdp_amd/lib/libpbprobe6.so from probes/r06_probe.hip; tool only).

python3 scripts/r06/probe.py gate [reps] [nbuf]
  configs[2] (2^25 frames) into nbuf buffers alive at once (each keeps its physical placement):
  per buffer the product build, the record pre-pass checked against it, then timed side by side
  the product kernel, the pre-pass, the page-kernel skeleton (pt + record loads, 4 KiB of
  record-dependent stores per wave) and the bare page stores at several occupancy caps, and the
  4-KiB-per-workgroup fills over the same bytes.
One JSON line per measurement."""
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

LIB = os.path.join(ROOT, "pb-af-xdp_amd", "lib", "libpbprobe6.so")
what = sys.argv[1]
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
NBUF = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ctx = GpuContext(0, lib_path=LIB)
L = ctx.lib
D = C.c_double
U64 = C.c_uint64
L.pr6_alloc.argtypes = [C.c_void_p, U64, U64]
L.pr6_prep.argtypes = [C.c_void_p, C.c_uint16, U64, U64, C.c_void_p, C.c_int, C.POINTER(D)]
L.pr6_check_out.argtypes = [C.c_void_p, C.c_uint16, C.c_void_p, U64, C.POINTER(C.c_ulonglong)]
L.pr6_gate_run.argtypes = [C.c_void_p, C.c_void_p, U64, U64, C.c_int, C.c_uint32, C.c_int, C.POINTER(D)]
L.pr6_build.argtypes = [C.c_void_p, C.c_uint16, U64, U64, C.c_void_p, C.c_int, C.POINTER(D)]
L.pr6_fill.argtypes = [C.c_void_p, C.c_void_p, U64, C.c_int, C.c_int, C.POINTER(D)]


def ok(rc, what):
    if rc != 0:
        raise SystemExit(f"{what}: rc {rc}")


def emit(d):
    print(json.dumps(d), flush=True)


CAPS = {8: 0, 6: 27136, 5: 32768, 4: 40960, 3: 54272}

if what in ("gate", "shapes"):
    n = 1 << 25
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    mf, mb = ctx.build_size(0, n)
    ok(L.pr6_alloc(ctx.h, n, mb), "alloc")
    bufs = [ctx.alloc_frames(mf, mb) for _ in range(NBUF)]
    ms = D()
    ms2 = (D * 2)()
    totals = []
    for i, fb in enumerate(bufs):
        ctx.build(0, 0, n, fb)
        ctx.sync()
        total = fb.total_bytes()
        totals.append(total)
        ok(L.pr6_prep(ctx.h, 0, 0, n, fb.ptr, 1, ms2), "prep")
        bad = (C.c_ulonglong * 4)()
        ok(L.pr6_check_out(ctx.h, 0, fb.ptr, total, bad), "check")
        emit({"buf": i, "total": total, "bad_offsets": bad[0], "bad_lengths": bad[1], "bad_csums": bad[2],
              "bad_pages": bad[3]})
    total = totals[0]
    # the gate variants read the last pre-pass's records (every buffer built the same frames)
    V = [("gate strided", 0)] + [(f"gate strided cap{c}", 0, CAPS[c]) for c in (6, 5, 4, 3)] + \
        [("gate contiguous", 1), ("gate contiguous cap4", 1, CAPS[4]), ("stores strided", 2),
         ("stores strided cap4", 2, CAPS[4]), ("stores contiguous", 3)]
    if what == "shapes":
        V = [("stores strided", 2), ("stores contiguous", 3), ("stores strided wg64", 4), ("stores contig wg64", 5),
             ("stores strided wg128", 6), ("stores contig wg128", 7), ("stores strided wg512", 8),
             ("stores contig wg512", 9), ("gate strided", 0), ("gate strided wg64", 10), ("gate strided wg128", 11),
             ("gate strided wg512", 12)]
    fills = {"fill 4KiB/wg": 2, "fill 4KiB/wg XCD-contig": 10, "fill 4KiB/wg cap4": 5, "fill 208KiB region": 12}
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.6:  # clock ramp
        ok(L.pr6_fill(ctx.h, C.c_void_p(bufs[0].f.data), total, 2, 10, C.byref(ms)), "ramp")
    res = {}

    def add(k, v):
        res.setdefault(k, []).append(v)

    for r in range(REPS):
        for i, fb in enumerate(bufs):
            dp = C.c_void_p(fb.f.data)
            ok(L.pr6_build(ctx.h, 0, 0, n, fb.ptr, 10, C.byref(ms)), "build")
            add((i, "product vline"), ms.value)
            ok(L.pr6_prep(ctx.h, 0, 0, n, fb.ptr, 10, ms2), "prep")
            add((i, "prep lengths+scan"), ms2[0])
            add((i, "prep records"), ms2[1])
            for v in V:
                pad = v[2] if len(v) > 2 else 0
                ok(L.pr6_gate_run(ctx.h, dp, total, n, v[1], pad, 10, C.byref(ms)), v[0])
                add((i, v[0]), ms.value)
            for k, m in fills.items():
                ok(L.pr6_fill(ctx.h, dp, total, m, 10, C.byref(ms)), k)
                add((i, k), ms.value)
    for (i, k), vals in res.items():
        med = statistics.median(vals)
        emit({"buf": i, "variant": k, "ms_med": round(med, 5), "ms_min": round(min(vals), 5),
              "tbps_med": round(total / med / 1e9, 3), "all": [round(x, 4) for x in vals]})
else:
    raise SystemExit(f"unknown mode {what}")
