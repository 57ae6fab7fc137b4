"""Round-5 A/B probe driver (lib/libpbprobe.so from probes/r05_probe.hip; tool only).

python3 scripts/r05/probe.py MODE [reps]
(the pb_fpage_kernel modes "fpage" / "fpord" are in commit 37dc421 with the kernel)
  xs / xs8 / xs9 / xsapi   64-B page-kernel shapes, the decomposition (full / stores only /
         arithmetic only / the 4-KiB fill), occupancy caps, count records; wave-local shapes
         checked byte for byte against the product launch
  xp / xpw   60-B / 98-B page kernels: SGPR budget, page-store shapes (wave-owned pages,
         wave-local builds)
  mix    configs[4]'s fused-launch variants on three buffers (MIX_V selects)
  ximg   the static-payload ICMP image kernel's block sizes / caps beside pb_xpage_kernel
  fxp    a page-owned 1500-B writer on pb_fstage_kernel's frame machinery, with decomposition
  place / detect / wfill / capx   the region kernels and write-only fill shapes on several large
         buffers alive at once (each keeps its physical placement); sub-range placement probes;
         occupancy caps
  vmm    frame buffers from physical chunks (hipMemCreate) mapped in order or shuffled vs
         hipMalloc, re-allocated ALLOCS times
  offswap  configs[2] with each buffer's frame bytes and every buffer's offset arrays; with VGEOM=1
         instead the packed kernel's store geometry as plain fills (pr_fill_vgeom modes), and with
         VTOTALS=b,b,... equal-region fills beside the page fill over the first b bytes
  remap  allocation-time detection (whole-buffer region / page fill ratio) and replacement of
         buffers that draw the slow placement
One JSON line per measurement."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

LIB = os.path.join(ROOT, "pb-af-xdp_amd", "lib", "libpbprobe.so")
what = sys.argv[1]
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ctx = GpuContext(0, lib_path=LIB)
L = ctx.lib
D = C.c_double
L.pr_xs.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int, C.c_uint32, C.c_uint32,
                    C.c_int, C.POINTER(D)]
L.pr_mix.argtypes = [C.c_void_p, C.POINTER(C.c_uint16), C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p), C.c_int,
                     C.c_int, C.POINTER(D)]
L.pr_build.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int, C.POINTER(D)]
L.pr_fill_vgeom_run.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.POINTER(D)]
L.pr_fill_prod.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.POINTER(D)]
L.pr_build_swap.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int,
                            C.POINTER(D)]
L.pr_fill.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_int, C.POINTER(D)]
L.pr_fill_name.restype = C.c_char_p
L.pr_compare.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
L.pr_fill_wave_at.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_uint32, C.c_int,
                             C.POINTER(D)]
L.pr_build_cap.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint32, C.c_int,
                          C.POINTER(D), C.POINTER(C.c_uint32)]
L.pr_xp.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int, C.c_int, C.POINTER(D)]
L.pr_fxp.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int, C.c_uint32, C.c_int,
                     C.POINTER(D)]
L.pr_frames_vmm.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p),
                           C.POINTER(C.c_uint64), C.c_uint32]
L.pr_frames_vmm_free.argtypes = [C.c_void_p, C.c_void_p]
L.pr_frames_vmm_free.restype = None
L.pr_ximg.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int, C.c_uint32, C.c_int,
                      C.POINTER(D)]
L.pr_xpw.argtypes = [C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int, C.c_uint32, C.c_int,
                     C.POINTER(D)]


def ok(rc, what):
    if rc != 0:
        raise SystemExit(f"{what}: rc {rc}")


def emit(d):
    print(json.dumps(d), flush=True)


def data_ptr(fb):
    return fb.f.data


def ramp(fn, secs=0.6):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        fn()


if what == "xs":
    n = 1 << 25
    ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(0, n))
    ref = ctx.alloc_frames(*ctx.build_size(0, n))
    ms = D()
    # variant: (name, id, lds_pad, pgrid)
    V = [("product", 0, 0, 0), ("product cap5", 0, 15000, 0), ("body full", 1, 0, 0), ("body stores only", 2, 0, 0),
         ("body arith only", 3, 0, 0), ("wave256", 4, 0, 0), ("wave64", 5, 0, 0), ("wave512", 6, 0, 0),
         ("persist256 g1024", 7, 0, 1024), ("persist256 g1536", 7, 0, 1536), ("persist64 g4096", 8, 0, 4096),
         ("persist64 g7168", 8, 0, 7168), ("wave256 stores only", 9, 0, 0), ("wave256 arith only", 10, 0, 0),
         ("wave256 s80", 11, 0, 0), ("wave64 s80", 12, 0, 0), ("wave256 cap5", 4, 15000, 0),
         ("wave256 cap4", 4, 23000, 0)]
    # parity of the real-frame shapes against the product launch
    ok(L.pr_xs(ctx.h, 0, 5, n, ref.ptr, 0, 0, 0, 1, C.byref(ms)), "ref")
    for name, v, pad, pg in V:
        if "only" in name:
            continue
        ok(L.pr_xs(ctx.h, 0, 5, n, fb.ptr, v, pad, pg, 1, C.byref(ms)), name)
        bad = C.c_uint64()
        ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(fb)), C.c_void_p(data_ptr(ref)), n * 64, C.byref(bad)), "cmp")
        emit({"check": name, "bad_dwords": bad.value})
    ramp(lambda: L.pr_xs(ctx.h, 0, 0, n, fb.ptr, 0, 0, 0, 8, C.byref(ms)))
    res = {name: [] for name, *_ in V}
    fills = {"fill 4KiB/wg": 0, "fill 16KiB/wg": 12}
    for k in fills:
        res[k] = []
    for r in range(REPS):
        for name, v, pad, pg in V:
            ok(L.pr_xs(ctx.h, 0, 0, n, fb.ptr, v, pad, pg, 20, C.byref(ms)), name)
            res[name].append(ms.value)
        for k, s in fills.items():
            ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), n * 64, s, 2048, 20, C.byref(ms)), k)
            res[k].append(ms.value)
    for k, v in res.items():
        s = sorted(v)
        emit({"variant": k, "ms_med": round(s[len(s) // 2], 5), "ms_min": round(s[0], 5),
              "tbps_med": round(n * 64 / (s[len(s) // 2] * 1e-3) / 1e12, 3), "all": [round(x, 4) for x in v]})
    fb.free()
    ref.free()

elif what == "xs8":
    # the 64-B shapes on NBUF 2-GiB buffers (each its own placement)
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "6"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
    ms = D()
    V = [("product", 0, 0), ("product cap5", 0, 15000), ("wave256", 4, 0), ("wave256 cap4", 4, 23000),
         ("wave256 cap3", 4, 25000), ("wave512", 6, 0), ("wave512 cap2", 6, 22000), ("wave1024", 13, 0)]
    ok(L.pr_xs(ctx.h, 0, 5, n, bufs[1].ptr, 0, 0, 0, 1, C.byref(ms)), "ref")
    ok(L.pr_xs(ctx.h, 0, 5, n, bufs[0].ptr, 13, 0, 0, 1, C.byref(ms)), "w1024")
    bad = C.c_uint64()
    ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[0])), C.c_void_p(data_ptr(bufs[1])), n * 64, C.byref(bad)), "cmp")
    emit({"check": "wave1024", "bad_dwords": bad.value})
    ramp(lambda: L.pr_xs(ctx.h, 0, 0, n, bufs[0].ptr, 0, 0, 0, 8, C.byref(ms)))
    for r in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"rep": r, "buf": i, "addr": hex(data_ptr(fb))}
            for name, v, pad in V:
                ok(L.pr_xs(ctx.h, 0, 0, n, fb.ptr, v, pad, 0, 20, C.byref(ms)), name)
                row[name] = round(ms.value, 5)
            ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), n * 64, 0, 2048, 20, C.byref(ms)), "fill")
            row["fill 4KiB/wg"] = round(ms.value, 5)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "xs9":
    # occupancy of the wave-local 64-B shape (dynamic LDS caps its workgroups per CU)
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
    ms = D()
    # (name, variant, pad): wave256 static LDS 16 KiB; wave128 8 KiB; wave512 32 KiB
    V = [("product as loaded", 15, 0), ("wave256 cap3", 4, 25000), ("wave256 cap2", 4, 40000), ("wave256 cap1", 4, 70000),
         ("wave128 cap6", 14, 20000), ("wave128 cap5", 14, 25000), ("wave128 cap4", 14, 33000),
         ("wave128 cap3", 14, 37000), ("wave512 cap1", 6, 50000), ("wave256 cap4", 4, 23000)]
    ok(L.pr_xs(ctx.h, 0, 5, n, bufs[1].ptr, 0, 0, 0, 1, C.byref(ms)), "ref")
    ok(L.pr_xs(ctx.h, 0, 5, n, bufs[0].ptr, 14, 0, 0, 1, C.byref(ms)), "w128")
    bad = C.c_uint64()
    ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[0])), C.c_void_p(data_ptr(bufs[1])), n * 64, C.byref(bad)), "cmp")
    emit({"check": "wave128", "bad_dwords": bad.value})
    ramp(lambda: L.pr_xs(ctx.h, 0, 0, n, bufs[0].ptr, 0, 0, 0, 8, C.byref(ms)))
    for r in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"rep": r, "buf": i}
            for name, v, pad in V:
                ok(L.pr_xs(ctx.h, 0, 0, n, fb.ptr, v, pad, 0, 20, C.byref(ms)), name)
                row[name] = round(ms.value, 5)
            for pad, nm in ((0, "fill 4KiB 8/CU"), (45000, "fill 4KiB 3/CU"), (36000, "fill 4KiB 4/CU")):
                ok(L.pr_fill_wave_at(ctx.h, C.c_void_p(data_ptr(fb)), n * 64, 0, 4096, pad, 20, C.byref(ms)), nm)
                row["wavefill " + nm] = round(ms.value, 5)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "wfill":
    # wave-local fill shapes (candidate store shapes for the region kernels) on NBUF large
    # buffers beside the packed and 1500-B kernels' own rates
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    ctx.load_sequence(1, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
    f0, b0 = ctx.build_size(0, n)
    f1, b1 = ctx.build_size(1, n)
    bufs = [ctx.alloc_frames(max(f0, f1), max(b0, b1)) for _ in range(nbuf)]
    fill_bytes = 27_600_000_000 // 4096 * 4096
    ms = D()
    S = [("natural 4KiB 8/CU", 0, 4096, 0), ("natural 4KiB 3/CU", 0, 4096, 45000), ("xpages 4KiB 8/CU", 1, 4096, 0),
         ("xpages 4KiB 3/CU", 1, 4096, 45000), ("natural 16.5KB 8/CU", 0, 16496, 0),
         ("natural 16.5KB 4/CU", 0, 16496, 36000), ("natural 16.5KB 3/CU", 0, 16496, 45000),
         ("xcdreg 16.5KB 8/CU", 2, 16496, 0), ("xcdreg 16.5KB 3/CU", 2, 16496, 45000),
         ("natural 6KB 3/CU", 0, 6000, 45000), ("natural 8KiB 3/CU", 0, 8192, 45000),
         ("natural 24KB 3/CU", 0, 24000, 45000), ("xcdreg 4KiB 3/CU", 2, 4096, 45000)]
    ramp(lambda: L.pr_build(ctx.h, 1, 0, n, bufs[0].ptr, 4, C.byref(ms)))
    for rnd in range(2):
        for i, fb in enumerate(bufs):
            row = {"round": rnd, "buf": i}
            ok(L.pr_build(ctx.h, 0, 0, n, fb.ptr, 6, C.byref(ms)), "c3")
            row["c3_ms"] = round(ms.value, 4)
            ok(L.pr_build(ctx.h, 1, 0, n, fb.ptr, 6, C.byref(ms)), "1500")
            row["c2_1500_ms"] = round(ms.value, 4)
            ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), fill_bytes, 1, 2048, 4, C.byref(ms)), "reg208")
            row["reg208"] = round(fill_bytes / (ms.value * 1e-3) / 1e12, 3)
            for nm, mode, ub, pad in S:
                ok(L.pr_fill_wave_at(ctx.h, C.c_void_p(data_ptr(fb)), fill_bytes, mode, ub, pad, 4, C.byref(ms)), nm)
                row[nm] = round(fill_bytes / (ms.value * 1e-3) / 1e12, 3)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "capx":
    # occupancy caps of the region kernels (packed configs[2], 1500-B) on NBUF large buffers, and the
    # 64-B page kernel as loaded beside its probe twin
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    ctx.load_sequence(1, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
    ctx.load_sequence(2, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
    f0, b0 = ctx.build_size(0, n)
    f1, b1 = ctx.build_size(1, n)
    bufs = [ctx.alloc_frames(max(f0, f1), max(b0, b1)) for _ in range(nbuf)]
    ms = D()
    base = C.c_uint32()
    ramp(lambda: L.pr_build(ctx.h, 1, 0, n, bufs[0].ptr, 4, C.byref(ms)))
    for rnd in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"round": rnd, "buf": i}
            for seq, nm, caps in ((0, "c3", (0, 3, 2)), (1, "1500", (0, 4, 3, 2))):
                for cap in caps:
                    ok(L.pr_build_cap(ctx.h, seq, 0, n, fb.ptr, cap, 6, C.byref(ms), C.byref(base)), nm)
                    row[f"{nm} cap{cap}"] = round(ms.value, 4)
                row[f"{nm} base_lds"] = base.value
            for name, v, pad in (("64B as loaded", 15, 0), ("64B wave256 cap3", 4, 25000),
                                 ("64B wave256 cap3 ring", 16, 25000), ("64B wave256 cap3 atomic", 17, 25000)):
                ok(L.pr_xs(ctx.h, 2, 0, n, fb.ptr, v, pad, 0, 20, C.byref(ms)), name)
                row[name] = round(ms.value, 5)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "xsapi":
    # the 64-B product through the C API (span timing, count ring), as bench.py runs it, beside the
    # probe's twins on the same buffer
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "3"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
    ctx.set_timing(ctx.TIMING_SPAN)
    ms = D()
    ramp(lambda: L.pr_xs(ctx.h, 0, 0, n, bufs[0].ptr, 0, 0, 0, 8, C.byref(ms)))
    for r in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"rep": r, "buf": i}
            for s_ in range(2):
                ctx.build(0, s_ * n, n, fb)
            ctx.sync()
            ctx.kernel_time()
            for s_ in range(20):
                ctx.build(0, s_ * n, n, fb)
            ctx.sync()
            t, k = ctx.kernel_time()
            row["api span"] = round(t / k, 5)
            for name, v, pad in (("as loaded", 15, 0), ("wave256 cap3", 4, 25000), ("wave256 cap3 ring", 16, 25000),
                                 ("wave256 cap3 atomic", 17, 25000)):
                ok(L.pr_xs(ctx.h, 0, 0, n, fb.ptr, v, pad, 0, 20, C.byref(ms)), name)
                row[name] = round(ms.value, 5)
            emit(row)
    p, b = ctx.counters(1)
    emit({"counters_frames": int(p[0]), "counters_bytes": int(b[0])})
    for fb in bufs:
        fb.free()

elif what == "xp":
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c4_tcp_syn")), pc.SEED_BASE)
    ctx.load_sequence(1, Sequence.from_config(pc.get("c5_icmp_echo")), pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(1, n)) for _ in range(nbuf)]
    ms = D()
    for seq in (0, 1):
        ok(L.pr_xp(ctx.h, seq, 5, n, bufs[1].ptr, 0, 1, C.byref(ms)), "ref")
        ok(L.pr_xp(ctx.h, seq, 5, n, bufs[0].ptr, 1, 1, C.byref(ms)), "s80")
        bad = C.c_uint64()
        nb = n * (60 if seq == 0 else 98)
        ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[0])), C.c_void_p(data_ptr(bufs[1])), nb, C.byref(bad)), "cmp")
        emit({"check": f"seq{seq} s80", "bad_dwords": bad.value})
    ramp(lambda: L.pr_xp(ctx.h, 0, 0, n, bufs[0].ptr, 0, 8, C.byref(ms)))
    for r in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"rep": r, "buf": i}
            for seq, nm in ((0, "tcp60"), (1, "icmp98")):
                for v, vn in ((0, "product"), (1, "s80"), (2, "s80 cap2"), (3, "s80 cap1")):
                    ok(L.pr_xp(ctx.h, seq, 0, n, fb.ptr, v, 20, C.byref(ms)), nm)
                    row[f"{nm} {vn}"] = round(ms.value, 5)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "xpw":
    # page-store shapes of the 60-B / 98-B page kernels (pr_xpw), each checked byte for byte
    # against the product launch, then timed on NBUF buffers; XPW_V: "variant:lds_pad,..."
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c4_tcp_syn")), pc.SEED_BASE)
    ctx.load_sequence(1, Sequence.from_config(pc.get("c5_icmp_echo")), pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(1, n)) for _ in range(nbuf)]
    ms = D()
    names = {0: "product", 1: "wg-build wave-store", 2: "wave kp1 w256", 3: "wave kp2 w256", 4: "wave kp4 w256",
             5: "wave kp4 w64", 6: "wave kp8 w64", 7: "wave kp2 w512", 8: "wave kp1 w512"}
    spec = os.environ.get("XPW_V", "0:0,1:0,2:0,3:0,4:0,5:0,6:0,7:0,8:0,2:25000,3:40000,4:40000")
    V = [(int(a), int(b)) for a, b in (x.split(":") for x in spec.split(","))]
    for seq in (0, 1):
        nb = n * (60 if seq == 0 else 98)
        ok(L.pr_xpw(ctx.h, seq, 5, n, bufs[1].ptr, 0, 0, 1, C.byref(ms)), "ref")
        for v in sorted({v for v, _ in V if v}):  # same sequence, same first iteration: byte-identical
            ok(L.pr_xpw(ctx.h, seq, 5, n, bufs[0].ptr, v, 0, 1, C.byref(ms)), names[v])
            bad = C.c_uint64()
            ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[0])), C.c_void_p(data_ptr(bufs[1])), nb, C.byref(bad)),
               "cmp")
            emit({"check": f"seq{seq} {names[v]}", "bad_dwords": bad.value})
    ramp(lambda: L.pr_xpw(ctx.h, 0, 0, n, bufs[0].ptr, 0, 0, 8, C.byref(ms)))
    for r in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"rep": r, "buf": i}
            for seq, nm in ((0, "tcp60"), (1, "icmp98")):
                for v, pad in V:
                    ok(L.pr_xpw(ctx.h, seq, 0, n, fb.ptr, v, pad, 20, C.byref(ms)), nm)
                    row[f"{nm} {names[v]}" + (f" lds{pad}" if pad else "")] = round(ms.value, 5)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "fxp":
    # page-owned 1500-B writer (pr_fxp) vs pb_fstage_kernel on NBUF 50-GB buffers alive at once;
    # each variant checked byte for byte against the product launch first.  FXP_V "variant:lds,..."
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
    ms = D()
    names = {0: "fstage", 1: "fxp np4", 2: "fxp np4 nt", 3: "fxp np8", 4: "fxp np2", 5: "fxp A only",
             6: "fxp A+B no stores", 7: "fxp B+S trivial A"}
    spec = os.environ.get("FXP_V", "0:0,1:0,2:0,3:0,4:0,1:32000,1:40000")
    V = [(int(a), int(b)) for a, b in (x.split(":") for x in spec.split(","))]
    cn = int(os.environ.get("FXP_CHECK_N", str(1 << 22)))
    for v in sorted({v for v, _ in V if 0 < v < 5}):
        ok(L.pr_fxp(ctx.h, 0, 5, cn, bufs[1].ptr, 0, 0, 1, C.byref(ms)), "ref")
        ok(L.pr_fxp(ctx.h, 0, 5, cn, bufs[0].ptr, v, 0, 1, C.byref(ms)), names[v])
        bad = C.c_uint64()
        ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[0])), C.c_void_p(data_ptr(bufs[1])), cn * 1500, C.byref(bad)),
           "cmp")
        emit({"check": names[v], "frames": cn, "bad_dwords": bad.value})
        # an odd-sized build: the stream's last page is partial
        ok(L.pr_fxp(ctx.h, 0, 7, 12345, bufs[1].ptr, 0, 0, 1, C.byref(ms)), "ref")
        ok(L.pr_fxp(ctx.h, 0, 7, 12345, bufs[0].ptr, v, 0, 1, C.byref(ms)), names[v])
        ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[0])), C.c_void_p(data_ptr(bufs[1])), 12345 * 1500,
                        C.byref(bad)), "cmp")
        emit({"check": names[v], "frames": 12345, "bad_dwords": bad.value})
    ramp(lambda: L.pr_fxp(ctx.h, 0, 0, n, bufs[0].ptr, 0, 0, 2, C.byref(ms)))
    for r in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"rep": r, "buf": i}
            for v, pad in V:
                ok(L.pr_fxp(ctx.h, 0, 0, n, fb.ptr, v, pad, 5, C.byref(ms)), names[v])
                row[names[v] + (f" lds{pad}" if pad else "")] = round(ms.value, 4)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "vmm":
    # does the VA -> physical chunk order decide the region kernels' slow placement?  Frame
    # buffers from hipMalloc vs physical chunks (hipMemCreate) mapped in creation order or
    # shuffled; per allocation kind NBUF buffers, configs[2] and 1500-B builds plus two fills
    import pbgpu as pg
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "2"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    ctx.load_sequence(1, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
    f0, b0 = ctx.build_size(0, n)
    f1, b1 = ctx.build_size(1, n)
    nf, nb = max(f0, f1), max(b0, b1)
    MB = 1 << 20
    kinds = [("malloc", 0, 0, 0), ("vmm 2M in order", 2 * MB, 0, 0), ("vmm 2M shuffled", 2 * MB, 7, 0),
             ("vmm 64M in order", 64 * MB, 0, 0), ("vmm 64M shuffled", 64 * MB, 7, 0), ("vmm 1G shuffled", 1024 * MB, 7, 0),
             ("vmm 2M in order + offsets", 2 * MB, 0, 1)]
    if os.environ.get("VMM_K"):
        keep = {int(x) for x in os.environ["VMM_K"].split(",")}
        kinds = [k for i, k in enumerate(kinds) if i in keep]
    ms = D()
    ref = None
    for alloc in range(int(os.environ.get("ALLOCS", "2"))):
        for label, chunk, shuf, vflags in kinds:
            bufs = []
            t0 = time.perf_counter()
            for i in range(nbuf):
                if chunk == 0:
                    bufs.append(("m", ctx.alloc_frames(nf, nb)))
                else:
                    p = C.c_void_p()
                    g = C.c_uint64()
                    ok(L.pr_frames_vmm(ctx.h, nf, nb, chunk, shuf + 1000 * alloc + i if shuf else 0, C.byref(p),
                                       C.byref(g), vflags), label)
                    bufs.append(("v", p))
            t_alloc = time.perf_counter() - t0
            for i, (kind, b) in enumerate(bufs):
                ptr = b.ptr if kind == "m" else b
                fr = C.cast(ptr, C.POINTER(pg.Frames)).contents
                if alloc == 0 and i == 0 and chunk == 0:
                    ramp(lambda: L.pr_build(ctx.h, 1, 0, n, ptr, 4, C.byref(ms)))
                row = {"alloc": alloc, "kind": label, "buf": i, "alloc_s": round(t_alloc, 2), "addr": hex(fr.data or 0)}
                ok(L.pr_build(ctx.h, 0, 0, n, ptr, 5, C.byref(ms)), "c3")
                row["c3_ms"] = round(ms.value, 4)
                ok(L.pr_build(ctx.h, 1, 0, n, ptr, 5, C.byref(ms)), "1500")
                row["c2_1500_ms"] = round(ms.value, 4)
                for sh, nm in ((1, "reg208 TB/s"), (0, "4KiB/wg TB/s")):
                    ok(L.pr_fill(ctx.h, C.c_void_p(fr.data), n * 1500, sh, 2048, 5, C.byref(ms)), nm)
                    row[nm] = round(n * 1500 / (ms.value * 1e-3) / 1e12, 3)
                emit(row)
            # parity of a build into a chunk-mapped buffer against a hipMalloc'ed one
            if alloc == 0 and chunk and shuf:
                if ref is None:
                    ref = ctx.alloc_frames(nf, nb)
                ok(L.pr_build(ctx.h, 1, 3, 1 << 22, ref.ptr, 1, C.byref(ms)), "ref")
                ok(L.pr_build(ctx.h, 1, 3, 1 << 22, bufs[0][1], 1, C.byref(ms)), "vmm")
                bad = C.c_uint64()
                dv = C.cast(bufs[0][1], C.POINTER(pg.Frames)).contents.data
                ok(L.pr_compare(ctx.h, C.c_void_p(dv), C.c_void_p(ref.f.data), (1 << 22) * 1500, C.byref(bad)), "cmp")
                emit({"check": label, "bad_dwords": bad.value})
                ref.free()
                ref = None
            for kind, b in bufs:
                if kind == "m":
                    b.free()
                else:
                    L.pr_frames_vmm_free(ctx.h, b)

elif what == "ximg":
    # pb_ximg_kernel shapes (block size, occupancy cap by dynamic LDS, SGPR budget) on NBUF 98-B
    # ICMP buffers, beside pb_xpage_kernel (sequence slot 1, loaded with PBGPU_XP_IMG=0 semantics
    # through a second context); each shape checked against the product launch first
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "3"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c5_icmp_echo")), pc.SEED_BASE)
    os.environ["PBGPU_XP_IMG"] = "0"  # slot 1: the same sequence on pb_xpage_kernel
    ctx.load_sequence(1, Sequence.from_config(pc.get("c5_icmp_echo")), pc.SEED_BASE)
    del os.environ["PBGPU_XP_IMG"]
    bufs = [ctx.alloc_frames(*ctx.build_size(0, n)) for _ in range(nbuf)]
    ms = D()
    names = {0: "product", 1: "w256", 2: "w512", 3: "w128", 4: "w256 nos80", 5: "w512 nos80"}
    spec = os.environ.get("XIMG_V", "0:0,1:0,1:40000,1:30000,1:25000,2:0,2:60000,2:45000,3:0,3:20000,4:0,4:30000,5:0")
    V = [(int(a), int(b)) for a, b in (x.split(":") for x in spec.split(","))]
    ok(L.pr_ximg(ctx.h, 0, 5, n, bufs[1].ptr, 0, 0, 1, C.byref(ms)), "ref")
    for v in sorted({v for v, _ in V if v}):
        ok(L.pr_ximg(ctx.h, 0, 5, n, bufs[0].ptr, v, 0, 1, C.byref(ms)), names[v])
        bad = C.c_uint64()
        ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[0])), C.c_void_p(data_ptr(bufs[1])), n * 98, C.byref(bad)),
           "cmp")
        emit({"check": names[v], "bad_dwords": bad.value})
    ramp(lambda: L.pr_ximg(ctx.h, 0, 0, n, bufs[0].ptr, 0, 0, 8, C.byref(ms)))
    for r in range(REPS):
        for i, fb in enumerate(bufs):
            row = {"rep": r, "buf": i}
            for v, pad in V:
                ok(L.pr_ximg(ctx.h, 0, 0, n, fb.ptr, v, pad, 20, C.byref(ms)), names[v])
                row[names[v] + (f" lds{pad}" if pad else "")] = round(ms.value, 5)
            ok(L.pr_build(ctx.h, 1, 0, n, fb.ptr, 20, C.byref(ms)), "xpage")
            row["pb_xpage_kernel"] = round(ms.value, 5)
            emit(row)
    for fb in bufs:
        fb.free()

elif what == "remap":
    # can a buffer that draws the slow placement be replaced at allocation time?  NBUF configs[2]
    # buffers (library allocation, chunk-mapped by default); each one's whole-buffer region-fill /
    # page-fill ratio (the detection) and configs[2] time; a buffer under RATIO gets up to TRIES
    # replacement allocations (held while trying, so each lands on other pages), the first one
    # at or over RATIO kept
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    thr = float(os.environ.get("RATIO", "0.99"))
    tries = int(os.environ.get("TRIES", "3"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    f0, b0 = ctx.build_size(0, n)
    ms = D()

    def measure(fb):
        ok(L.pr_build(ctx.h, 0, 0, n, fb.ptr, 5, C.byref(ms)), "c3")
        c3 = ms.value
        tot = int(b0) // 16 * 16
        ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), tot, 1, 2048, 5, C.byref(ms)), "reg")
        reg = tot / (ms.value * 1e-3) / 1e12
        ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), tot, 0, 2048, 5, C.byref(ms)), "page")
        page = tot / (ms.value * 1e-3) / 1e12
        r = {"c3_ms": round(c3, 4), "reg_tbps": round(reg, 3), "page_tbps": round(page, 3),
             "ratio": round(reg / page, 4), "addr": hex(data_ptr(fb))}
        for sh in (int(x) for x in os.environ.get("XSHAPES", "").split(",") if x):
            # extra detection candidates: XCD-contiguous fills (2: 96 KiB per workgroup, 7: 24 KiB)
            ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), tot, sh, 2048, 5, C.byref(ms)), f"s{sh}")
            r[f"s{sh}_ratio"] = round(tot / (ms.value * 1e-3) / 1e12 / page, 4)
        return r

    bufs = [ctx.alloc_frames(f0, b0) for _ in range(nbuf)]
    ramp(lambda: L.pr_build(ctx.h, 0, 0, n, bufs[0].ptr, 2, C.byref(ms)))
    for i in range(nbuf):
        m = measure(bufs[i])
        emit({"buf": i, "try": 0, **m})
        held = []
        t = 0
        while m["ratio"] < thr and t < tries:
            t += 1
            nb = ctx.alloc_frames(f0, b0)
            m = measure(nb)
            emit({"buf": i, "try": t, **m})
            if m["ratio"] >= thr:
                bufs[i].free()
                bufs[i] = nb
            else:
                held.append(nb)
        for h in held:
            h.free()
    for i, fb in enumerate(bufs):
        emit({"buf": i, "final": True, **measure(fb)})
    for fb in bufs:
        fb.free()

elif what == "offswap":
    # does configs[2]'s slow placement follow the frame bytes or the 4-B offset arrays?  NBUF
    # buffers alive at once; the packed kernel timed for every (data buffer, offsets buffer) pair,
    # ROUNDS times
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "3"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    f0, b0 = ctx.build_size(0, n)
    ms = D()
    bufs = [ctx.alloc_frames(f0, b0) for _ in range(nbuf)]
    ramp(lambda: L.pr_build(ctx.h, 0, 0, n, bufs[0].ptr, 2, C.byref(ms)))
    if os.environ.get("VGEOM"):
        # the kernel's store geometry as plain fills (pr_fill_vgeom modes), per buffer, beside the build
        wf = 252
        nreg = (n + wf - 1) // wf
        for rnd in range(int(os.environ.get("ROUNDS", "2"))):
            for i, fb in enumerate(bufs):
                ok(L.pr_build(ctx.h, 0, 0, n, fb.ptr, 3, C.byref(ms)), "c3")
                row = {"round": rnd, "buf": i, "c3_ms": round(ms.value, 4)}
                tot = int(os.environ.get("VTOTAL", "27649414866"))  # configs[2]'s bytes at first 0, 2^25 frames
                for mode in range(5):
                    ok(L.pr_fill_vgeom_run(ctx.h, fb.ptr, nreg, tot, mode, 5, C.byref(ms)), "vgeom")
                    row[f"g{mode}_ms"] = round(ms.value, 4)
                for t2 in (int(x) for x in os.environ.get("VTOTALS", "").split(",") if x):
                    # equal 208-KiB regions over the first t2 bytes, and the page fill over them
                    nr2 = (t2 + 212991) // 212992
                    ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), t2 // 16 * 16, 0, 2048, 5, C.byref(ms)), "page")
                    e = {"page_ms": round(ms.value, 4)}
                    for mode in [int(x) for x in os.environ.get("VMODES", "2").split(",") if x]:
                        ok(L.pr_fill_vgeom_run(ctx.h, fb.ptr, nr2, t2, mode, 5, C.byref(ms)), "vgeom2")
                        e[f"m{mode}"] = round(ms.value / e["page_ms"], 3)
                    for kib in [int(x) for x in os.environ.get("VREG", "").split(",") if x]:
                        # equal regions of kib KiB (contiguous eighths)
                        ok(L.pr_fill_vgeom_run(ctx.h, fb.ptr, t2 // (kib << 10), t2, 2, 5, C.byref(ms)), "vreg")
                        e[f"r{kib}K"] = round(ms.value / e["page_ms"], 3)
                    for g in [int(x) for x in os.environ.get("VWIN", "").split(",") if x]:
                        # window-coherent walks (modes 10: 4-KiB units, 11: 16-KiB units) with a grid of g
                        for mode in (10, 11):
                            ok(L.pr_fill_vgeom_run(ctx.h, fb.ptr, g, t2, mode, 5, C.byref(ms)), "vwin")
                            e[f"w{mode}g{g}"] = round(ms.value / e["page_ms"], 3)
                    for m in [int(x) for x in os.environ.get("VPROD", "").split(",") if x]:
                        # the product's write-probe shapes (pbk_launch_fill modes)
                        ok(L.pr_fill_prod(ctx.h, C.c_void_p(data_ptr(fb)), t2 // 16 * 16, m, 5, C.byref(ms)), "prod")
                        e[f"p{m}"] = round(ms.value / e["page_ms"], 3)
                    for sh in [int(x) for x in os.environ.get("VPR", "").split(",") if x]:
                        # the probe's own fill shapes (pr_fill: 8, 9 XCD-owned pages as pb_xsmall_kernel)
                        ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), t2 // 16 * 16, sh, 2048, 5, C.byref(ms)), "pr")
                        e[f"s{sh}"] = round(ms.value / e["page_ms"], 3)
                    for kib in [int(x) for x in os.environ.get("VREG9", "").split(",") if x]:
                        # equal regions of kib KiB in blockIdx order (consecutive regions on different XCDs)
                        ok(L.pr_fill_vgeom_run(ctx.h, fb.ptr, t2 // (kib << 10), t2, 9, 5, C.byref(ms)), "vreg9")
                        e[f"b{kib}K"] = round(ms.value / e["page_ms"], 3)
                    row[f"t{t2 >> 30}G"] = e
                emit(row)
        for fb in bufs:
            fb.free()
        sys.exit(0)
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for i in range(nbuf):
            for j in range(nbuf):
                ok(L.pr_build_swap(ctx.h, 0, 0, n, bufs[i].ptr, bufs[j].ptr, 5, C.byref(ms)), "swap")
                emit({"round": rnd, "data": i, "offs": j, "ms": round(ms.value, 4)})
    for fb in bufs:
        fb.free()

elif what == "detect":
    # can a short probe at allocation time tell a slow placement?  Region vs page fills over
    # sub-ranges of each buffer, beside the packed and 1500-B kernels' own rates; ALLOCS
    # allocation rounds (all buffers freed in between)
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    ctx.load_sequence(1, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
    f0, b0 = ctx.build_size(0, n)
    f1, b1 = ctx.build_size(1, n)
    ms = D()
    for alloc in range(int(os.environ.get("ALLOCS", "3"))):
        bufs = [ctx.alloc_frames(max(f0, f1), max(b0, b1)) for _ in range(nbuf)]
        if alloc == 0:
            ramp(lambda: L.pr_build(ctx.h, 1, 0, n, bufs[0].ptr, 4, C.byref(ms)))
        for i, fb in enumerate(bufs):
            row = {"alloc": alloc, "buf": i, "addr": hex(data_ptr(fb))}
            ok(L.pr_build(ctx.h, 0, 0, n, fb.ptr, 6, C.byref(ms)), "c3")
            row["c3_ms"] = round(ms.value, 4)
            ok(L.pr_build(ctx.h, 1, 0, n, fb.ptr, 6, C.byref(ms)), "1500")
            row["c2_1500_ms"] = round(ms.value, 4)
            for gb in (1, 4, 16):
                nb = gb << 30
                r = {}
                for s_, nm in ((0, "page"), (1, "reg208"), (2, "reg96")):
                    ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), nb, s_, 2048, 10 if gb < 16 else 4, C.byref(ms)), nm)
                    r[nm] = round(nb / (ms.value * 1e-3) / 1e12, 3)
                r["ratio208"] = round(r["reg208"] / r["page"], 3)
                row[f"{gb}GiB"] = r
            emit(row)
        for fb in bufs:
            fb.free()

elif what == "mix":
    n = 1 << 24
    names = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"]
    for i, nm in enumerate(names):
        ctx.load_sequence(i, Sequence.from_config(pc.get(nm)), pc.SEED_BASE)
    bufs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
    refs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
    seqs = (C.c_uint16 * 3)(0, 1, 2)
    outs = (C.c_void_p * 3)(*[C.cast(b.ptr, C.c_void_p) for b in bufs])
    routs = (C.c_void_p * 3)(*[C.cast(b.ptr, C.c_void_p) for b in refs])
    ms = D()
    V = [("product fused 512", 0), ("mix 512 product parts", 1), ("mix 512 wave-local 64B", 2),
         ("mix 512 wave-local 64B s80", 3), ("mix 512 product parts s80", 4), ("three launches", 5),
         ("mix 256 wave-local 64B", 6), ("mix 512 wave-owned stores s80", 7)]
    if os.environ.get("MIX_V"):
        keep = {int(x) for x in os.environ["MIX_V"].split(",")}
        V = [(nm, v) for nm, v in V if v in keep]
    ok(L.pr_mix(ctx.h, seqs, 3, n, routs, 5, 1, C.byref(ms)), "ref")
    for name, v in V:
        ok(L.pr_mix(ctx.h, seqs, 3, n, outs, v, 1, C.byref(ms)), name)
        bad = 0
        for i in range(3):
            b = C.c_uint64()
            nb = n * int(bufs[i].f.fixed_len)
            ok(L.pr_compare(ctx.h, C.c_void_p(data_ptr(bufs[i])), C.c_void_p(data_ptr(refs[i])), nb, C.byref(b)),
               "cmp")
            bad += b.value
        emit({"check": name, "bad_dwords": bad})
    ramp(lambda: L.pr_mix(ctx.h, seqs, 0, n, outs, 0, 8, C.byref(ms)))
    res = {name: [] for name, _ in V}
    for r in range(REPS):
        for name, v in V:
            ok(L.pr_mix(ctx.h, seqs, 0, n, outs, v, 20, C.byref(ms)), name)
            res[name].append(ms.value)
    tot = sum(n * int(b.f.fixed_len) for b in bufs)
    for k, v in res.items():
        s = sorted(v)
        emit({"variant": k, "ms_med": round(s[len(s) // 2], 5), "ms_min": round(s[0], 5),
              "tbps_med": round(tot / (s[len(s) // 2] * 1e-3) / 1e12, 3), "all": [round(x, 4) for x in v]})
    for b in bufs + refs:
        b.free()

elif what == "place":
    n = 1 << 25
    nbuf = int(os.environ.get("NBUF", "4"))
    ctx.load_sequence(0, Sequence.from_config(pc.get("c3_udp_var")), pc.SEED_BASE)
    ctx.load_sequence(1, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
    f0, b0 = ctx.build_size(0, n)
    f1, b1 = ctx.build_size(1, n)
    bufs = [ctx.alloc_frames(max(f0, f1), max(b0, b1)) for _ in range(nbuf)]
    nfill = L.pr_fill_count()
    fill_bytes = 27_600_000_000 // 4096 * 4096
    ms = D()
    ramp(lambda: L.pr_build(ctx.h, 1, 0, n, bufs[0].ptr, 4, C.byref(ms)))
    for rnd in range(int(os.environ.get("ROUNDS", "2"))):
        for i, fb in enumerate(bufs):
            row = {"round": rnd, "buf": i, "addr": hex(data_ptr(fb))}
            ok(L.pr_build(ctx.h, 0, 0, n, fb.ptr, 10, C.byref(ms)), "c3")
            row["c3_vline_ms"] = round(ms.value, 4)
            ok(L.pr_build(ctx.h, 1, 0, n, fb.ptr, 10, C.byref(ms)), "1500")
            row["c2_1500_ms"] = round(ms.value, 4)
            fills = {}
            for s in range(nfill):
                ok(L.pr_fill(ctx.h, C.c_void_p(data_ptr(fb)), fill_bytes, s, 2048, 5, C.byref(ms)), f"fill{s}")
                fills[L.pr_fill_name(s).decode()] = round(fill_bytes / (ms.value * 1e-3) / 1e12, 3)
            row["fill_tbps"] = fills
            emit(row)
    for fb in bufs:
        fb.free()
ctx.close()
