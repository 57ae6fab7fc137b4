"""GPU parity: libpbgpu.so (the HIP kernels, through the C ABI) against the
committed golden vectors and the CPU oracle, bit-exact; full-size properties
at BASELINE.json sizes.  Run on the MI355X box: pytest -m gpu."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import oracle_binding as ob
import pb_configs as pc
import pbgpu
import pyverify as pv
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
INDEX = json.load(open(os.path.join(GOLD, "index.json")))["fixtures"]


@pytest.fixture(scope="module")
def ctx():
    c = GpuContext(0)
    yield c
    c.close()


def gpu_build(ctx, cfg, first, n, seq_idx=0, rule=0, fold=0, seed_base=pc.SEED_BASE):
    seq = Sequence.from_config(cfg)
    ctx.load_sequence(seq_idx, seq, seed_base, payload_rule=rule, iph_fold=fold)
    mf, mb = ctx.build_size(seq_idx, n)
    fb = ctx.alloc_frames(mf, mb)
    ctx.build(seq_idx, first, n, fb)
    ctx.sync()
    data, off = fb.packed(), fb.offsets()
    fb.free()
    return data, off


@pytest.mark.parametrize("fx", INDEX, ids=[f["file"] for f in INDEX])
def test_gpu_matches_golden(ctx, fx):
    z = np.load(os.path.join(GOLD, fx["file"]), allow_pickle=False)
    data, off = gpu_build(ctx, pc.get(fx["config"]), fx["first_iter"], fx["n_iter"], fx["seq_idx"],
                          fx["payload_rule"], fx["iph_fold"], fx["seed_base"])
    assert np.array_equal(off, z["offsets"])
    assert np.array_equal(data, z["data"])


def _window_iters(cfg):
    mx = 54 + max([p.get("length", {}).get("max", 0) for p in cfg.get("payloads", [])] + [256])
    return max(64, min(40000, (24 << 20) // mx))


CASES = [(n, 0, 0) for n in pc.ALL] + list(pc.RULE_CASES)


@pytest.mark.parametrize("name,rule,fold", CASES)
def test_gpu_matches_oracle(ctx, name, rule, fold):
    """Thousands of iterations per config at an odd first_iter: every byte equal."""
    cfg = pc.get(name)
    n = _window_iters(cfg)
    first = 987654321
    g_data, g_off = gpu_build(ctx, cfg, first, n, 3, rule, fold)
    o_data, o_off = ob.build(Sequence.from_config(cfg), 3, first, n, pc.SEED_BASE, payload_rule=rule,
                             iph_fold=fold)
    assert np.array_equal(g_off, o_off)
    if not np.array_equal(g_data, o_data):
        bad = int(np.nonzero(g_data != o_data)[0][0])
        f = int(np.searchsorted(o_off, bad, side="right") - 1)
        pytest.fail(f"{name}: first mismatch at byte {bad} (frame {f}, offset {bad - int(o_off[f])})")


def test_sharded_builds_concatenate(ctx):
    """The multi-GPU invariant: any split of the iteration range builds the
    same frames (seeds depend only on (seq, k))."""
    for name in ("c2_udp_64", "c3_udp_var", "c4_tcp_syn", "udp_multi_payload"):
        cfg = pc.get(name)
        whole, woff = gpu_build(ctx, cfg, 5000, 3000)
        parts = [gpu_build(ctx, cfg, 5000 + a, b - a) for a, b in ((0, 1000), (1000, 1001), (1001, 3000))]
        assert np.array_equal(np.concatenate([p[0] for p in parts]), whole)


def _verify_fixed(frames: np.ndarray, proto: int):
    """Vectorised RFC 1071 check of every frame (n, flen)."""
    w = frames[:, 14:34].astype(np.uint32)
    s = (w[:, 0::2] << 8 | w[:, 1::2]).sum(axis=1)
    while (s >> 16).any():
        s = (s & 0xFFFF) + (s >> 16)
    assert (s == 0xFFFF).all(), "IPv4 checksum"
    n, flen = frames.shape
    seg = frames[:, 34:].astype(np.uint32)
    if seg.shape[1] & 1:
        seg = np.concatenate([seg, np.zeros((n, 1), np.uint32)], axis=1)
    s = (seg[:, 0::2] << 8 | seg[:, 1::2]).sum(axis=1).astype(np.uint64)
    ip = frames[:, 26:34].astype(np.uint64)
    s += (ip[:, 0::2] << 8 | ip[:, 1::2]).sum(axis=1)
    s += proto + (flen - 34)
    while (s >> 16).any():
        s = (s & 0xFFFF) + (s >> 16)
    assert (s == 0xFFFF).all(), "L4 checksum"


@pytest.mark.parametrize("name,n_iter", [("c2_udp_64", 1 << 25), ("c4_tcp_syn", 1 << 25), ("c2_udp_1500", 1 << 21)])
def test_full_size_properties(ctx, name, n_iter):
    """BASELINE.json sizes: every checksum of every frame verifies, and random
    sampled frames equal the oracle's."""
    cfg = pc.get(name)
    seq = Sequence.from_config(cfg)
    ctx.load_sequence(0, seq, pc.SEED_BASE)
    mf, mb = ctx.build_size(0, n_iter)
    fb = ctx.alloc_frames(mf, mb)
    ctx.build(0, 0, n_iter, fb)
    ctx.sync()
    flen = int(fb.f.fixed_len)
    assert flen > 0
    data = fb.packed()
    fb.free()
    frames = data.reshape(n_iter, flen)
    proto = 17 if cfg["ip"]["protocol"] == "udp" else 6
    for lo in range(0, n_iter, 1 << 22):
        _verify_fixed(frames[lo:lo + (1 << 22)], proto)
    rng = np.random.default_rng(1)
    for k in rng.integers(0, n_iter, 200):
        want = ob.frames(seq, 0, int(k), 1, pc.SEED_BASE)[0]
        assert frames[int(k)].tobytes() == want


@pytest.mark.parametrize("name", ["c2_udp_1500", "c3_udp_var", "c5_icmp_echo"])
def test_full_size_every_checksum(ctx, name):
    """SURVEY.md §8d sizes (2^25 iterations, 50 GB of 1500-B frames, 27.6 GB of packed
    configs[2] frames): every frame's IPv4 checksum, tot_len and L4 checksum verify,
    checked in host chunks by the C checker (pbo_verify_frames, RFC 1071 over the frame
    bytes); configs[2]'s offsets are a prefix sum of lengths in [106, 1542]."""
    seq = Sequence.from_config(pc.get(name))
    n = 1 << 25
    ctx.load_sequence(0, seq, pc.SEED_BASE)
    mf, mb = ctx.build_size(0, n)
    fb = ctx.alloc_frames(mf, mb)
    try:
        ctx.build(0, 0, n, fb)
        ctx.sync()
        flen = int(fb.f.fixed_len)
        off = None if flen else fb.offsets()
        if off is not None:
            lens = np.diff(off.astype(np.int64))
            assert off[0] == 0 and lens.min() >= 106 and lens.max() <= 1542
        ch = 1 << 21
        buf = np.empty(ch * (flen or 1542), dtype=np.uint8)
        bad = 0
        for lo in range(0, n, ch):
            hi = min(n, lo + ch)
            b0, b1 = (lo * flen, hi * flen) if flen else (int(off[lo]), int(off[hi]))
            assert ctx.lib.pbgpu_copy_packed(ctx.h, fb.ptr, buf.ctypes.data, b0, b1 - b0) == 0
            bad += ob.verify_frames(buf, None if flen else off[lo:hi + 1], flen, hi - lo, 16)
        assert bad == 0
    finally:
        fb.free()


def test_variable_full_size_offsets(ctx):
    """configs[2] at 2^22 frames: offsets are a prefix sum of lengths in
    [106, 1542], every sampled frame equals the oracle's, every checksum verifies."""
    cfg = pc.get("c3_udp_var")
    seq = Sequence.from_config(cfg)
    n = 1 << 22
    ctx.load_sequence(0, seq, pc.SEED_BASE)
    mf, mb = ctx.build_size(0, n)
    fb = ctx.alloc_frames(mf, mb)
    ctx.build(0, 0, n, fb)
    ctx.sync()
    off = fb.offsets()
    data = fb.packed()
    fb.free()
    lens = np.diff(off.astype(np.int64))
    assert lens.min() >= 106 and lens.max() <= 1542 and off[0] == 0
    rng = np.random.default_rng(2)
    for k in rng.integers(0, n, 300):
        k = int(k)
        got = data[int(off[k]):int(off[k + 1])].tobytes()
        assert got == ob.frames(seq, 0, k, 1, pc.SEED_BASE)[0]
        assert pv.ip_csum_ok(got) and pv.l4_csum_value(got) == pv.parse(got)["l4_csum"]


def test_counters_and_umem_landing(ctx):
    cfg = pc.get("c3_udp_var")
    seq = Sequence.from_config(cfg)
    ctx.load_sequence(7, seq, pc.SEED_BASE)
    p0, b0 = ctx.counters(8)
    mf, mb = ctx.build_size(7, 5000)
    fb = ctx.alloc_frames(mf, mb)
    ctx.build(7, 100, 5000, fb)
    ctx.sync()
    total = fb.total_bytes()
    p1, b1 = ctx.counters(8)
    assert int(p1[7] - p0[7]) == 5000 and int(b1[7] - b0[7]) == total
    want = ob.frames(seq, 7, 100, 5000, pc.SEED_BASE)
    umem = np.zeros(4096 * 1000, dtype=np.uint8)
    lens = fb.to_umem(umem, 4096, 2000, 1000)
    for j in range(1000):
        ln = int(lens[j])
        assert ln == len(want[2000 + j])
        assert umem[j * 4096:j * 4096 + ln].tobytes() == want[2000 + j]
    fb.free()
    # fixed length: 2-D copy into 4096-B slots
    ctx.load_sequence(8, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(8, 4096))
    ctx.build(8, 0, 4096, fb)
    ctx.sync()
    want = ob.frames(Sequence.from_config(pc.get("c2_udp_64")), 8, 0, 4096, pc.SEED_BASE)
    umem = np.zeros(4096 * 4096, dtype=np.uint8)
    lens = fb.to_umem(umem, 4096, 0, 4096)
    assert (lens == 64).all()
    for j in range(0, 4096, 97):
        assert umem[j * 4096:j * 4096 + 64].tobytes() == want[j]
    fb.free()


@pytest.mark.parametrize("name", ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo", "c2_udp_1500", "c1_udp_static_106"])
def test_umem_landing_registered(ctx, name):
    """Fixed-length frames into registered (mapped) UMEM: the GPU scatter kernel
    stores every frame into its 4 KiB slot (af_xdp.c:211-214); slot bytes past
    the frame are untouched."""
    seq = Sequence.from_config(pc.get(name))
    ctx.load_sequence(9, seq, pc.SEED_BASE)
    n = 3000
    fb = ctx.alloc_frames(*ctx.build_size(9, n))
    ctx.build(9, 555, n, fb)
    ctx.sync()
    want = ob.frames(seq, 9, 555, n, pc.SEED_BASE)
    umem = np.full(4096 * 1024, 0xEE, dtype=np.uint8)
    assert ctx.lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes) == 0
    try:
        lens = fb.to_umem(umem, 4096, 1000, 1024)
    finally:
        ctx.lib.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
    fb.free()
    flen = len(want[0])
    assert (lens == flen).all()
    slots = umem.reshape(1024, 4096)
    for j in range(1024):
        assert slots[j, :flen].tobytes() == want[1000 + j]
    assert (slots[:, flen:] == 0xEE).all()


def test_error_behaviour(ctx):
    seq = Sequence.from_config(pc.get("c2_udp_64"))
    ctx.load_sequence(0, seq, 1)
    fb = ctx.alloc_frames(10, 640)
    with pytest.raises(pbgpu.PbError) as e:
        ctx.build(0, 0, 11, fb)
    assert e.value.code == -28
    with pytest.raises(pbgpu.PbError) as e:
        ctx.build(200, 0, 1, fb)
    assert e.value.code == -2
    fb.free()
    bad = pc.get("c2_udp_64")
    bad["ip"]["ttl"] = {"min": 9, "max": 3}
    with pytest.raises(pbgpu.PbError) as e:
        ctx.load_sequence(1, Sequence.from_config(bad), 1)
    assert e.value.code == -22
    nodst = pc.get("c2_udp_64")
    del nodst["ip"]["dip"]
    with pytest.raises(pbgpu.PbError) as e:
        ctx.load_sequence(1, Sequence.from_config(nodst), 1)
    assert e.value.code == -22


def test_fill_probe_runs(ctx):
    ms = ctx.fill_probe(1 << 30, 5)
    gbps = (1 << 30) / (ms * 1e-3) / 1e9
    assert 500 < gbps < 9000


def test_timing_modes(ctx):
    """PBGPU_TIMING_LAUNCH sums per-launch event pairs; PBGPU_TIMING_SPAN spans
    the launches since the last kernel_time() with one pair; output identical."""
    seq = Sequence.from_config(pc.get("c2_udp_1500"))
    ctx.load_sequence(0, seq, pc.SEED_BASE)
    n = 4096
    fb = ctx.alloc_frames(*ctx.build_size(0, n))
    out = {}
    for mode in (ctx.TIMING_SPAN, ctx.TIMING_LAUNCH):
        ctx.set_timing(mode)
        for s in range(3):
            ctx.build(0, 1000 + s * n, n, fb)
        ctx.sync()
        ms, k = ctx.kernel_time()
        assert k == 3 and ms > 0
        assert ctx.kernel_time() == (0.0, 0)
        out[mode] = fb.packed().copy()
    assert np.array_equal(out[0], out[1])
    with pytest.raises(pbgpu.PbError):
        ctx.set_timing(7)
    fb.free()


@pytest.mark.parametrize("name", ["c3_udp_var", "c2_udp_1500", "tcp_all_flags_var"])
def test_async_landings_overlap_the_next_build(ctx, name):
    """pbgpu_copy_to_umem_async: three landings queued into registered 4 KiB slots
    (the second buffer building meanwhile on the build stream), waited oldest
    first; every slot holds its frame and nothing past it (af_xdp.c:211-214)."""
    seq = Sequence.from_config(pc.get(name))
    ctx.load_sequence(10, seq, pc.SEED_BASE)
    n = 3000
    a = ctx.alloc_frames(*ctx.build_size(10, n))
    b = ctx.alloc_frames(*ctx.build_size(10, n))
    umem = np.full(4096 * 4096, 0xEE, dtype=np.uint8)
    assert ctx.lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes) == 0
    lens = np.zeros(4096, dtype=np.uint16)
    L = ctx.lib
    L.pbgpu_copy_to_umem_async.argtypes = [C.c_void_p, C.POINTER(pbgpu.Frames), C.c_void_p, C.c_uint32, C.c_uint32,
                                           C.c_uint64, C.c_uint32, C.c_void_p]
    L.pbgpu_land_wait.argtypes = [C.c_void_p, C.c_uint32]
    try:
        ctx.build(10, 7, n, a)
        # first landing of a context synchronises the build stream; later ones wait on events
        assert L.pbgpu_copy_to_umem_async(ctx.h, a.ptr, umem.ctypes.data, 4096, 0, 0, 100, lens.ctypes.data) == 0
        assert L.pbgpu_land_wait(ctx.h, 0) == 0
        ctx.build(10, 7 + n, n, b)  # queued behind nothing the landings wait for
        chunks = [(100, 1000, 1500), (1600, 2500, 500), (3600, 0, 496)]  # (slot, first frame, count)
        for slot, first, cnt in chunks:
            assert L.pbgpu_copy_to_umem_async(ctx.h, a.ptr, umem.ctypes.data, 4096, slot, first, cnt,
                                              lens[slot:].ctypes.data) == 0
        assert L.pbgpu_land_wait(ctx.h, 2) == 0 and L.pbgpu_land_wait(ctx.h, 0) == 0
        ctx.sync()
    finally:
        L.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
    want_a = ob.frames(seq, 10, 7, n, pc.SEED_BASE)
    want_b = ob.frames(seq, 10, 7 + n, n, pc.SEED_BASE)
    slots = umem.reshape(4096, 4096)
    for slot, first, cnt in [(0, 0, 100)] + chunks:
        for j in range(cnt):
            f = want_a[first + j]
            assert int(lens[slot + j]) == len(f)
            assert slots[slot + j, :len(f)].tobytes() == f
            assert (slots[slot + j, len(f):] == 0xEE).all()
    assert b.frames() == want_b
    a.free()
    b.free()


def test_jumbo_frames_refused_by_4k_slots(ctx):
    """A frame longer than its UMEM slot is refused (-EINVAL), registered or not,
    fixed or variable length: nothing is written past a slot."""
    for name in ("udp_jumbo_var", "udp_jumbo_fixed_odd"):
        seq = Sequence.from_config(pc.get(name))
        ctx.load_sequence(11, seq, pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(11, 64))
        ctx.build(11, 0, 64, fb)
        ctx.sync()
        umem = np.full(4096 * 64, 0xEE, dtype=np.uint8)
        lens = np.zeros(64, dtype=np.uint16)
        for registered in (True, False):
            if registered:
                assert ctx.lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes) == 0
            rc = ctx.lib.pbgpu_copy_to_umem(ctx.h, fb.ptr, umem.ctypes.data, 4096, 0, 0, 64,
                                            lens.ctypes.data_as(C.POINTER(C.c_uint16)))
            if registered:
                ctx.lib.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
            assert rc == -22
            assert (umem == 0xEE).all()
        fb.free()


def test_unregistered_landing_of_a_large_batch(ctx):
    """Fixed-length frames into unregistered memory land by strided DMA: a 2^18-frame batch (the
    bench's D2H size) in runs of at most 32768 rows (one 2^18-row hipMemcpy2DAsync failed),
    every frame in its 4 KiB slot and the slot bytes past it untouched."""
    seq = Sequence.from_config(pc.get("c2_udp_64"))
    ctx.load_sequence(9, seq, pc.SEED_BASE)
    n = 1 << 18
    fb = ctx.alloc_frames(*ctx.build_size(9, n))
    ctx.build(9, 77, n, fb)
    ctx.sync()
    umem = np.full(4096 * n, 0xEE, dtype=np.uint8)
    lens = fb.to_umem(umem, 4096, 0, n)
    data = fb.packed()
    fb.free()
    assert (lens == 64).all()
    slots = umem.reshape(n, 4096)
    assert np.array_equal(slots[:, :64], data.reshape(n, 64))
    assert (slots[::511, 64:] == 0xEE).all()
    want = ob.frames(seq, 9, 77 + n - 40, 40, pc.SEED_BASE)
    assert [slots[n - 40 + j, :64].tobytes() for j in range(40)] == want


@pytest.mark.parametrize("dma_min", ["64", "100000"])
@pytest.mark.parametrize("name", ["c2_udp_64", "c2_udp_1500", "c5_icmp_echo"])
def test_umem_landing_dma_or_scatter(monkeypatch, name, dma_min):
    """Registered UMEM, both landing paths whatever the length (PBGPU_LAND_DMA_MIN: fixed frames
    of at least that many bytes go by strided DMA, the rest by the scatter kernel, the default):
    every frame in its 4 KiB slot, the bytes past it untouched, over two queued landings of
    40,000 frames each (two 32768-row DMA runs)."""
    monkeypatch.setenv("PBGPU_LAND_DMA_MIN", dma_min)
    c = GpuContext(0)
    try:
        seq = Sequence.from_config(pc.get(name))
        c.load_sequence(3, seq, pc.SEED_BASE)
        n = 80000
        fb = c.alloc_frames(*c.build_size(3, n))
        c.build(3, 9, n, fb)
        c.sync()
        data = fb.packed()
        flen = len(data) // n
        umem = np.full(4096 * n, 0xEE, dtype=np.uint8)
        assert c.lib.pbgpu_host_register(c.h, umem.ctypes.data, umem.nbytes) == 0
        try:
            lens_a = fb.to_umem(umem, 4096, 0, 40000)
            lens_b = fb.to_umem(umem, 4096, 40000, 40000, first_slot=40000)
        finally:
            c.lib.pbgpu_host_unregister(c.h, umem.ctypes.data)
        fb.free()
        assert (lens_a == flen).all() and (lens_b == flen).all()
        slots = umem.reshape(n, 4096)
        assert np.array_equal(slots[:, :flen], data.reshape(n, flen))
        assert (slots[::97, flen:] == 0xEE).all()
        assert slots[n - 1, :flen].tobytes() == ob.frames(seq, 3, 9 + n - 1, 1, pc.SEED_BASE)[0]
    finally:
        c.close()


@pytest.mark.parametrize("name,slot,whole", [("c2_udp_64", 64, True), ("c4_tcp_syn", 64, True),
                                             ("c5_icmp_echo", 128, True), ("c5_icmp_echo", 256, False),
                                             ("c2_udp_1500", 2048, False), ("c2_udp_64", 128, False)])
def test_umem_landing_tight_slots(ctx, name, slot, whole):
    """--umemslot: slots smaller than 4 KiB.  A tight slot (no longer than the frame rounded up to
    64 B) is written whole (the frame, then unspecified bytes: the packed stream's next ones, zeros
    past the buffer), so back-to-back slots reach the host as contiguous writes; a wider slot gets
    the frame's bytes only.  Every frame in its slot; nothing written outside the landed slots."""
    seq = Sequence.from_config(pc.get(name))
    ctx.load_sequence(9, seq, pc.SEED_BASE)
    n = 5000
    fb = ctx.alloc_frames(*ctx.build_size(9, n))
    ctx.build(9, 321, n, fb)
    ctx.sync()
    want = ob.frames(seq, 9, 321, n, pc.SEED_BASE)
    flen = len(want[0])
    first, cnt, s0 = 1000, n - 1000, 7  # the landing runs to the buffer's last frame
    umem = np.full(slot * (cnt + s0 + 3), 0xEE, dtype=np.uint8)
    assert ctx.lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes) == 0
    try:
        lens = fb.to_umem(umem, slot, first, cnt, first_slot=s0)
    finally:
        ctx.lib.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
    fb.free()
    assert (lens == flen).all()
    slots = umem.reshape(-1, slot)
    for j in range(cnt):
        assert slots[s0 + j, :flen].tobytes() == want[first + j], j
    assert (slots[:s0] == 0xEE).all() and (slots[s0 + cnt:] == 0xEE).all()
    if whole:
        # the filler is the next frame's leading bytes (the last slot's: the buffer's tail)
        nxt = np.frombuffer(b"".join(want[first + 1:]), dtype=np.uint8)
        tail = slots[s0:s0 + cnt - 1, flen:]
        assert np.array_equal(tail, np.stack([nxt[j * flen:j * flen + slot - flen] for j in range(cnt - 1)]))
        assert (slots[s0 + cnt - 1, flen:] != 0xEE).any() or slot == flen
    else:
        assert (slots[s0:s0 + cnt, flen:] == 0xEE).all()
