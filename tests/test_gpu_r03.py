"""Round-3 GPU checks of behaviour around the kernels: counters that count work
(sequence.c:633-653: every workgroup adds the frames it built and the bytes it
stored), a rebuild of a buffer whose landing is still queued, and the drop-in
binary's seeding (sequence.c:434-441)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle_binding as ob
import pb_configs as pc
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "pb-af-xdp_amd", "bin", "pcktbatch-gpu")


@pytest.fixture(scope="module")
def ctx():
    c = GpuContext(0)
    yield c
    c.close()


def _count(ctx, name, n, first=0, idx=3):
    seq = Sequence.from_config(pc.get(name))
    ctx.load_sequence(idx, seq, pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(idx, n))
    p0, b0 = ctx.counters(idx + 1)
    ctx.build(idx, first, n, fb)
    ctx.sync()
    p1, b1 = ctx.counters(idx + 1)
    total = fb.total_bytes()
    kern = ctx.kernel_name(idx)
    fb.free()
    return int(p1[idx] - p0[idx]), int(b1[idx] - b0[idx]), total, kern


# every kernel shape: the small / page / staged / variable / group-per-frame paths
@pytest.mark.parametrize("name", ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo", "c1_udp_static_106", "c2_udp_1500",
                                  "c3_udp_var", "udp_multi_payload", "udp_jumbo_var", "udp_fixed_odd_65",
                                  "tcp_all_flags_var", "udp_tiny_var"])
@pytest.mark.parametrize("n", [1, 777, 40000])
def test_counters_count_built_frames_and_stored_bytes(ctx, name, n):
    frames, stored, total, kern = _count(ctx, name, n, first=12345)
    fpi = max(1, len(pc.get(name).get("payloads", [])))
    assert frames == n * fpi, kern
    assert stored == total, kern


def test_rebuild_waits_for_the_queued_landing(ctx):
    """copy_to_umem_async from a buffer, then pbgpu_build into the same buffer at
    once: the landed slots hold the first build's frames (the build stream waits
    for the landing, pbgpu.h)."""
    lib = ctx.lib
    lib.pbgpu_copy_to_umem_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64,
                                             C.c_uint32, C.POINTER(C.c_uint16)]
    lib.pbgpu_land_wait.argtypes = [C.c_void_p, C.c_uint32]
    seq = Sequence.from_config(pc.get("c2_udp_1500"))
    ctx.load_sequence(5, seq, pc.SEED_BASE)
    n = 4096
    fb = ctx.alloc_frames(*ctx.build_size(5, n))
    umem = np.zeros(4096 * n, dtype=np.uint8)
    assert lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes) == 0
    lens = np.zeros(n, dtype=np.uint16)
    try:
        for rep in range(3):
            ctx.build(5, rep * 10 * n, n, fb)
            assert lib.pbgpu_copy_to_umem_async(ctx.h, fb.ptr, umem.ctypes.data, 4096, 0, 0, n,
                                                lens.ctypes.data_as(C.POINTER(C.c_uint16))) == 0
            for r2 in range(3):  # rebuild the same buffer while the landing is queued
                ctx.build(5, rep * 10 * n + (r2 + 1) * n, n, fb)
            assert lib.pbgpu_land_wait(ctx.h, 0) == 0
            ctx.sync()
            want = ob.frames(seq, 5, rep * 10 * n, 64, pc.SEED_BASE)
            slots = umem.reshape(n, 4096)
            for j in range(64):
                assert slots[j, :1500].tobytes() == want[j]
            assert (lens == 1500).all()
    finally:
        lib.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
        fb.free()


def _pcap_frames(path):
    raw = open(path, "rb").read()
    out, p = [], 24
    while p + 16 <= len(raw):
        n = int.from_bytes(raw[p + 8:p + 12], "little")
        out.append(raw[p + 16:p + 16 + n])
        p += 16 + n
    return out


def test_binary_draws_a_seed_per_run_unless_given(tmp_path):
    """pcktbatch-gpu without --seed: a fresh seed base per run (printed, replayable);
    with --seed S: the same frames every run."""
    def run(tag, *extra):
        pcap = tmp_path / f"{tag}.pcap"
        cmd = [BIN, "-z", "--interface", "pbnodev0", "--smac", pc.SMAC, "--dmac", pc.DMAC, "--dip", pc.DIP,
               "--sip", "10.20.0.0/16", "--protocol", "udp", "--udport", "27015", "--pmin", "22", "--pmax", "22",
               "--maxpckts", "200", "--delay", "0", "--gpubatch", "200", "--pcap", str(pcap), *extra]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, PB_SEQ_GAP_MS="0"))
        assert r.returncode == 0, r.stderr
        seed = [l for l in r.stdout.splitlines() if l.startswith("Seed base =>")]
        assert len(seed) == 1
        return _pcap_frames(pcap), seed[0]

    a, sa = run("a")
    b, sb = run("b")
    assert len(a) == len(b) == 200 and sa != sb and a != b
    c, _ = run("c", "--seed", "0x1234")
    d, _ = run("d", "--seed", "0x1234")
    assert c == d
    # the printed seed replays the drawn run exactly
    replay = sa.split("--seed ")[1].rstrip(").")
    e, _ = run("e", "--seed", replay)
    assert e == a


# span timing: each sequence builds on a stream of its own, so the kernels of different
# sequences overlap; a buffer rebuilt by another sequence, the counters, the span and the
# copies must still see every build in order
def test_sequence_streams_build_the_same_bytes(ctx):
    names = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo", "c3_udp_var"]
    n = 5000
    seqs = [Sequence.from_config(pc.get(nm)) for nm in names]
    for i, s in enumerate(seqs):
        ctx.load_sequence(4 + i, s, pc.SEED_BASE)
    cap = [ctx.build_size(4 + i, n) for i in range(len(names))]
    shared = ctx.alloc_frames(max(c[0] for c in cap), max(c[1] for c in cap))
    bufs = [ctx.alloc_frames(*c) for c in cap]
    ctx.set_timing(ctx.TIMING_SPAN)
    try:
        p0, b0 = ctx.counters(4 + len(names))
        for rep in range(3):
            for i in range(len(names)):
                ctx.build(4 + i, 100 + rep * n, n, bufs[i])
        # one buffer built by every sequence in turn, last by the variable-length one
        for i in range(len(names)):
            ctx.build(4 + i, 77, n, shared)
        ms, k = ctx.kernel_time()
        assert k == 3 * len(names) + len(names) and ms > 0
        p1, b1 = ctx.counters(4 + len(names))
        for i, s in enumerate(seqs):
            data, off = bufs[i].packed(), bufs[i].offsets()
            o_data, o_off = ob.build(s, 4 + i, 100 + 2 * n, n, pc.SEED_BASE)
            assert np.array_equal(off, o_off) and np.array_equal(data, o_data), names[i]
            assert int(p1[4 + i] - p0[4 + i]) == 4 * n
        o_data, o_off = ob.build(seqs[-1], 4 + len(names) - 1, 77, n, pc.SEED_BASE)
        assert np.array_equal(shared.offsets(), o_off) and np.array_equal(shared.packed(), o_data)
    finally:
        ctx.set_timing(ctx.TIMING_LAUNCH)
        for b in bufs + [shared]:
            b.free()


# pb_vpage_kernel's record pass and pb_vline_kernel write 4-B offsets and region starts; offsets[]
# is expanded on first use and must follow every rebuild of the buffer (a stale expansion would
# keep the first build's)
@pytest.mark.parametrize("kernel", ["vpage", "vline"])
def test_packed_offsets_expand_after_every_build(ctx, monkeypatch, kernel):
    if kernel == "vpage":
        monkeypatch.setenv("PBGPU_KERNEL", "vpage")
    seq = Sequence.from_config(pc.get("c3_udp_var"))
    ctx.load_sequence(9, seq, pc.SEED_BASE)
    n = 3001
    fb = ctx.alloc_frames(*ctx.build_size(9, n))
    try:
        assert ctx.kernel_name(9).startswith("pb_%s_kernel" % kernel)
        for first in (5, 123457, 5):
            ctx.build(9, first, n, fb)
            fb.fill_offsets()
            fb.fill_offsets()  # a second call is a no-op
            o_data, o_off = ob.build(seq, 9, first, n, pc.SEED_BASE)
            assert np.array_equal(fb.offsets(), o_off)
            assert np.array_equal(fb.packed(), o_data)
    finally:
        fb.free()


def test_counters_survive_reloading_a_slot(ctx):
    """A slot reloaded with a sequence of another length keeps the counts it had."""
    p0, b0 = ctx.counters(12)
    for name, n in (("c2_udp_64", 1000), ("c5_icmp_echo", 3000), ("c3_udp_var", 700), ("c2_udp_64", 10)):
        seq = Sequence.from_config(pc.get(name))
        ctx.load_sequence(11, seq, pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(11, n))
        ctx.build(11, 0, n, fb)
        ctx.sync()
        fb.free()
    p1, b1 = ctx.counters(12)
    assert int(p1[11] - p0[11]) == 1000 + 3000 + 700 + 10
