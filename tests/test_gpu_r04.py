"""Round-4 GPU checks: the counters' per-workgroup record ring (pb_count writes one record per
workgroup with a plain store; pb_ctr_fold adds the records into the counters when the ring is
full, when a slot is reloaded and when pbgpu_counters reads them), across timing modes, the
three kernel families of configs[4] and configs[2], and against the atomic form."""
import numpy as np
import pytest

import pb_configs as pc
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu

NAMES = ["c2_udp_64", "c3_udp_var", "c5_icmp_echo", "c4_tcp_syn"]


def _run(monkeypatch, ring=None, atomic=False, launches=12, n=100000, reload_at=5):
    """Builds `launches` batches of every sequence, alternating span / per-launch timing and
    reading the counters part way; returns (counted frames, counted bytes, expected frames,
    expected bytes) per sequence."""
    if ring:
        monkeypatch.setenv("PBGPU_CTR_RING", str(ring))
    if atomic:
        monkeypatch.setenv("PBGPU_CTR_ATOMIC", "1")
    with GpuContext(0) as ctx:
        seqs = [Sequence.from_config(pc.get(nm)) for nm in NAMES]
        for i, s in enumerate(seqs):
            ctx.load_sequence(i, s, pc.SEED_BASE)
        bufs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(len(NAMES))]
        want_p = np.zeros(len(NAMES), dtype=np.int64)
        want_b = np.zeros(len(NAMES), dtype=np.int64)
        for k in range(launches):
            ctx.set_timing(ctx.TIMING_SPAN if k % 2 == 0 else ctx.TIMING_LAUNCH)
            for i in range(len(NAMES)):
                ctx.build(i, 1000 + k * n, n, bufs[i])
            ctx.sync()
            for i, fb in enumerate(bufs):
                want_p[i] += n
                want_b[i] += fb.total_bytes()
            ctx.kernel_time()
            if k == reload_at:
                # a reload folds the slot's pending records into its running totals first
                ctx.load_sequence(2, seqs[2], pc.SEED_BASE)
            if k % 4 == 3:
                p, b = ctx.counters(len(NAMES))
                assert np.array_equal(p.astype(np.int64), want_p) and np.array_equal(b.astype(np.int64), want_b)
        p, b = ctx.counters(len(NAMES))
        for fb in bufs:
            fb.free()
    return p.astype(np.int64), b.astype(np.int64), want_p, want_b


@pytest.mark.parametrize("ring", [None, 3000, 900])
def test_counter_ring_counts_every_launch(monkeypatch, ring):
    """Default ring (no fold before the reads), a ring that folds every few launches, and one
    smaller than a single launch's records (it grows)."""
    p, b, wp, wb = _run(monkeypatch, ring=ring)
    assert np.array_equal(p, wp), (p, wp)
    assert np.array_equal(b, wb), (b, wb)


def test_counter_ring_matches_the_atomic_form(monkeypatch):
    ring = _run(monkeypatch, ring=3000, launches=6)
    monkeypatch.delenv("PBGPU_CTR_RING")
    atomic = _run(monkeypatch, atomic=True, launches=6)
    for r, a in zip(ring, atomic):
        assert np.array_equal(r, a)


def test_xsmall_first_build_is_one_launch(monkeypatch):
    """The 64-B page kernel's shape (one wave per page, 3 workgroups per CU) is fixed when the
    sequence is loaded: the first >= 2^22-frame build into a fresh buffer is one asynchronous
    launch (no calibration launches into the caller's buffer, round-4 advisor), the frames equal
    the oracle's and the counters count exactly the builds."""
    import oracle_binding as ob

    n = (1 << 22) + 77  # a page-group tail (pages past the stream skipped)
    seq = Sequence.from_config(pc.get("c2_udp_64"))
    with GpuContext(0) as ctx:
        ctx.load_sequence(0, seq, pc.SEED_BASE)
        ctx.set_timing(ctx.TIMING_LAUNCH)
        fb = ctx.alloc_frames(*ctx.build_size(0, n))
        ctx.build(0, 777, n, fb)
        ctx.sync()
        assert ctx.kernel_time()[1] == 1
        ctx.build(0, 777, n, fb)
        ctx.sync()
        p, b = ctx.counters(1)
        assert int(p[0]) == 2 * n and int(b[0]) == 2 * n * 64
        assert ctx.kernel_name(0) == "pb_xsmall_kernel<16, 17, true, 256>"
        data = fb.packed()
        fb.free()
    o_data, _ = ob.build(seq, 0, 777, n, pc.SEED_BASE)
    assert np.array_equal(data, o_data)
