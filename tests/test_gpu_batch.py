"""pbgpu_build_batch: configs[4]'s three sequences (64-B UDP, 60-B TCP SYN, 98-B ICMP echo) as
one fused launch (pb_batch_kernel), bit-exact against the CPU oracle part by part, at both block
sizes and both timing modes, with ragged part sizes (partial pages, tail workgroups), against the
per-sequence launches at size, and the counters; other sets fall back to one launch per part."""
import numpy as np
import pytest

import oracle_binding as ob
import pb_configs as pc
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu

MIX = ("c2_udp_64", "c4_tcp_syn", "c5_icmp_echo")


@pytest.fixture(scope="module")
def seqs():
    return [Sequence.from_config(pc.get(nm)) for nm in MIX]


def _load(ctx, seqs, slots=(0, 1, 2)):
    for i, s in zip(slots, seqs):
        ctx.load_sequence(i, s, pc.SEED_BASE)


def _oracle_check(seq, idx, first, n, fb):
    o_data, o_off = ob.build(seq, idx, first, n, pc.SEED_BASE)
    g = fb.packed()
    assert np.array_equal(fb.offsets(), o_off)
    if not np.array_equal(g, o_data):
        bad = int(np.nonzero(g != o_data)[0][0])
        pytest.fail(f"seq {idx}: first mismatch at byte {bad} (frame {bad // int(fb.f.fixed_len)})")


@pytest.mark.parametrize("wgt", ["512", "256"])
@pytest.mark.parametrize("timing", ["span", "launch"])
def test_batch_matches_oracle(monkeypatch, seqs, wgt, timing):
    monkeypatch.setenv("PBGPU_BATCH_WGT", wgt)
    sizes = [(7, 70001), (100, 5003), (3, 64)]  # (first_iter, n_iter) per part: ragged tails
    with GpuContext(0) as ctx:
        _load(ctx, seqs)
        ctx.set_timing(ctx.TIMING_SPAN if timing == "span" else ctx.TIMING_LAUNCH)
        bufs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i, (_, n) in enumerate(sizes)]
        # parts in another order than the kinds: the library sorts them
        order = [2, 0, 1]
        ctx.build_batch([(i, sizes[i][0], sizes[i][1], bufs[i]) for i in order])
        ctx.sync()
        ms, cnt = ctx.kernel_time()
        assert cnt == 1, "one fused launch"
        for i, (first, n) in enumerate(sizes):
            _oracle_check(seqs[i], i, first, n, bufs[i])
        for fb in bufs:
            fb.free()


def test_batch_matches_separate_builds_at_size(seqs):
    """2^22 iterations per part: the fused launch builds the bytes the three page kernels do."""
    n = 1 << 22
    with GpuContext(0) as ctx:
        _load(ctx, seqs)
        a = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
        b = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
        ctx.build_batch([(i, 12345 + i, n, a[i]) for i in range(3)])
        for i in range(3):
            ctx.build(i, 12345 + i, n, b[i])
        ctx.sync()
        for i in range(3):
            assert np.array_equal(a[i].packed(), b[i].packed()), MIX[i]
        for fb in a + b:
            fb.free()


def test_batch_counters(seqs):
    n = 300007
    with GpuContext(0) as ctx:
        _load(ctx, seqs)
        bufs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
        ctx.set_timing(ctx.TIMING_SPAN)
        for k in range(5):
            ctx.build_batch([(i, k * n, n, bufs[i]) for i in range(3)])
        ctx.build(1, 0, n, bufs[1])  # a single build between batches keeps counting
        ctx.build_batch([(i, 0, n, bufs[i]) for i in range(3)])
        ctx.sync()
        p, b = ctx.counters(3)
        want = [6 * n, 7 * n, 6 * n]
        assert [int(x) for x in p] == want
        assert [int(x) for x in b] == [w * int(fb.f.fixed_len) for w, fb in zip(want, bufs)]
        for fb in bufs:
            fb.free()


def test_batch_fallback_sets(seqs, monkeypatch):
    """Sets without a fused form (two parts; a repeated kind; PBGPU_BATCH=0) build one launch per
    part, with the same bytes."""
    with GpuContext(0) as ctx:
        _load(ctx, seqs)
        _load(ctx, [seqs[1]], slots=(3,))
        ctx.set_timing(ctx.TIMING_LAUNCH)
        n = 4099
        bufs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(4)]
        ctx.build_batch([(0, 5, n, bufs[0]), (2, 6, n, bufs[2])])
        ctx.sync()
        assert ctx.kernel_time()[1] == 2
        _oracle_check(seqs[0], 0, 5, n, bufs[0])
        _oracle_check(seqs[2], 2, 6, n, bufs[2])
        ctx.build_batch([(1, 9, n, bufs[1]), (3, 9, n, bufs[3]), (2, 9, n, bufs[2])])
        ctx.sync()
        assert ctx.kernel_time()[1] == 3
        _oracle_check(seqs[1], 1, 9, n, bufs[1])
        _oracle_check(seqs[1], 3, 9, n, bufs[3])
        monkeypatch.setenv("PBGPU_BATCH", "0")  # read when a sequence is loaded
        _load(ctx, seqs)
        ctx.build_batch([(i, 11, n, bufs[i]) for i in range(3)])
        ctx.sync()
        assert ctx.kernel_time()[1] == 3
        for i in range(3):
            _oracle_check(seqs[i], i, 11, n, bufs[i])
        for fb in bufs:
            fb.free()


def test_batch_failure_leaves_counters_exact(seqs):
    """A part that cannot be built (its buffer too small) fails the whole call before any part
    reserves count records or is launched: the counters afterwards are exactly the earlier
    builds' (advisor, round 4), and the next batch counts normally."""
    n = 70001
    with GpuContext(0) as ctx:
        _load(ctx, seqs)
        bufs = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
        small = ctx.alloc_frames(*ctx.build_size(2, n // 2))
        ctx.build_batch([(i, 0, n, bufs[i]) for i in range(3)])
        with pytest.raises(Exception) as e:
            ctx.build_batch([(0, n, n, bufs[0]), (1, n, n, bufs[1]), (2, n, n, small)])
        assert "ENOSPC" in str(e.value)
        ctx.sync()
        p, b = ctx.counters(3)
        assert [int(x) for x in p] == [n] * 3
        assert [int(x) for x in b] == [n * int(fb.f.fixed_len) for fb in bufs]
        ctx.build_batch([(i, 2 * n, n, bufs[i]) for i in range(3)])
        ctx.sync()
        p, b = ctx.counters(3)
        assert [int(x) for x in p] == [2 * n] * 3
        for fb in bufs + [small]:
            fb.free()
