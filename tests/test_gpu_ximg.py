"""pb_ximg_body: static-payload ICMP frames built as a copy of the stream's first img_np pages
(made once at load by pb_xpage_kernel) with each frame's IPv4 ID, TTL, checksum and source
address written over it.  It runs as configs[4]'s ICMP part of pb_batch_kernel;
PBGPU_XP_IMG=2 runs it for single builds too (pb_ximg_kernel), which the length sweep uses.  Bit-exact against the oracle with every one of those
fields random (TTL, ID, several CIDR ranges), at every even length from 52 to 126 B (slots past 64
per page below 66 B), odd first iterations, counts that end inside a page and past the image
period; the >= 2^31 first-frame path; and inside configs[4]'s fused launch at full size."""
import copy

import numpy as np
import pytest

import oracle_binding as ob
import pb_configs as pc
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = GpuContext(0)
    yield c
    c.close()


def _cfg(flen, rnd=True):
    cfg = copy.deepcopy(pc.get("c5_icmp_echo"))
    cfg["payloads"] = [{"exact": " ".join("%02X" % ((i * 29 + 3) & 255) for i in range(flen - 42))}]
    if rnd:
        cfg["ip"]["ttl"] = {"min": 3, "max": 250}
        cfg["ip"]["id"] = {"min": 7, "max": 65000}
        cfg["ip"]["ranges"] = ["10.20.0.0/16", "192.168.7.0/24", "172.16.0.1/32"]
    return cfg


@pytest.fixture(autouse=True)
def _solo(monkeypatch):
    monkeypatch.setenv("PBGPU_XP_IMG", "2")


def _check(ctx, cfg, first, n):
    seq = Sequence.from_config(cfg)
    ctx.load_sequence(3, seq, pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(3, n))
    ctx.build(3, first, n, fb)
    ctx.sync()
    g = fb.packed()
    fb.free()
    o, _ = ob.build(seq, 3, first, n, pc.SEED_BASE)
    assert g.shape == o.shape
    if not np.array_equal(g, o):
        bad = int(np.nonzero(g != o)[0][0])
        flen = cfg_len = len(g) // n
        pytest.fail(f"first mismatch at byte {bad} (frame {bad // flen}, offset {bad % cfg_len})")
    return ctx.kernel_name(3)


@pytest.mark.parametrize("flen", [52, 54, 58, 62, 66, 70, 74, 90, 98, 102, 106, 110, 114, 118, 122, 126])
def test_ximg_matches_oracle(ctx, flen):
    cfg = _cfg(flen)
    period = flen // np.gcd(flen, 4096) * 4096 // flen  # frames per image period
    for first, n in ((1, 1), (12345, 77), (999_999_937, 4096 * 3 // flen + 5), (31, 3 * period + 13),
                     (7, 40000)):
        kern = _check(ctx, cfg, first, n)
        assert kern.startswith("pb_ximg_kernel"), kern


def test_ximg_fixed_fields(ctx):
    """No random field at all (only the source range's draw): the page copies alone."""
    cfg = _cfg(98, rnd=False)
    cfg["ip"]["ranges"] = ["10.20.30.40/32"]
    kern = _check(ctx, cfg, 5, 50000)
    assert kern.startswith("pb_ximg_kernel"), kern


def test_ximg_64bit_first_frame(ctx, monkeypatch):
    """PBGPU_XP_FA64=1: the pages' first frames by the 64-bit path at every size."""
    monkeypatch.setenv("PBGPU_XP_FA64", "1")
    kern = _check(ctx, _cfg(98), 424242, 30000)
    assert kern.startswith("pb_ximg_kernel"), kern


def test_ximg_in_batch_matches_separate_builds(ctx, monkeypatch):
    """configs[4]'s fused launch (pb_batch_kernel's ICMP part runs pb_ximg_body) equals the three
    sequences' own builds at 2^22 frames each."""
    monkeypatch.delenv("PBGPU_XP_IMG")  # the default: pb_ximg_body in the batch only
    names = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"]
    n = 1 << 22
    for i, nm in enumerate(names):
        ctx.load_sequence(i, Sequence.from_config(pc.get(nm)), pc.SEED_BASE)
    a = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
    b = [ctx.alloc_frames(*ctx.build_size(i, n)) for i in range(3)]
    ctx.build_batch([(i, 3 * n, n, a[i]) for i in range(3)])
    for i in range(3):
        ctx.build(i, 3 * n, n, b[i])
    ctx.sync()
    assert "pb_ximg_body" in ctx.kernel_name(2) and ctx.kernel_name(2).startswith("pb_xpage_kernel")
    for i in range(3):
        assert np.array_equal(a[i].packed(), b[i].packed()), names[i]
    o, _ = ob.build(Sequence.from_config(pc.get("c5_icmp_echo")), 2, 3 * n + n - 5000, 5000, pc.SEED_BASE)
    assert np.array_equal(a[2].packed()[-len(o):], o)
    for fb in a + b:
        fb.free()
