"""GPU parity of every kernel shape the library can select, not only the
default one: the staged kernel at other lane-group / window / workgroup sizes,
the group-per-frame kernel (the fallback for frames too long for an LDS stage)
and the tile kernel, each bit-exact against the CPU oracle on every config.
Selection is through the library's PBGPU_* environment overrides, which
pbgpu_load_sequence() reads.  Run on the MI355X box: pytest -m gpu."""
import copy
import os

import numpy as np
import pytest

import oracle_binding as ob
import pb_configs as pc
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu

SHAPES = [
    ("gpf", {"PBGPU_KERNEL": "gpf"}, ("pb_gpf_kernel", "pb_xsmall_kernel", "pb_small_kernel<")),
    ("nopage_small", {"PBGPU_KERNEL": "nopage"},
     ("pb_small_kernel", "pb_xsmall_kernel", "pb_stage_kernel", "pb_gpf_kernel", "pb_fstage_kernel", "pb_vstage_kernel",
      "pb_vline_kernel", "pb_vpage_kernel")),
    ("xpage_forced", {"PBGPU_XP_FORCE": "1"},
     ("pb_xpage_kernel", "pb_xsmall_kernel", "pb_small_kernel<", "pb_stage_kernel", "pb_gpf_kernel", "pb_fstage_kernel",
      "pb_vstage_kernel", "pb_vline_kernel", "pb_vpage_kernel")),
    ("linear_small", {"PBGPU_KERNEL": "linear"},
     ("pb_small_kernel", "pb_stage_kernel", "pb_gpf_kernel", "pb_fstage_kernel", "pb_vstage_kernel", "pb_vline_kernel",
      "pb_vpage_kernel")),
    # the page-shaped packed writer (pb_vrec_kernel + pb_vpage_kernel) on every config
    ("vpage", {"PBGPU_KERNEL": "vpage"},
     ("pb_vpage_kernel", "pb_vline_kernel", "pb_vstage_kernel", "pb_xsmall_kernel", "pb_xpage_kernel", "pb_small_kernel<",
      "pb_fstage_kernel", "pb_stage_kernel", "pb_gpf_kernel", "pb_ximg_kernel")),
    ("stage_g8_wgf5", {"PBGPU_KERNEL": "stage", "PBGPU_G": "8", "PBGPU_WGF": "5"},
     ("pb_stage_kernel<8", "pb_xsmall_kernel", "pb_small_kernel<")),
    ("stage_g64_kb4", {"PBGPU_KERNEL": "stage", "PBGPU_G": "64", "PBGPU_STAGE_KB": "4"},
     ("pb_stage_kernel<64", "pb_xsmall_kernel", "pb_small_kernel<")),
    ("stage_wave", {"PBGPU_KERNEL": "stage", "PBGPU_WGT": "64", "PBGPU_WGF": "24"},
     ("pb_stage_kernel", "pb_xsmall_kernel", "pb_small_kernel<")),
    ("stage_g32_kb36", {"PBGPU_KERNEL": "stage", "PBGPU_G": "32", "PBGPU_STAGE_KB": "36"},
     ("pb_stage_kernel<32", "pb_xsmall_kernel", "pb_small_kernel<")),
    # pb_vstage_kernel (random payloads) at other lane-group / window / workgroup sizes;
    # static and mixed payloads keep pb_stage_kernel at the same shape
    ("vstage_g16", {"PBGPU_G": "16", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<16", "pb_stage_kernel<16", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<")),
    ("vstage_g64_kb8", {"PBGPU_G": "64", "PBGPU_STAGE_KB": "8", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<64", "pb_stage_kernel<64", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<")),
    ("vstage_g32_wgf7", {"PBGPU_G": "32", "PBGPU_WGF": "7", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<32", "pb_stage_kernel<32", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<")),
    # pb_vstage_kernel's lane layouts by window: fixed 8-lane groups (bit 4) and
    # no 32-lane groups (bit 5) build the same bytes as the default 32/16/8 layout
    ("vstage_fixed8", {"PBGPU_VST_SHAPE": "16", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<", "pb_stage_kernel", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<",
      "pb_xpage_kernel", "pb_gpf_kernel")),
    ("vstage_no32", {"PBGPU_VST_SHAPE": "32", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<", "pb_stage_kernel", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<",
      "pb_xpage_kernel", "pb_gpf_kernel")),
    # the other correct-output switches: workgroup edges at frame starts (lines split between
    # workgroups, masked stores at every edge), natural window order, the 3-pass offsets scan
    ("vstage_split_edges", {"PBGPU_VST_SHAPE": "64", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<", "pb_stage_kernel", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<",
      "pb_xpage_kernel", "pb_gpf_kernel")),
    ("vstage_no_order", {"PBGPU_VST_SHAPE": "256", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<", "pb_stage_kernel", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<",
      "pb_xpage_kernel", "pb_gpf_kernel")),
    ("vstage_3pass_kb8", {"PBGPU_VST_SCAN": "3pass", "PBGPU_STAGE_KB": "8", "PBGPU_KERNEL": "vstage"},
     ("pb_vstage_kernel<", "pb_stage_kernel", "pb_fstage_kernel", "pb_xsmall_kernel", "pb_small_kernel<",
      "pb_xpage_kernel", "pb_gpf_kernel")),
]

# pb_fstage_kernel shapes (fixed lengths > 128 B, multiple of 4, random payload)
FST_SHAPES = [
    ("fst_default", {}),
    ("fst_g32", {"PBGPU_FST_G": "32"}),
    ("fst_g16_nb2", {"PBGPU_FST_G": "16", "PBGPU_FST_NBUF": "2"}),
    ("fst_g64_nb1", {"PBGPU_FST_G": "64", "PBGPU_FST_NBUF": "1"}),
    ("fst_g16_nb1_wgf48", {"PBGPU_FST_G": "16", "PBGPU_FST_NBUF": "1", "PBGPU_FST_WGF": "48"}),
    ("fst_g32_wgf256", {"PBGPU_FST_G": "32", "PBGPU_FST_WGF": "256"}),
]


@pytest.fixture(scope="module")
def ctx():
    c = GpuContext(0)
    yield c
    c.close()


def _iters(cfg, budget=6 << 20):
    mx = 54 + max([p.get("length", {}).get("max", 0) for p in cfg.get("payloads", [])] + [256])
    return max(32, min(6000, budget // mx))


def _check(ctx, cfg, first, n, rule=0, fold=0):
    seq = Sequence.from_config(cfg)
    ctx.load_sequence(5, seq, pc.SEED_BASE, payload_rule=rule, iph_fold=fold)
    fb = ctx.alloc_frames(*ctx.build_size(5, n))
    ctx.build(5, first, n, fb)
    ctx.sync()
    g_data, g_off = fb.packed(), fb.offsets()
    fb.free()
    o_data, o_off = ob.build(seq, 5, first, n, pc.SEED_BASE, payload_rule=rule, iph_fold=fold)
    assert np.array_equal(g_off, o_off)
    if not np.array_equal(g_data, o_data):
        bad = int(np.nonzero(g_data != o_data)[0][0])
        f = int(np.searchsorted(o_off, bad, side="right") - 1)
        pytest.fail(f"first mismatch at byte {bad} (frame {f}, offset {bad - int(o_off[f])})")
    return ctx.kernel_name(5)


@pytest.mark.parametrize("shape,env,kernels", SHAPES, ids=[s[0] for s in SHAPES])
@pytest.mark.parametrize("name", pc.ALL)
def test_kernel_shape_matches_oracle(ctx, monkeypatch, shape, env, kernels, name):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg = pc.get(name)
    kern = _check(ctx, cfg, 123456789, _iters(cfg))
    if "pb_xsmall_kernel" in kernels:  # small frames keep their page kernels under the staged overrides
        kernels = kernels + ("pb_xpage_kernel",)
    assert kern.startswith(kernels), kern


@pytest.mark.parametrize("shape,env,kernels", [s for s in SHAPES if s[0] in ("gpf", "stage_g8_wgf5")],
                         ids=["gpf", "stage_g8_wgf5"])
@pytest.mark.parametrize("name,rule,fold", pc.RULE_CASES)
def test_kernel_shape_rules(ctx, monkeypatch, shape, env, kernels, name, rule, fold):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg = pc.get(name)
    _check(ctx, cfg, 42, _iters(cfg), rule, fold)


@pytest.mark.parametrize("plen", [57000, 60000, 65000])
def test_huge_frames(ctx, plen):
    """The longest frames: up to ~57 KB still fit the LDS stage; longer ones fall
    back to the group-per-frame kernel.  Bit-exact either way."""
    cfg = copy.deepcopy(pc.get("c2_udp_1500"))
    cfg["payloads"] = [{"length": {"min": plen, "max": plen}}]
    kern = _check(ctx, cfg, 7, 96)
    assert kern.startswith(("pb_vstage_kernel", "pb_stage_kernel") if plen < 58000 else "pb_gpf_kernel"), kern
    cfg["payloads"] = [{"length": {"min": 30000, "max": plen}}]
    kern = _check(ctx, cfg, 7, 96)
    assert kern.startswith("pb_gpf_kernel"), kern


# Small frames: lengths dividing 4096 (64, 128 B) take pb_xsmall_kernel (4 KiB
# pages owned per XCD), other multiples of 4 pb_xpage_kernel (the same pages, frames
# cut at page edges built by both owners), the rest pb_small_kernel.  Frame lengths 42..128 B
# cover every LDS placement mode (16-B, 8-B, 4-B and byte-aligned frames); the
# frame counts hit < 1 page, exactly 32 pages (one full group of 8 workgroups),
# one frame past it, and a ragged tail after several full groups.
XS_LENS = [42, 43, 44, 48, 52, 56, 60, 64, 72, 96, 98, 100, 106, 108, 116, 120, 124, 127, 128]
XS_COUNTS = [1, 5, 200, 2048, 2049, 2 * 2048 * 5 + 77]


@pytest.mark.parametrize("force_xpage", [False, True, 512, "lin64", "lin128", "fa64", "img"],
                         ids=["default", "xpage_forced", "xpage_forced_512", "linear_wg64", "linear_wg128",
                              "xpage_forced_fa64", "ximg_single_builds"])
@pytest.mark.parametrize("proto", ["udp", "tcp", "icmp"])
@pytest.mark.parametrize("flen", XS_LENS)
def test_small_frames_pages(ctx, monkeypatch, proto, flen, force_xpage):
    if force_xpage == "fa64":  # pb_xpage_kernel's 64-bit first-frame path at every size
        monkeypatch.setenv("PBGPU_XP_FA64", "1")
    solo = force_xpage == "img"  # static-payload ICMP frames on pb_ximg_kernel in single builds too
    if solo:
        monkeypatch.setenv("PBGPU_XP_IMG", "2")
        force_xpage = False
    if force_xpage:
        monkeypatch.setenv("PBGPU_XP_FORCE", "1")
    if force_xpage == 512:
        monkeypatch.setenv("PBGPU_XP_WGT", "512")
    elif force_xpage is True:  # the 256-thread form (two passes of slots per lane)
        monkeypatch.setenv("PBGPU_XP_WGT", "256")
    lin = force_xpage in ("lin64", "lin128")
    if lin:  # the linear small kernel at 64 / 128 frames per workgroup, for every length
        monkeypatch.delenv("PBGPU_XP_FORCE", raising=False)
        monkeypatch.setenv("PBGPU_KERNEL", "linear")
        monkeypatch.setenv("PBGPU_SMALL_WGT", force_xpage[3:])
    hl = 54 if proto == "tcp" else 42
    if flen < hl or (proto == "icmp" and flen == hl):
        pytest.skip("shorter than the headers / empty static payload")
    cfg = copy.deepcopy(pc.get({"udp": "c2_udp_64", "tcp": "c4_tcp_syn", "icmp": "c5_icmp_echo"}[proto]))
    if proto == "icmp":  # static payload
        cfg["payloads"] = [{"exact": " ".join("%02X" % (i * 7 & 255) for i in range(flen - hl))}]
    else:
        cfg["payloads"] = [{"length": {"min": flen - hl, "max": flen - hl}}]
    for n in XS_COUNTS:
        n = max(1, n * 64 // flen)  # page counts as named above at every length
        kern = _check(ctx, cfg, 1000003 + n, n)
        # pbgpu_load_sequence: 52-64 B multiples of 4; static payloads at even 52-128 B
        xp_default = 52 <= flen <= 64 and flen % 4 == 0 or (proto == "icmp" and 52 <= flen <= 128)
        # pb_ximg_kernel (PBGPU_XP_IMG=2): static-payload ICMP frames on the page kernel's pages
        img = proto == "icmp" and flen % 2 == 0 and solo and 4096 % flen and xp_default
        if lin:
            want = "pb_small_kernel<"
        elif img:
            want = "pb_ximg_kernel"
        elif flen % 2 == 0 and (force_xpage or (4096 % flen and xp_default)):
            want = "pb_xpage_kernel"
        else:
            want = "pb_xsmall_kernel" if 4096 % flen == 0 else "pb_small_kernel<"
        assert kern.startswith(want), kern


# pb_fstage_kernel: frame lengths (multiples of 4) that start frames at every
# dword offset of a 16-B chunk and end them at every one, for each protocol,
# with and without checksums; frame counts that leave a ragged last window and
# a ragged last workgroup.
FST_LENS = [132, 148, 256, 1000, 1500, 1508, 2052, 4096]
FST_COUNTS = [1, 15, 17, 64, 65, 333, 1027]


def _fst_cfg(proto, flen, csum=True):
    hl = 54 if proto == "tcp" else 42
    cfg = copy.deepcopy(pc.get({"udp": "c2_udp_1500", "tcp": "c4_tcp_syn", "icmp": "c5_icmp_echo"}[proto]))
    cfg["payloads"] = [{"length": {"min": flen - hl, "max": flen - hl}}]
    if not csum:
        cfg["l4csum"] = 0
    return cfg


@pytest.mark.parametrize("shape,env", FST_SHAPES, ids=[s[0] for s in FST_SHAPES])
@pytest.mark.parametrize("proto", ["udp", "tcp", "icmp"])
@pytest.mark.parametrize("flen", FST_LENS)
def test_fstage_frames(ctx, monkeypatch, shape, env, proto, flen):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cfg = _fst_cfg(proto, flen)
    for n in FST_COUNTS:
        if n * flen > (8 << 20):
            continue
        kern = _check(ctx, cfg, 77 + 3 * n, n)
        if _fst_fits(env, flen):
            assert kern.startswith("pb_fstage_kernel<%s" % env.get("PBGPU_FST_G", "")), kern


def _fst_fits(env, flen):
    """Whether a forced shape fits 64 KiB of LDS (else the library takes pb_stage_kernel)."""
    if "PBGPU_FST_G" not in env:
        return True  # the default picks a shape that fits
    g = int(env["PBGPU_FST_G"])
    nbs = [int(env["PBGPU_FST_NBUF"])] if "PBGPU_FST_NBUF" in env else [1, 2]
    ngw = 256 // g
    wgf = max(ngw, min(256, int(env.get("PBGPU_FST_WGF", 64)) // ngw * ngw))
    return any(nb * ((ngw * flen + 15) // 16 * 16) + wgf * 72 <= 65536 for nb in nbs)


@pytest.mark.parametrize("flen", [132, 1500, 1508])
def test_fstage_no_l4_csum(ctx, flen):
    for proto in ("udp", "tcp", "icmp"):
        cfg = _fst_cfg(proto, flen, csum=False)
        kern = _check(ctx, cfg, 5, 1027)
        assert kern.startswith("pb_fstage_kernel<") and kern.endswith(", 0>"), kern


def test_fstage_not_for_other_shapes(ctx, monkeypatch):
    """Lengths not a multiple of 4 take pb_vstage_kernel, the literal rule keeps
    pb_stage_kernel; PBGPU_KERNEL=stage forces it."""
    cfg = _fst_cfg("udp", 1502)
    assert _check(ctx, cfg, 9, 100).startswith("pb_vstage_kernel"), "odd dword"
    cfg = _fst_cfg("udp", 1500)
    assert _check(ctx, cfg, 9, 100, rule=1).startswith("pb_stage_kernel"), "literal rule"
    monkeypatch.setenv("PBGPU_KERNEL", "stage")
    assert _check(ctx, cfg, 9, 100).startswith("pb_stage_kernel"), "forced"


# pb_vstage_kernel on fixed lengths that are not a multiple of 4 (frames start at
# every byte offset of a chunk), with and without L4 checksums
VST_LENS = [129, 130, 131, 133, 1501, 1502, 1503, 4097]


@pytest.mark.parametrize("proto", ["udp", "tcp", "icmp"])
@pytest.mark.parametrize("flen", VST_LENS)
def test_vstage_fixed_odd_lengths(ctx, proto, flen):
    for csum in (True, False):
        cfg = _fst_cfg(proto, flen, csum)
        for n in (1, 7, 33, 129, 1031):
            kern = _check(ctx, cfg, 3 + n, n)
            assert kern.startswith("pb_vstage_kernel<"), kern


@pytest.mark.parametrize("lo,hi", [(0, 1), (0, 5), (0, 40), (60, 1500), (1400, 1500), (0, 3000)])
@pytest.mark.parametrize("proto", ["udp", "tcp", "icmp"])
def test_vstage_variable_lengths(ctx, monkeypatch, proto, lo, hi):
    """Packed variable frames from header-only (frames sharing chunks on both
    sides, empty payloads) to 3 KB."""
    monkeypatch.setenv("PBGPU_KERNEL", "vstage")
    hl = 54 if proto == "tcp" else 42
    cfg = _fst_cfg(proto, hl + 100)
    cfg["payloads"] = [{"length": {"min": lo, "max": hi}}]
    n = max(64, min(6000, (6 << 20) // (hl + hi + 1)))
    kern = _check(ctx, cfg, 11, n)
    assert kern.startswith("pb_vstage_kernel<"), kern


@pytest.mark.parametrize("pls", [
    [{"length": {"min": 10, "max": 50}}, {"length": {"min": 100, "max": 200}}],
    [{"length": {"min": 1458, "max": 1458}}, {"length": {"min": 1458, "max": 1458}}],
    [{"length": {"min": 0, "max": 3}}, {"length": {"min": 7, "max": 7}}, {"length": {"min": 500, "max": 1400}}],
], ids=["two_var", "two_fixed_1500", "three_mixed_lengths"])
@pytest.mark.parametrize("proto", ["udp", "tcp"])
@pytest.mark.parametrize("kernel", ["default", "vstage"])
def test_multi_random_payloads(ctx, monkeypatch, proto, pls, kernel):
    """Several random payloads per iteration (one frame each, later payloads drawn
    from the advanced seed, sequence.c:529-561): packed variable frames through
    pb_vline_kernel (every payload >= 32 B) or pb_vstage_kernel, bit-exact against
    the oracle."""
    if kernel == "vstage":
        monkeypatch.setenv("PBGPU_KERNEL", "vstage")
    cfg = _fst_cfg(proto, 200)
    cfg["payloads"] = pls
    kern = _check(ctx, cfg, 31, 1500)
    vl = kernel == "default" and min(p["length"]["min"] for p in pls) >= 32
    assert kern.startswith("pb_vline_kernel<" if vl else "pb_vstage_kernel<"), kern


# pb_vline_kernel: packed variable frames with payloads of >= 32 B (two frame starts in one
# 128-B line at 32-40 B), up to 4096-B frames, every protocol, with and without the L4
# checksum; frame counts that leave ragged workgroups and single-frame launches
VL_RANGES = [(32, 33), (32, 40), (32, 200), (60, 1500), (64, 1500), (1400, 1500), (500, 4000), (3000, 4042)]


@pytest.mark.parametrize("lo,hi", VL_RANGES)
@pytest.mark.parametrize("proto", ["udp", "tcp", "icmp"])
@pytest.mark.parametrize("csum", [True, False])
@pytest.mark.parametrize("kernel", ["vpage", "vline"])
def test_vline_variable_lengths(ctx, monkeypatch, proto, lo, hi, csum, kernel):
    """pb_vline_kernel (the default) and pb_vpage_kernel (PBGPU_KERNEL=vpage: up to 57 frames per
    page at 74 B, frames up to 4 KiB starting up to a page before the page)."""
    if kernel == "vpage":
        monkeypatch.setenv("PBGPU_KERNEL", "vpage")
    hl = 54 if proto == "tcp" else 42
    cfg = _fst_cfg(proto, hl + 100, csum)
    cfg["payloads"] = [{"length": {"min": lo, "max": hi}}]
    big = max(300, min(40000, (24 << 20) // (hl + hi)))
    for first, n in ((5, 1), (0, 3), (11, 253), (2 ** 40 + 7, 1000), (1, big)):
        kern = _check(ctx, cfg, first, n)
        assert kern.startswith("pb_%s_kernel<%d, %d>" % (kernel, hl, int(csum))), kern


@pytest.mark.parametrize("wgf", ["32", "100", "252"])
def test_vline_workgroup_sizes(ctx, monkeypatch, wgf):
    """Own frames per workgroup (PBGPU_VL_WGF): every region split and ghost count."""
    monkeypatch.setenv("PBGPU_VL_WGF", wgf)
    for lo, hi in ((32, 33), (64, 1500)):
        cfg = pc.get("c3_udp_var")
        cfg["payloads"] = [{"length": {"min": lo, "max": hi}}]
        kern = _check(ctx, cfg, 77, 20011)
        assert kern.startswith("pb_vline_kernel<"), kern


def test_vline_offsets_across_4gib_boundaries(ctx, monkeypatch):
    """pb_vline_kernel keeps each frame's offset as its low 32 bits plus its region's 64-bit
    start (pb_expand_offsets rebuilds offset = rstart + (u32)(low - (u32)rstart)): a build of
    2^23 configs[2] frames (~6.9 GB) crosses 2^32, so the offsets must equal
    pb_vstage_kernel's 64-bit ones everywhere, and the frames around each 2^32 multiple must
    be the oracle's bytes at the oracle's offsets."""
    seq = Sequence.from_config(pc.get("c3_udp_var"))
    n, first = 1 << 23, 12345
    offs, data = {}, {}
    for kernel in ("vline", "vpage", "vstage"):
        if kernel != "vline":
            monkeypatch.setenv("PBGPU_KERNEL", kernel)
        ctx.load_sequence(6, seq, pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(6, n))
        ctx.build(6, first, n, fb)
        ctx.sync()
        offs[kernel] = fb.offsets()
        assert ctx.kernel_name(6).startswith("pb_%s_kernel" % kernel)
        if kernel != "vstage":
            data[kernel] = fb.packed()
        fb.free()
    o = offs["vpage"]
    assert o[-1] > (1 << 32)  # the build crosses a 4-GiB boundary
    assert np.array_equal(o, offs["vstage"]) and np.array_equal(o, offs["vline"])
    assert np.array_equal(data["vpage"], data["vline"])
    for k in range(1, int(o[-1] >> 32) + 1):
        f = int(np.searchsorted(o, k << 32, side="right")) - 1  # the frame holding byte k * 2^32
        f0 = max(0, f - 16)
        od, oo = ob.build(seq, 6, first + f0, 32, pc.SEED_BASE)
        assert np.array_equal(o[f0:f0 + 33] - o[f0], oo), k
        assert np.array_equal(data["vpage"][int(o[f0]):int(o[f0 + 32])], od), k


def test_vline_matches_vstage_at_size(ctx, monkeypatch):
    """configs[2] at 2^22 frames: the three variable-length kernels build the same bytes."""
    seq = Sequence.from_config(pc.get("c3_udp_var"))
    out = {}
    for kernel in ("vline", "vpage", "vstage"):
        if kernel != "vline":
            monkeypatch.setenv("PBGPU_KERNEL", kernel)
        ctx.load_sequence(6, seq, pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(6, 1 << 22))
        ctx.build(6, 3 << 30, 1 << 22, fb)
        ctx.sync()
        out[kernel] = (fb.packed(), fb.offsets(), ctx.kernel_name(6))
        fb.free()
    for kernel in out:
        assert out[kernel][2].startswith("pb_%s_kernel" % kernel)
    for kernel in ("vline", "vstage"):
        assert np.array_equal(out["vpage"][1], out[kernel][1])
        assert np.array_equal(out["vpage"][0], out[kernel][0])


@pytest.mark.parametrize("pct", ["1", "30", "100"])
def test_vpage_short_grid_waves_take_several_pages(ctx, monkeypatch, pct):
    """pb_vpage_kernel's grid covers the expected stream; a longer one is built by the same waves
    in later rounds (PBGPU_VP_PAGES_PCT shrinks the grid so every wave loops): bit-exact."""
    monkeypatch.setenv("PBGPU_KERNEL", "vpage")
    monkeypatch.setenv("PBGPU_VP_PAGES_PCT", pct)
    for lo, hi in ((32, 33), (64, 1500), (3000, 4042)):
        cfg = pc.get("c3_udp_var")
        cfg["payloads"] = [{"length": {"min": lo, "max": hi}}]
        kern = _check(ctx, cfg, 99, 30011)
        assert kern.startswith("pb_vpage_kernel<"), kern
