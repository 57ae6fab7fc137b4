"""Oracle pinning (CPU, no GPU): the restatement is checked against what the
reference's environment itself provides — glibc rand_r, the two known-answer
frames of images/test1.gif — and against an independent RFC verifier."""
import ctypes
import ctypes.util
import json
import os
import random
import struct

import numpy as np
import pytest

import oracle_binding as ob
import pyverify as pv
from pbgpu import Sequence

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_rand_r_matches_host_glibc():
    """pbo_rand_r == the libc rand_r the reference links (sequence.c:554)."""
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.rand_r.restype = ctypes.c_int
    libc.rand_r.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    rng = random.Random(1234)
    seeds = [0, 1, 2, 0xFFFFFFFF, 0x80000000, 12345] + [rng.getrandbits(32) for _ in range(200)]
    for s0 in seeds:
        a = ctypes.c_uint(s0)
        b = s0
        for _ in range(8):
            ra = libc.rand_r(ctypes.byref(a))
            rb, b = ob.rand_r(b)
            assert ra == rb
            assert a.value == b


def test_seed_stream_is_splitmix64():
    def splitmix(x):
        z = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return z ^ (z >> 31)

    for base, seq, k in [(0x5EEDBA5E, 0, 0), (0x5EEDBA5E, 3, 12345), (0, 255, 2**40), (2**63 + 5, 1, 7)]:
        assert ob.seed(base, seq, k) == splitmix(base ^ (((seq << 48) + k) & (2**64 - 1))) & 0xFFFFFFFF


def kat_cases():
    with open(os.path.join(GOLD, "kat_test1_gif.json")) as f:
        kat = json.load(f)
    for fr in kat["frames"]:
        cfg = json.loads(json.dumps(kat["config"]))
        cfg["udp"]["sport"] = fr["sport"]
        yield cfg, bytes.fromhex(fr["hex"].replace(" ", ""))


@pytest.mark.parametrize("faithful", [False, True])
def test_known_answer_frames_from_reference_gif(faithful):
    """The two receiver-captured frames (udp sum ok) are reproduced byte for byte:
    pins the IPv4 header checksum and the UDP pseudo-header checksum composition."""
    n = 0
    for cfg, want in kat_cases():
        seq = Sequence.from_config(cfg)
        got = ob.frames(seq, 0, 0, 3, 0x5EEDBA5E, faithful=faithful)
        for g in got:  # static everything: every iteration equals the capture
            assert g == want
        n += 1
    assert n == 2


def test_kat_frames_verify_independently():
    for _, want in kat_cases():
        assert pv.ip_csum_ok(want)
        assert pv.l4_csum_value(want) == pv.parse(want)["l4_csum"]


def test_checksum_helpers_vs_rfc1071():
    rng = np.random.default_rng(7)
    for _ in range(300):
        hdr = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
        hdr[10:12] = b"\0\0"
        c = ob.lib().pbo_iph_csum(bytes(hdr), 0)
        assert struct.pack("<H", c) == struct.pack("!H", pv.inet_csum(bytes(hdr)))
        ln = int(rng.integers(8, 200))
        l4 = bytearray(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
        sa, da = rng.integers(0, 2**32, 2, dtype=np.uint64)
        for proto in (17, 6, 1):
            l4c = bytearray(l4)
            ck = ob.lib().pbo_l4_csum(bytes(l4c), ln, int(sa), int(da), proto)
            if proto == 1:
                want = pv.inet_csum(bytes(l4c))
            else:
                pseudo = struct.pack("<I", int(sa)) + struct.pack("<I", int(da)) + struct.pack("!BBH", 0, proto, ln)
                want = pv.inet_csum(pseudo + bytes(l4c))
            assert struct.pack("<H", ck) == struct.pack("!H", want)


def test_single_fold_differs_only_on_carry():
    """B6: the single-fold IPv4 variant equals the full fold unless the first fold carries."""
    rng = np.random.default_rng(11)
    diff = 0
    for _ in range(20000):
        h = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
        h[10:12] = b"\0\0"
        a = ob.lib().pbo_iph_csum(bytes(h), 0)
        b = ob.lib().pbo_iph_csum(bytes(h), 1)
        s = sum(struct.unpack("<10H", bytes(h)))
        carry = (s & 0xFFFF) + (s >> 16) > 0xFFFF
        assert (a != b) == carry
        diff += a != b
    # a header that forces the carry: five 0xFFFF words + 1 -> s = 0x4FFFC
    h = struct.pack("<10H", 0xFFFF, 0xFFFF, 0xFFFF, 0xFFFF, 0xFFFF, 0, 1, 0, 0, 0)
    a = ob.lib().pbo_iph_csum(h, 0)
    b = ob.lib().pbo_iph_csum(h, 1)
    assert a != b and a == struct.unpack("<H", struct.pack("!H", pv.inet_csum(h)))[0]


def test_frame_checker_on_reference_kats_and_oracle_frames():
    """pbo_verify_frames (the full-size GPU tests' checker) accepts the reference's captured
    frames and every BASELINE / edge config's oracle frames that carry both checksums, and
    rejects a frame with one flipped bit in the IPv4 header, the L4 header or the payload."""
    import pb_configs as pc

    for _, want in kat_cases():
        a = np.frombuffer(want, dtype=np.uint8).copy()
        assert ob.verify_frames(a, None, len(want), 1, 1) == 0
    for name in pc.ALL:
        cfg = pc.get(name)
        if cfg.get("l4csum", 1) == 0 or cfg["ip"].get("csum", 1) == 0 or "jumbo" in name:
            continue
        seq = Sequence.from_config(cfg)
        data, off = ob.build(seq, 0, 0, 300, pc.SEED_BASE)
        n = len(off) - 1
        assert ob.verify_frames(data, off, 0, n, 4) == 0, name
        for pos in (16, 24, 36, int(off[1]) - 1):  # tot_len, IPv4 csum, L4 header, last byte of frame 0
            bad = data.copy()
            bad[pos] ^= 0x10
            assert ob.verify_frames(bad, off, 0, n, 4) == 1, (name, pos)
