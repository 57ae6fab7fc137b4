"""rand_num pinned by the reference's own demo captures (README.md:23-27).

The demo build behind images/test1.gif and images/test2.gif seeded every
rand_num call with time(NULL), so the source port (one draw, sequence.c:505-527)
changes once a second and consecutive ports are rand_num(1, 65535, t) at
consecutive t.  The oracle's rand_num (min + rand_r(&seed) % (max - min + 1),
oracle/pb_oracle.c) must reproduce both chains at consecutive seconds, put the
test1 chain where the receiver's tcpdump stamps it, and the nearby forms must
not reproduce them at all.  Fixture: tests/golden/kat_gif_ports.json.
"""
import datetime
import json
import os

import numpy as np
import pytest

import oracle_binding as ob

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "kat_gif_ports.json")))

A, C = np.uint32(1103515245), np.uint32(12345)
PERIOD = 1 << 27  # rand_r reads bits 0-26 of its seed only


def _rand_r_np(s):
    """glibc rand_r, vectorised (the oracle's pbo_rand_r restated in numpy)."""
    x = s * A + C
    o = (x >> 16) & np.uint32(0x7FF)
    x = x * A + C
    o = (o << 10) ^ ((x >> 16) & np.uint32(0x3FF))
    x = x * A + C
    return (o << 10) ^ ((x >> 16) & np.uint32(0x3FF))


def _chain_starts(cases, lo=0, hi=PERIOD):
    """cases: {key: (chain, form)}.  Returns {key: every t in [lo, hi) at which
    form(rand_r(t + i)) == chain[i] for all i}; rand_r is computed once."""
    hits = {k: [] for k in cases}
    step = 1 << 23
    n = max(len(c) for c, _ in cases.values())
    for base in range(lo, hi, step):
        t = np.arange(base, min(hi, base + step) + n, dtype=np.uint64).astype(np.uint32)
        r = _rand_r_np(t).astype(np.int64)
        m = min(step, hi - base)
        for key, (chain, form) in cases.items():
            v = form(r)
            cand = np.nonzero(v[:m] == chain[0])[0]
            for i in range(1, len(chain)):
                cand = cand[v[cand + i] == chain[i]]
            hits[key] += [base + int(c) for c in cand]
    return hits


@pytest.mark.parametrize("cap", ["test1", "test2"])
def test_oracle_rand_num_reproduces_the_capture(cap):
    ports = FIX[cap]["ports"]
    t0 = FIX["expected"][f"{cap}_first_second_utc"]
    got = [ob.rand_num(1, 65535, (t0 + i) & 0xFFFFFFFF) for i in range(len(ports))]
    assert got == ports
    # rand_r sees only the low 27 bits of the seed: the chain repeats every 2^27 s
    assert [ob.rand_num(1, 65535, (t0 + PERIOD + i) & 0xFFFFFFFF) for i in range(len(ports))] == ports
    # and the numpy restatement used for the search below agrees with the oracle
    t = np.arange(t0, t0 + len(ports), dtype=np.uint64).astype(np.uint32)
    assert list(1 + _rand_r_np(t).astype(np.int64) % 65535) == ports


def test_test1_chain_sits_in_the_tcpdump_second():
    t0 = FIX["expected"]["test1_first_second_utc"]
    ports = FIX["test1"]["ports"]
    for stamp in FIX["test1"]["receiver_tcpdump"]:
        t = t0 + ports.index(stamp["sport"])
        utc = datetime.datetime.fromtimestamp(t, datetime.timezone.utc)
        assert utc.date() == datetime.date(2024, 4, 22)
        assert utc.strftime("%H:%M:%S") == stamp["time"].split(".")[0]
    # test2 was recorded 144 s later on the same sender
    assert FIX["expected"]["test2_first_second_utc"] - t0 == 144


def test_the_form_is_unique_over_one_full_period():
    """Over all 2^27 seed residues (= every second of any era), only
    1 + rand_r % 65535 reproduces either chain, and exactly once per period."""
    forms = {
        "1+r%65535": lambda r: 1 + r % 65535,
        "r%65535": lambda r: r % 65535,
        "1+r%65534": lambda r: 1 + r % 65534,
        "r%65536": lambda r: r % 65536,
        "1+r%65536": lambda r: 1 + r % 65536,
    }
    cases = {(cap, name): (FIX[cap]["ports"], f) for cap in ("test1", "test2") for name, f in forms.items()}
    for (cap, name), hits in _chain_starts(cases).items():
        t0 = FIX["expected"][f"{cap}_first_second_utc"]
        if name == "1+r%65535":
            assert hits == [t0 % PERIOD], (cap, hits)
        else:
            assert hits == [], (cap, name, hits)


def test_every_rand_num_field_uses_the_pinned_form():
    """TTL, ID, range index, ports and payload length all go through rand_num
    (sequence.c:445, 451, 460, 505-525, 548): spot-check the oracle's export
    against the pinned form for their ranges."""
    rng = np.random.default_rng(5)
    for lo, hi in ((1, 65535), (0, 64000), (64, 128), (0, 3), (64, 1500), (22, 22)):
        for s in rng.integers(0, 1 << 32, size=200, dtype=np.uint64):
            r, _ = ob.rand_r(int(s))
            assert ob.rand_num(lo, hi, int(s)) == lo + r % (hi - lo + 1)
