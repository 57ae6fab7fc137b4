"""The C oracle against the independent Python restatement (tests/pyspec.py)
and the RFC verifier (tests/pyverify.py), over every BASELINE config and edge
case, both declared payload rules and both IPv4 fold variants."""
import ipaddress

import pytest

import oracle_binding as ob
import pb_configs as pc
import pyspec
import pyverify as pv
from pbgpu import Sequence

N_ITER = 24
FIRST = 1000


def cases():
    for name in pc.ALL:
        yield name, 0, 0
    for name, lit, sf in pc.RULE_CASES:
        yield name, lit, sf


@pytest.mark.parametrize("name,literal,single", list(cases()))
def test_oracle_equals_pyspec(name, literal, single):
    cfg = pc.get(name)
    seq = Sequence.from_config(cfg)
    want = pyspec.build(cfg, 2, FIRST, N_ITER, pc.SEED_BASE, literal=bool(literal), single_fold=bool(single))
    lean = ob.frames(seq, 2, FIRST, N_ITER, pc.SEED_BASE, payload_rule=literal, iph_fold=single)
    faithful = ob.frames(seq, 2, FIRST, N_ITER, pc.SEED_BASE, payload_rule=literal, iph_fold=single, faithful=True)
    assert len(want) == len(lean) == len(faithful)
    for i, (w, a, b) in enumerate(zip(want, lean, faithful)):
        assert a == w, f"{name} frame {i}"
        assert b == w, f"{name} frame {i} (faithful)"


@pytest.mark.parametrize("name", pc.ALL)
def test_oracle_frames_are_valid_packets(name):
    """Field-range and checksum properties (sequence.c:443-602) on 200 iterations."""
    cfg = pc.get(name)
    seq = Sequence.from_config(cfg)
    frames = ob.frames(seq, 1, 0, 200, pc.SEED_BASE)
    ip = cfg["ip"]
    nets = [ipaddress.ip_network(r, strict=False) for r in ip.get("ranges", []) if _valid(r)]
    for fr in frames:
        d = pv.parse(fr)
        assert d["ethertype"] == 0x0800 and d["vihl"] == 0x45
        assert d["tot_len"] == len(fr) - 14
        if cfg.get("ip", {}).get("csum", 1):
            assert pv.ip_csum_ok(fr)
        else:
            assert d["ip_csum"] == 0
        if cfg.get("l4csum", 1):
            assert d["l4_csum"] == pv.l4_csum_value(fr)
        ttl = ip.get("ttl", {"min": 64, "max": 64})
        assert ttl["min"] <= d["ttl"] <= ttl["max"]
        idr = ip.get("id", {"min": 0, "max": 64000})
        assert idr["min"] <= d["id"] <= idr["max"]
        if d["proto"] in (6, 17):
            key = "udp" if d["proto"] == 17 else "tcp"
            ports = cfg.get(key, {})
            if not ports.get("sport"):
                assert 1 <= d["sport"] <= 65535
            if not ports.get("sport") and not ports.get("dport"):
                assert d["sport"] == d["dport"]  # quirk B4: one draw per iteration
            if d["proto"] == 17:
                assert d["udp_len"] == len(fr) - 34
        sa = ipaddress.ip_address(d["saddr"])
        if ip.get("sip"):
            assert str(sa) == ip["sip"]
        elif nets:
            assert any(sa in n for n in nets) or str(sa) == "127.0.0.1"
        else:
            assert str(sa) == "127.0.0.1"


def _valid(r):
    try:
        net = ipaddress.ip_network(r, strict=False)
        return "/" in r and net.prefixlen <= 32
    except ValueError:
        return False
