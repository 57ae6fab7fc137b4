"""The C host's JSON config reader (host/config_json.c, in place of PB-Common's
parse_config, src/main.c:94) and MAC discovery (host/mac.c, the reference's
get_src_mac_address / get_gw_mac, src/sequence.c:111-130).

The JSON reader must fill pb_sequence_t exactly as the Python loader
(Sequence.from_config, README.md:216-575 schema) does, over the same
clear_sequence() defaults; both are this build's restatements of an
un-vendored PB-Common function, so they are checked against each other and
against hand-written expectations for the README's examples."""
import ctypes as C
import json
import os
import subprocess

import pytest

import pb_configs as pc
from pbgpu import MAX_PAYLOADS, MAX_RANGES, SequenceT, Sequence

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTLIB = os.path.join(ROOT, "pb-af-xdp_amd", "lib", "libpbhost.so")
BIN = os.path.join(ROOT, "pb-af-xdp_amd", "bin", "pcktbatch-gpu")
MAX_SEQUENCES = 256


class ConfigT(C.Structure):
    """pb_config_t (include/pb_config.h)."""

    _fields_ = [("interface", C.c_char_p), ("seq", SequenceT * MAX_SEQUENCES)]


@pytest.fixture(scope="module")
def lib():
    lib = C.CDLL(HOSTLIB)
    lib.pb_parse_config_text.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(ConfigT), C.POINTER(C.c_int),
                                         C.POINTER(C.c_char_p)]
    lib.pb_parse_config.argtypes = [C.c_char_p, C.POINTER(ConfigT), C.POINTER(C.c_int), C.c_int]
    lib.pb_get_gw_mac_from.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p]
    lib.pb_get_src_mac_from.argtypes = [C.c_char_p, C.c_char_p]
    lib.pb_get_src_mac_address.argtypes = [C.c_char_p, C.c_char_p]
    return lib


def defaults():
    cfg = ConfigT()
    for i in range(MAX_SEQUENCES):
        s = cfg.seq[i]
        s.block, s.delay, s.l4_csum = 1, 1000000, 1
        s.ip.csum, s.ip.min_ttl, s.ip.max_ttl, s.ip.max_id = 1, 64, 64, 64000
    return cfg


def parse(lib, text):
    cfg, n, err = defaults(), C.c_int(-1), C.c_char_p()
    raw = text.encode()
    rc = lib.pb_parse_config_text(raw, len(raw), C.byref(cfg), C.byref(n), C.byref(err))
    return rc, cfg, n.value, (err.value.decode() if err.value else None)


def as_dict(s):
    """Every field of a pb_sequence_t as plain values."""
    st = lambda b: b.decode() if b else None  # noqa: E731
    d = {k: getattr(s, k) for k in ("block", "track", "max_pckts", "max_bytes", "pps", "bps", "time", "threads",
                                    "delay", "l4_csum", "pl_cnt")}
    d["interface"] = st(s.interface)
    d["eth"] = (st(s.eth.src_mac), st(s.eth.dst_mac))
    ip = s.ip
    d["ip"] = (st(ip.src_ip), st(ip.dst_ip), st(ip.protocol), ip.tos, ip.csum, ip.min_ttl, ip.max_ttl, ip.min_id,
               ip.max_id, tuple(st(ip.ranges[i]) for i in range(ip.range_count)))
    d["udp"] = (s.udp.src_port, s.udp.dst_port)
    d["tcp"] = tuple(getattr(s.tcp, n) for n, _ in s.tcp._fields_)
    d["icmp"] = (s.icmp.code, s.icmp.type)
    d["pls"] = tuple((st(p.exact), p.is_static, p.is_file, p.is_string, p.min_len, p.max_len)
                     for p in s.pls[:s.pl_cnt])
    return d


@pytest.mark.parametrize("name", list(pc.ALL))
def test_json_config_matches_python_loader(lib, name):
    seq = pc.get(name)
    text = json.dumps({"interface": "ens1", "sequences": [seq, pc.get("c4_tcp_syn")]}, indent=2)
    rc, cfg, n, err = parse(lib, text)
    assert rc == 0, err
    assert n == 2 and cfg.interface == b"ens1"
    assert as_dict(cfg.seq[0]) == as_dict(Sequence.from_config(seq).c)
    assert as_dict(cfg.seq[1]) == as_dict(Sequence.from_config(pc.get("c4_tcp_syn")).c)
    assert as_dict(cfg.seq[2]) == as_dict(defaults().seq[2])  # untouched


def test_json_readme_example_and_value_forms(lib):
    """README.md:244-262 style sequence; booleans as true/false or 0/1, 64-bit
    integers exact, string escapes, repeated keys (last wins)."""
    text = r'''{
      "interface": "dev",
      "sequences": [{
        "interface": "dev2", "block": false, "track": true, "time": 20, "delay": 100000,
        "maxpckts": 18446744073709551615, "maxbytes": 1e3, "pps": 300, "threads": 4, "l4csum": 0,
        "eth": {"smac": "1a:c4:df:70:d8:a6", "dmac": "ae:21:14:4b:3a:6d"},
        "ip": {"sip": null, "dip": "10.50.0.4", "protocol": "TCP", "tos": 16, "csum": false,
               "ttl": {"min": 32, "max": 128}, "id": {"min": 1, "max": 9},
               "ranges": ["10.0.0.0/8", "192.168.1.0/24"]},
        "tcp": {"sport": 1234, "dport": 80, "syn": true, "ack": 1, "psh": 0, "urg": true},
        "udp": {"sport": 1, "sport": 53},
        "icmp": {"code": 3, "type": 8},
        "payloads": [{"exact": "FF FF", "isstatic": true},
                     {"exact": "tab\there \"q\" é", "isstring": true},
                     {"length": {"min": 10, "max": 1400}}]
      }]
    }'''
    rc, cfg, n, err = parse(lib, text)
    assert rc == 0, err
    s = cfg.seq[0]
    assert n == 1 and cfg.interface == b"dev" and s.interface == b"dev2"
    assert (s.block, s.track, s.time, s.delay, s.threads, s.l4_csum) == (0, 1, 20, 100000, 4, 0)
    assert s.max_pckts == (1 << 64) - 1 and s.max_bytes == 1000 and s.pps == 300
    assert (s.eth.src_mac, s.eth.dst_mac) == (b"1a:c4:df:70:d8:a6", b"ae:21:14:4b:3a:6d")
    assert s.ip.src_ip is None and s.ip.dst_ip == b"10.50.0.4" and s.ip.protocol == b"TCP"
    assert (s.ip.tos, s.ip.csum, s.ip.min_ttl, s.ip.max_ttl, s.ip.min_id, s.ip.max_id) == (16, 0, 32, 128, 1, 9)
    assert [s.ip.ranges[i] for i in range(s.ip.range_count)] == [b"10.0.0.0/8", b"192.168.1.0/24"]
    assert (s.tcp.src_port, s.tcp.dst_port, s.tcp.syn, s.tcp.ack, s.tcp.psh, s.tcp.urg) == (1234, 80, 1, 1, 0, 1)
    assert s.udp.src_port == 53 and (s.icmp.code, s.icmp.type) == (3, 8)
    assert s.pl_cnt == 3
    assert (s.pls[0].exact, s.pls[0].is_static) == (b"FF FF", 1)
    assert s.pls[1].exact == 'tab\there "q" é'.encode() and s.pls[1].is_string == 1
    assert (s.pls[2].exact, s.pls[2].min_len, s.pls[2].max_len) == (None, 10, 1400)


@pytest.mark.parametrize("text", ["", "[]", "{", '{"sequences": [}', '{"a": tru}', '{"a": 01}', '{"a": "x\\q"}',
                                  '{"a": 1} x', '{"a": "\x01"}', '{"a" 1}'])
def test_json_syntax_errors(lib, text):
    rc, _, _, err = parse(lib, text)
    assert rc == -22 and err  # -EINVAL with a message


def test_json_limits(lib):
    too_many = json.dumps({"sequences": [{"ip": {"ranges": ["10.0.0.0/8"] * (MAX_RANGES + 1)}}]})
    assert parse(lib, too_many)[0] == -7  # -E2BIG
    too_many = json.dumps({"sequences": [{"payloads": [{}] * (MAX_PAYLOADS + 1)}]})
    assert parse(lib, too_many)[0] == -7
    rc, _, n, _ = parse(lib, json.dumps({"sequences": [{}] * (MAX_SEQUENCES + 5)}))
    assert rc == 0 and n == MAX_SEQUENCES


def test_config_file_missing(lib, tmp_path):
    cfg, n = defaults(), C.c_int()
    assert lib.pb_parse_config(str(tmp_path / "none.json").encode(), C.byref(cfg), C.byref(n), 0) == -2  # -ENOENT


def test_binary_lists_config_file(tmp_path):
    """pcktbatch-gpu -c FILE -l: the reference's list mode over the config's sequences;
    -z overrides apply to the first sequence after the file (main.c:90-103)."""
    path = tmp_path / "conf.json"
    path.write_text(json.dumps({"interface": "ens9", "sequences": [pc.get("c2_udp_64"), pc.get("c4_tcp_syn"),
                                                                    pc.get("c5_icmp_echo")]}))
    r = subprocess.run([BIN, "-c", str(path), "-l"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("Sequence #")]
    assert len(lines) == 3
    assert "10.20.0.0/16 -> %s proto udp" % pc.DIP in lines[0] and "proto tcp" in lines[1] and "proto icmp" in lines[2]
    r = subprocess.run([BIN, "-c", str(path), "-z", "--protocol", "tcp", "--dip", "10.9.9.9", "-l"],
                       capture_output=True, text=True, timeout=60)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("Sequence #")]
    assert r.returncode == 0 and len(lines) == 3 and "-> 10.9.9.9 proto tcp" in lines[0]
    r = subprocess.run([BIN, "-c", str(tmp_path / "missing.json"), "-l"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "Error opening config file" in r.stderr


def test_gateway_mac_from_route_and_arp(lib, tmp_path):
    route = tmp_path / "route"
    route.write_text(
        "Iface\tDestination\tGateway \tFlags\tRefCnt\tUse\tMetric\tMask\t\tMTU\tWindow\tIRTT\n"
        "eth0\t0000A8C0\t00000000\t0001\t0\t0\t0\t00FFFFFF\t0\t0\t0\n"
        "eth0\t00000000\t0100A8C0\t0003\t0\t0\t100\t00000000\t0\t0\t0\n")
    arp = tmp_path / "arp"
    arp.write_text(
        "IP address       HW type     Flags       HW address            Mask     Device\n"
        "192.168.0.7      0x1         0x2         11:22:33:44:55:66     *        eth0\n"
        "192.168.0.1      0x1         0x2         52:54:00:12:35:02     *        eth0\n")
    mac = C.create_string_buffer(6)
    assert lib.pb_get_gw_mac_from(str(route).encode(), str(arp).encode(), mac) == 0
    assert mac.raw == bytes.fromhex("525400123502")
    # no default route / gateway not in the neighbour table
    route.write_text("Iface\tDestination\tGateway \tFlags\n" "eth0\t0000A8C0\t00000000\t0001\n")
    assert lib.pb_get_gw_mac_from(str(route).encode(), str(arp).encode(), mac) == -2
    route.write_text("Iface\tDestination\tGateway \tFlags\n" "eth0\t00000000\t0900A8C0\t0003\n")
    assert lib.pb_get_gw_mac_from(str(route).encode(), str(arp).encode(), mac) == -2


def test_source_mac(lib, tmp_path):
    addr = tmp_path / "address"
    addr.write_text("0a:1b:2c:3d:4e:5f\n")
    mac = C.create_string_buffer(6)
    assert lib.pb_get_src_mac_from(str(addr).encode(), mac) == 0 and mac.raw == bytes.fromhex("0a1b2c3d4e5f")
    assert lib.pb_get_src_mac_address(b"no-such-dev0", mac) < 0
    assert lib.pb_get_src_mac_address(b"../etc", mac) == -22
    if os.path.exists("/sys/class/net/lo/address"):
        assert lib.pb_get_src_mac_address(b"lo", mac) == 0 and mac.raw == bytes(6)
