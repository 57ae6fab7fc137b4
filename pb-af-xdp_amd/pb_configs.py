"""The BASELINE.json workloads (configs[0..4]) and the extra parity cases, as
sequence objects in the reference's JSON schema (README.md:216-575).

SURVEY.md §8(d) fixes the concrete synthetic inputs; the destination address
and MACs are this build's choice (the survey leaves them open)."""
import copy

SEED_BASE = 0x5EEDBA5E

DMAC = "52:54:00:d5:50:54"
SMAC = "52:54:00:59:29:cc"
DIP = "10.60.0.195"


def _base(protocol="udp"):
    return {
        "interface": "eth0",
        "block": 1,
        "threads": 1,
        "delay": 0,
        "l4csum": 1,
        "eth": {"smac": SMAC, "dmac": DMAC},
        "ip": {"dip": DIP, "protocol": protocol, "csum": 1},
    }


def c1_udp_static_106():
    """configs[0]: fixed src IP/port, 64-B static payload (0x00..0x3F) -> 106-B frame."""
    c = _base()
    c["ip"]["sip"] = "10.0.0.1"
    c["udp"] = {"sport": 1234, "dport": 80}
    c["payloads"] = [{"exact": " ".join("%02X" % i for i in range(64))}]
    return c


def c1_udp_static_64():
    """configs[0], 64-B frame variant (22-B static payload)."""
    c = c1_udp_static_106()
    c["payloads"] = [{"exact": " ".join("%02X" % i for i in range(22))}]
    return c


def c2_udp_64():
    """configs[1] (the metric config): UDP 64-B frame, one /16 random source,
    random source port, 22-B random payload, TTL 64, ID 0..64000, both checksums."""
    c = _base()
    c["ip"]["ranges"] = ["10.20.0.0/16"]
    c["udp"] = {"sport": 0, "dport": 27015}
    c["payloads"] = [{"length": {"min": 22, "max": 22}}]
    return c


def c2_udp_1500():
    """configs[1], 1500-B frame variant (1458-B random payload)."""
    c = c2_udp_64()
    c["payloads"] = [{"length": {"min": 1458, "max": 1458}}]
    return c


def c3_udp_var():
    """configs[2]: random payload length 64..1500 -> 106..1542-B frames, packed."""
    c = c2_udp_64()
    c["payloads"] = [{"length": {"min": 64, "max": 1500}}]
    return c


def c4_tcp_syn():
    """configs[3]: TCP SYN 60-B frame (54-B headers + 6-B random payload),
    4 CIDR ranges, random source port, dport 80, TCP checksum."""
    c = _base("tcp")
    c["ip"]["ranges"] = ["10.1.0.0/16", "10.2.0.0/16", "172.16.0.0/12", "192.168.0.0/24"]
    c["tcp"] = {"sport": 0, "dport": 80, "syn": 1}
    c["payloads"] = [{"length": {"min": 6, "max": 6}}]
    return c


def c5_icmp_echo():
    """configs[4] third sequence: ICMP echo request, 56-B static payload -> 98-B frame."""
    c = _base("icmp")
    c["ip"]["ranges"] = ["10.20.0.0/16"]
    c["icmp"] = {"type": 8, "code": 0}
    c["payloads"] = [{"exact": " ".join("%02x" % ((i * 7 + 3) & 0xFF) for i in range(56))}]
    return c


def c5_mix():
    """configs[4]: three sequences (UDP 64 B, TCP SYN 60 B, ICMP 98 B)."""
    return [c2_udp_64(), c4_tcp_syn(), c5_icmp_echo()]


BASELINE = {
    "c1_udp_static_106": c1_udp_static_106,
    "c1_udp_static_64": c1_udp_static_64,
    "c2_udp_64": c2_udp_64,
    "c2_udp_1500": c2_udp_1500,
    "c3_udp_var": c3_udp_var,
    "c4_tcp_syn": c4_tcp_syn,
    "c5_icmp_echo": c5_icmp_echo,
}


def _edge_cases():
    e = {}
    c = c2_udp_64()
    c["ip"]["ttl"] = {"min": 10, "max": 200}
    c["ip"]["id"] = {"min": 100, "max": 9000}
    c["ip"]["tos"] = 0x2E
    e["udp_rnd_ttl_id_tos"] = c

    c = c2_udp_64()
    c["ip"]["ranges"] = ["0.0.0.0/0", "10.9.8.7/32", "bogus", "10.0.0.0", "192.168.7.0/33", "172.16.5.4/20"]
    e["udp_range_edges"] = c

    c = c2_udp_64()
    del c["ip"]["ranges"]
    e["udp_no_src_localhost"] = c

    c = c2_udp_64()
    c["udp"] = {"sport": 0, "dport": 0}
    c["payloads"] = [{"length": {"min": 0, "max": 33}}]
    e["udp_both_ports_rnd_var_small"] = c

    c = c2_udp_64()
    c["payloads"] = [{"length": {"min": 1, "max": 1}}]
    e["udp_payload_1"] = c

    c = c2_udp_64()
    c["payloads"] = []
    e["udp_no_payload"] = c

    c = c2_udp_64()
    c["l4csum"] = 0
    c["ip"]["csum"] = 0
    e["udp_no_csums"] = c

    c = c4_tcp_syn()
    c["tcp"] = {"sport": 0, "dport": 0, "syn": 1, "ack": 1, "psh": 1, "fin": 1, "rst": 1, "urg": 1, "ece": 1,
                "cwr": 1}
    c["payloads"] = [{"length": {"min": 0, "max": 777}}]
    e["tcp_all_flags_var"] = c

    c = c5_icmp_echo()
    c["payloads"] = [{"length": {"min": 0, "max": 301}}]
    c["icmp"] = {"type": 13, "code": 5}
    e["icmp_rnd_var"] = c

    c = c2_udp_64()
    c["payloads"] = [{"exact": "de ad be ef 0G 1"}, {"length": {"min": 3, "max": 97}},
                     {"isstatic": 1, "length": {"min": 5, "max": 40}}, {"exact": "hello, world", "isstring": 1}]
    e["udp_multi_payload"] = c

    # several short payloads: under the literal rule each random one draws until the first
    # j with data_len[j] <= j (quirk B8), which these lengths make land anywhere in 0..6
    c = c2_udp_64()
    c["payloads"] = [{"length": {"min": 0, "max": 3}}, {"exact": "ab cd"}, {"length": {"min": 1, "max": 6}},
                     {"isstatic": 1, "length": {"min": 2, "max": 4}}, {"length": {"min": 0, "max": 40}},
                     {"length": {"min": 5, "max": 5}}]
    e["udp_multi_short"] = c

    c = c2_udp_64()
    c["payloads"] = [{"length": {"min": 2000, "max": 16000}}]
    e["udp_jumbo_var"] = c

    c = c2_udp_64()
    c["payloads"] = [{"length": {"min": 9001, "max": 9001}}]
    e["udp_jumbo_fixed_odd"] = c

    c = c2_udp_64()
    c["payloads"] = [{"length": {"min": 23, "max": 23}}]
    e["udp_fixed_odd_65"] = c

    c = c3_udp_var()
    c["payloads"] = [{"length": {"min": 0, "max": 1}}]
    e["udp_tiny_var"] = c
    return e


EDGE = _edge_cases()

# configs also run under the declared alternative rules
RULE_CASES = [
    ("c2_udp_64", 1, 0),           # literal payload rule
    ("c3_udp_var", 1, 0),
    ("udp_rnd_ttl_id_tos", 0, 1),  # single-fold IPv4 checksum
    ("c4_tcp_syn", 1, 1),
    ("udp_multi_payload", 1, 0),   # literal rule, several payloads (B8)
    ("udp_multi_short", 1, 0),
]


def get(name):
    if name in BASELINE:
        return BASELINE[name]()
    return copy.deepcopy(EDGE[name])


ALL = list(BASELINE) + list(EDGE)
