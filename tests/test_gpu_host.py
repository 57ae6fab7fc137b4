"""The C host driver end to end on the GPU: pcktbatch-gpu -z (the reference's
first-sequence CLI) builds frames through libpbgpu, lands them in UMEM slots
and writes them to a pcap through the TX hook; the capture must equal the
oracle's frames for the same sequence and seed stream."""
import json
import os
import struct
import subprocess

import pytest

import oracle_binding as ob
import pb_configs as pc
from pbgpu import Sequence

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "pb-af-xdp_amd", "bin", "pcktbatch-gpu")


def read_pcap(path):
    with open(path, "rb") as f:
        data = f.read()
    assert struct.unpack("<I", data[:4])[0] == 0xA1B2C3D4 and struct.unpack("<I", data[20:24])[0] == 1
    frames, pos = [], 24
    while pos < len(data):
        _, _, incl, orig = struct.unpack("<IIII", data[pos:pos + 16])
        frames.append(data[pos + 16:pos + 16 + incl])
        pos += 16 + incl
    return frames


@pytest.mark.parametrize("batch", [2000, 4096])
def test_cli_pcap_equals_oracle(tmp_path, batch):
    pcap = tmp_path / "out.pcap"
    seed = 0x1234567
    cmd = [BIN, "-z", "--interface", "eth0", "--smac", pc.SMAC, "--dmac", pc.DMAC, "--dip", pc.DIP,
           "--sip", "10.20.0.0/16", "--protocol", "udp", "--udport", "27015", "--pmin", "22", "--pmax", "22",
           "--maxpckts", "5000", "--delay", "0", "--track", "1", "--gpubatch", str(batch), "--seed", str(seed),
           "--pcap", str(pcap)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Completed 1 sequences!" in r.stdout and "total of 5000 packets" in r.stdout
    got = read_pcap(pcap)
    want = ob.frames(Sequence.from_config(pc.c2_udp_64()), 0, 0, 5000, seed)
    assert len(got) == 5000
    assert got == want


@pytest.mark.parametrize("name,args,slot,threads", [
    ("c2_udp_64", ["--protocol", "udp", "--udport", "27015", "--pmin", "22", "--pmax", "22"], 64, 1),
    ("c2_udp_64", ["--protocol", "udp", "--udport", "27015", "--pmin", "22", "--pmax", "22", "--sharedumem"], 64, 3),
    ("tcp60", ["--protocol", "tcp", "--tdport", "80", "--syn", "1", "--pmin", "6", "--pmax", "6"], 64, 1),
    ("udpvar", ["--protocol", "udp", "--udport", "27015", "--pmin", "0", "--pmax", "900"], 1024, 2),
])
def test_cli_umemslot_pcap_equals_oracle(tmp_path, name, args, slot, threads):
    """--umemslot S: frames land in S-byte slots (tight 64-B slots are written whole)
    and the TX descriptors address them; the capture taken from the UMEM at the descriptors
    equals the oracle's frames."""
    pcap = tmp_path / "slot.pcap"
    seed, n = 99, 6000
    cmd = [BIN, "-z", "--interface", "pbnodev0", "--smac", pc.SMAC, "--dmac", pc.DMAC, "--dip", pc.DIP,
           "--sip", "10.20.0.0/16"] + args + ["--maxpckts", str(n), "--delay", "0", "--gpubatch", "1000", "--seed",
                                              str(seed), "--threads", str(threads), "--umemslot", str(slot),
                                              "--pcap", str(pcap)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = read_pcap(pcap)
    cfg = pc.c2_udp_64()  # what the -z options above give
    cfg["payloads"] = [{"length": {"min": int(args[args.index("--pmin") + 1]),
                                   "max": int(args[args.index("--pmax") + 1])}}]
    if args[1] == "tcp":
        cfg["ip"]["protocol"] = "tcp"
        del cfg["udp"]
        cfg["tcp"] = {"dport": 80, "syn": 1}
    if threads == 1:
        assert got == ob.frames(Sequence.from_config(cfg), 0, 0, n, seed)
    else:
        # thread t builds iterations (step * threads + t) * 1000 + j
        assert len(got) == n and len(set(got)) == n
        assert set(got) <= set(ob.frames(Sequence.from_config(cfg), 0, 0, 3 * n, seed))


def test_cli_variable_tcp_time_limited(tmp_path):
    """No --smac on a device that does not exist: the source MAC stays zero with
    the reference's warnings (sequence.c:111-121)."""
    pcap = tmp_path / "tcp.pcap"
    cmd = [BIN, "-z", "--interface", "pbnodev0", "--dmac", pc.DMAC, "--dip", pc.DIP, "--sip", "172.16.0.0/12",
           "--protocol", "tcp", "--tdport", "80", "--syn", "1", "--pmin", "0", "--pmax", "900", "--maxpckts", "3000",
           "--delay", "0", "--gpubatch", "1000", "--seed", "7", "--pcap", str(pcap)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "WARNING - Failed to retrieve MAC address for pbnodev0." in r.stdout
    assert "WARNING - Source MAC address retrieved is 00:00:00:00:00:00." in r.stdout
    got = read_pcap(pcap)
    cfg = {"eth": {"dmac": pc.DMAC}, "ip": {"dip": pc.DIP, "ranges": ["172.16.0.0/12"], "protocol": "tcp"},
           "tcp": {"dport": 80, "syn": 1}, "payloads": [{"length": {"min": 0, "max": 900}}]}
    want = ob.frames(Sequence.from_config(cfg), 0, 0, 3000, 7)
    assert got == want


def test_json_config_sequences_equal_oracle(tmp_path):
    """pcktbatch-gpu -c conf.json: three sequences (UDP 64 B, TCP SYN, ICMP echo:
    the configs[4] mix) run in order through seq_send(); the capture is each
    sequence's oracle frames in turn (sequence index s in the seed stream)."""
    seqs = []
    for name, n in (("c2_udp_64", 3000), ("c4_tcp_syn", 2000), ("c5_icmp_echo", 1000)):
        c = dict(pc.get(name))
        c.update({"maxpckts": n, "delay": 0, "block": 1})
        seqs.append(c)
    path = tmp_path / "conf.json"
    path.write_text(json.dumps({"interface": "pbnodev0", "sequences": seqs}))
    pcap = tmp_path / "mix.pcap"
    import time

    t0 = time.perf_counter()
    r = subprocess.run([BIN, "-c", str(path), "--gpubatch", "1024", "--seed", "99", "--pcap", str(pcap)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Completed 3 sequences!" in r.stdout
    assert time.perf_counter() - t0 > 2.5  # main.c:113: a second after each sequence
    want = []
    for i, c in enumerate(seqs):
        want += ob.frames(Sequence.from_config(c), i, 0, c["maxpckts"], 99)
    assert read_pcap(pcap) == want


def test_json_config_literal_multi_payload_equals_oracle(tmp_path):
    """--literal with a sequence of six short payloads (static, exact and random):
    under the literal rule each random payload draws until the first j with
    data_len[j] <= j (quirk B8, sequence.c:545-556); the capture equals the oracle's
    frames under the same rule, six frames per iteration."""
    c = dict(pc.get("udp_multi_short"))
    c.update({"maxpckts": 6 * 700, "delay": 0, "block": 1})
    path = tmp_path / "lit.json"
    path.write_text(json.dumps({"interface": "pbnodev0", "sequences": [c]}))
    pcap = tmp_path / "lit.pcap"
    r = subprocess.run([BIN, "-c", str(path), "--gpubatch", "256", "--seed", "31", "--literal", "--pcap", str(pcap)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    want = ob.frames(Sequence.from_config(c), 0, 0, 700, 31, payload_rule=1)
    assert len(want) == 6 * 700
    assert read_pcap(pcap) == want


def test_cli_two_threads_send_distinct_iterations(tmp_path):
    """--threads 2 on one GPU (sequence.c:741: one TX thread per queue, here two
    pbgpu contexts on one GPU): the max_pckts quota is split exactly and every
    frame sent is a distinct iteration's frame of the seed stream."""
    pcap = tmp_path / "t2.pcap"
    seed = 4242
    cmd = [BIN, "-z", "--interface", "pbnodev0", "--smac", pc.SMAC, "--dmac", pc.DMAC, "--dip", pc.DIP,
           "--sip", "10.20.0.0/16", "--protocol", "udp", "--udport", "27015", "--pmin", "22", "--pmax", "22",
           "--maxpckts", "6000", "--delay", "0", "--threads", "2", "--gpubatch", "1000", "--seed", str(seed),
           "--pcap", str(pcap)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = read_pcap(pcap)
    assert len(got) == 6000 and len(set(got)) == 6000
    # thread t builds iterations (step * 2 + t) * 1000 + j: all within [0, 12000)
    universe = set(ob.frames(Sequence.from_config(pc.c2_udp_64()), 0, 0, 12000, seed))
    assert set(got) <= universe


def test_cli_null_tx_end_to_end(tmp_path):
    """Build -> land in UMEM slots -> TX descriptors on the in-memory ring, no pcap:
    the end-to-end rate of the host pipeline (DESIGN.md §6 records the numbers)."""
    import time

    n = 1 << 22
    cmd = [BIN, "-z", "--interface", "pbnodev0", "--smac", pc.SMAC, "--dmac", pc.DMAC, "--dip", pc.DIP,
           "--sip", "10.20.0.0/16", "--protocol", "udp", "--udport", "27015", "--pmin", "22", "--pmax", "22",
           "--maxpckts", str(n), "--delay", "0", "--track", "1", "--gpubatch", str(1 << 18)]
    env = dict(os.environ, PB_SEQ_GAP_MS="0")
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    dt = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr
    assert f"total of {n} packets and {64 * n} bytes" in r.stdout
    print(f"end-to-end (null TX ring, 64-B frames): {n / dt / 1e6:.1f} Mpps incl. process start")
    assert n / dt > 2e6  # sanity only: process start and GPU init are in dt (scripts/e2e_probe.py measures)


def _sent_line(seq_num, pl_idx, frame, src_ip, dst_ip):
    """The reference's verbose line for one sent frame (sequence.c:612-631), formatted from the
    oracle's bytes: the configured source (or the frame's drawn one), the UDP / TCP ports."""
    src = src_ip if src_ip else ".".join(str(b) for b in frame[26:30])
    sport = dport = 0
    if frame[23] in (6, 17):
        l4 = 14 + 4 * (frame[14] & 15)
        sport, dport = struct.unpack(">HH", frame[l4:l4 + 4])
    return "[%d][%d] Sent %d bytes of data from %s:%d to %s:%d." % (seq_num, pl_idx + 1, len(frame), src, sport, dst_ip,
                                                                     dport)


@pytest.mark.parametrize("proto,extra,cfg_l4", [
    ("udp", ["--udport", "27015", "--pmin", "0", "--pmax", "300"], {"udp": {"dport": 27015}}),
    ("tcp", ["--tdport", "80", "--syn", "1", "--pmin", "6", "--pmax", "6"], {"tcp": {"dport": 80, "syn": 1}}),
    ("icmp", ["--pmin", "10", "--pmax", "60"], {}),
])
def test_cli_verbose_sent_lines(tmp_path, proto, extra, cfg_l4):
    """pcktbatch-gpu -v prints the reference's per-packet line for every frame it submits
    (sequence.c:612-631; README.md:23 runs the demo with -v): the lines, in order, equal the
    ones formatted from the oracle's frames, and the pcap holds those frames."""
    pcap = tmp_path / "v.pcap"
    n, seed = 700, 0xABCDE
    cmd = [BIN, "-z", "-v", "--interface", "pbnodev0", "--smac", pc.SMAC, "--dmac", pc.DMAC, "--dip", pc.DIP,
           "--sip", "10.30.0.0/16", "--protocol", proto] + extra + [
           "--maxpckts", str(n), "--delay", "0", "--gpubatch", "256", "--seed", str(seed), "--pcap", str(pcap)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if " Sent " in ln]
    cfg = {"eth": {"smac": pc.SMAC, "dmac": pc.DMAC}, "ip": {"dip": pc.DIP, "ranges": ["10.30.0.0/16"], "protocol": proto},
           "payloads": [{"length": {"min": int(extra[extra.index("--pmin") + 1]),
                                    "max": int(extra[extra.index("--pmax") + 1])}}]}
    cfg.update(cfg_l4)
    want = ob.frames(Sequence.from_config(cfg), 0, 0, n, seed)
    assert read_pcap(pcap) == want
    assert lines == [_sent_line(1, 0, f, None, pc.DIP) for f in want]


def test_cli_verbose_static_source(tmp_path):
    """With a static --sip the line names the configured source string (sequence.c:630)."""
    cmd = [BIN, "-z", "-v", "--interface", "pbnodev0", "--smac", pc.SMAC, "--dmac", pc.DMAC, "--dip", pc.DIP,
           "--sip", "192.168.9.9", "--protocol", "udp", "--usport", "4000", "--udport", "27015", "--pmin", "8",
           "--pmax", "8", "--maxpckts", "50", "--delay", "0", "--gpubatch", "64", "--seed", "5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if " Sent " in ln]
    assert lines == ["[1][1] Sent 50 bytes of data from 192.168.9.9:4000 to %s:27015." % pc.DIP] * 50
