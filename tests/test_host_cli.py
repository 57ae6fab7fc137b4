"""The C host surface: this build's parse_cmd_line_af_xdp (libpbhost.so)
parses every reference command line exactly like the reference's own
src/cmd_line.c (live when oracle/_ref is built, else via the committed
fixture), and pcktbatch-gpu refuses to run without a GPU."""
import ctypes as C
import json
import os
import subprocess

import pytest

import cmdline_binding as cb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTLIB = os.path.join(ROOT, "pb-af-xdp_amd", "lib", "libpbhost.so")
REFLIB = os.path.join(ROOT, "oracle", "_ref", "libref_cmdline.so")
BIN = os.path.join(ROOT, "pb-af-xdp_amd", "bin", "pcktbatch-gpu")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "cmdline_ref.json")))


def ours():
    lib = C.CDLL(HOSTLIB)
    return lib


@pytest.mark.parametrize("case", GOLD["cases"], ids=[" ".join(c["argv"]) or "(none)" for c in GOLD["cases"]])
def test_af_xdp_options_match_reference_fixture(case):
    lib = ours()
    got = cb.parse(lib, cb.OurCmd, case["argv"])
    for n in cb.NAMES:
        assert int(getattr(got, n)) == case["fields"][n], n


@pytest.mark.skipif(not os.path.exists(REFLIB), reason="reference cmd_line.c not built here")
def test_af_xdp_options_match_reference_live():
    lib, ref = ours(), C.CDLL(REFLIB)
    for argv in cb.ARGV_CASES + [["--queue", str(q), "--batchsize", str(b)] for q in (0, 9, 65) for b in (1, 512)]:
        a = cb.parse(lib, cb.OurCmd, argv)
        b = cb.parse(ref, cb.RefCmd, argv)
        for n in cb.NAMES:
            assert int(getattr(a, n)) == int(getattr(b, n)), (argv, n)


def test_gpu_options():
    lib = ours()
    got = cb.parse(lib, cb.OurCmd, ["--gpus", "8", "--gpu", "2", "--gpubatch", "0x100000", "--seed", "42",
                                    "--literal", "--singlefold", "--pcap", "/tmp/x.pcap", "--queue", "1"],
                   defaults=lib.cmd_line_af_xdp_defaults)
    assert (got.gpus, got.gpu_first, got.gpu_batch, got.seed_base) == (8, 2, 1 << 20, 42)
    assert got.literal_payload == 1 and got.single_fold == 1 and got.pcap == b"/tmp/x.pcap"
    assert got.queue_set == 1 and got.queue == 1 and got.batch_size == 1


def test_binary_help_and_no_gpu_failure():
    r = subprocess.run([BIN, "-h"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--gpubatch" in r.stdout
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([BIN, "-z", "--interface", "eth0", "--dip", "10.0.0.2", "--maxpckts", "10", "--delay", "0"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "no such GPU" in r.stderr


def test_struct_layout_probe(tmp_path):
    """The ctypes view matches GCC's layout of the reference struct (byte offsets)."""
    src = tmp_path / "probe.c"
    src.write_text(r"""
#include <stdio.h>
#include <string.h>
#include "cmd_line.h"
int main(void) { struct cmd_line_af_xdp c; unsigned char *b = (unsigned char *)&c;
#define P(s) memset(&c, 0, sizeof c); s; for (int i = 0; i < (int)sizeof c; i++) if (b[i]) printf("%d %d\n", i, b[i]);
P(c.queue_set = 1) P(c.queue = 1) P(c.no_wake_up = 1) P(c.shared_umem = 1) P(c.batch_size = 1)
P(c.skb_mode = 1) P(c.zero_copy = 1) P(c.copy = 1) printf("%zu\n", sizeof c); }
""")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "pb-af-xdp_amd", "host"), "-o", str(exe), str(src)], check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    probe = [tuple(map(int, l.split())) for l in lines if len(l.split()) == 2]
    buf = (C.c_ubyte * C.sizeof(cb.RefCmd))()
    view = cb.RefCmd.from_buffer(buf)
    got = []
    for n in cb.NAMES:
        C.memset(buf, 0, C.sizeof(buf))
        setattr(view, n, 1)
        got += [(i, v) for i, v in enumerate(buf) if v]
    assert got == probe
    # this build's struct = the reference's 20 bytes + the GPU options
    assert int(lines[len(probe)]) == C.sizeof(cb.OurCmd) and C.sizeof(cb.RefCmd) == 20
    assert cb.OurCmd.gpus.offset == 20


def test_two_pass_command_line():
    """Common (-z) options and AF_XDP/GPU options interleaved in any order parse in
    both passes (main.c:23-46 two-pass scheme) without getopt permutation losses."""
    r = subprocess.run([BIN, "-z", "--seed", "77", "--interface", "eth0", "--queue", "3", "--sip", "10.20.0.0/16",
                        "--pcap", "/tmp/x.pcap", "--dip", "10.0.0.2", "--gpubatch", "99", "--skb", "--protocol", "tcp",
                        "--batchsize", "16", "--gpus", "2", "-l"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "queue_set=1 queue=3" in r.stdout and "batchsize=16 skb=1" in r.stdout
    assert "gpus=2 gpu=0 gpubatch=99 seed=77" in r.stdout and "pcap=/tmp/x.pcap" in r.stdout
    assert "10.20.0.0/16 -> 10.0.0.2 proto tcp" in r.stdout


def test_seed_and_batch_flags_record_that_they_were_given():
    lib = ours()
    got = cb.parse(lib, cb.OurCmd, ["--seed", "0x10", "--veryrandom", "--batchsize", "32"],
                   defaults=lib.cmd_line_af_xdp_defaults)
    assert (got.seed_base, got.seed_set, got.very_random, got.batch_size, got.batch_set) == (16, 1, 1, 32, 1)
    got = cb.parse(lib, cb.OurCmd, [], defaults=lib.cmd_line_af_xdp_defaults)
    assert (got.seed_set, got.very_random, got.batch_size, got.batch_set) == (0, 0, 1, 0)


def test_list_prints_a_drawn_seed_without_seed_flag():
    """-l shows the seed base the run would use: drawn per run unless --seed is given."""
    outs = [subprocess.run([BIN, "-z", "--dip", "10.0.0.2", "-l"], capture_output=True, text=True, timeout=60).stdout
            for _ in range(2)]
    seeds = [o.split("seed=")[1].split()[0] for o in outs]
    assert seeds[0] != seeds[1]
    o = subprocess.run([BIN, "-z", "--dip", "10.0.0.2", "--seed", "5", "-l"], capture_output=True, text=True,
                       timeout=60).stdout
    assert "seed=5 " in o
