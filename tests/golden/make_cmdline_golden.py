"""Golden argv -> struct cmd_line_af_xdp values from the REFERENCE's own
src/cmd_line.c (compiled by `make -C oracle ref` into oracle/_ref/, in the
build container only).  Run: python tests/golden/make_cmdline_golden.py"""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests")]
import cmdline_binding as cb  # noqa: E402

lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_cmdline.so"))
out = []
for argv in cb.ARGV_CASES:
    r = cb.parse(lib, cb.RefCmd, argv)
    out.append({"argv": argv, "fields": {n: int(getattr(r, n)) for n in cb.NAMES}})
json.dump({"source": "reference src/cmd_line.c compiled from /root/reference (oracle/Makefile target ref)",
           "cases": out}, open(os.path.join(HERE, "cmdline_ref.json"), "w"), indent=1)
print(len(out), "cases")
