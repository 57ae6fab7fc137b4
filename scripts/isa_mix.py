"""Instruction mix of kernels in a device .s file: python3 isa_mix.py file.s name_substring..."""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    for line in s.split("\n"):
        if line.startswith("_Z") and line.split(":")[0].endswith("") and pat in line.split(":")[0]:
            name = line.split(":")[0]
            a = s.index(name + ":")
            b = s.index(".Lfunc_end", a)
            ins = [l.strip() for l in s[a:b].split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
            c = Counter(i.split()[0] for i in ins)
            print(name, len(ins), "valu", sum(v for k, v in c.items() if k.startswith("v_")),
                  "salu", sum(v for k, v in c.items() if k.startswith("s_")))
            print("  ", c.most_common(30))
            break
