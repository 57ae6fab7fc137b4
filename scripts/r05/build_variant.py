"""Build a variant of libpbgpu.so with literal source substitutions (tool only):
python3 scripts/r05/build_variant.py NAME FILE 'old' 'new' [FILE 'old' 'new' ...]
-> pb-af-xdp_amd/lib/ab/libpbgpu_NAME.so (every substitution must match exactly once)."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "pb-af-xdp_amd")
name, subs = sys.argv[1], sys.argv[2:]
tmp = tempfile.mkdtemp(prefix="pbvar_")
shutil.copytree(os.path.join(SRC, "csrc"), os.path.join(tmp, "pb", "csrc"))
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))  # (../../include from csrc)
for i in range(0, len(subs), 3):
    f, old, new = subs[i:i + 3]
    p = os.path.join(tmp, "pb", "csrc", f)
    s = open(p).read()
    if s.count(old) != 1:
        raise SystemExit(f"{f}: {s.count(old)} matches for {old!r}")
    open(p, "w").write(s.replace(old, new))
out = os.path.join(SRC, "lib", "ab", f"libpbgpu_{name}.so")
os.makedirs(os.path.dirname(out), exist_ok=True)
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-function",
       "-shared", "-o", out, os.path.join(tmp, "pb", "csrc", "pbgpu_kernels.hip"), os.path.join(tmp, "pb", "csrc", "pbgpu.cpp")]
subprocess.run(cmd, check=True, cwd=tmp)
shutil.rmtree(tmp)
print(out)
