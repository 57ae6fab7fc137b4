"""pb_vstage_kernel phase stamps (a -DPB_TIMING=1 build, scripts/build_variants.sh tim=-DPB_TIMING=1):
python3 vst_timing.py LIB CONFIG PACKETS [VAR=val ...]; the library prints one pbgpu_timing JSON
line per build on stderr (cycles: A = prologue through the frame records, C = window starts +
build order, B / S summed over the workgroup's windows)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

lib, cfg, n = os.path.join(ROOT, sys.argv[1]), sys.argv[2], int(sys.argv[3])
for e in sys.argv[4:]:
    k, v = e.split("=", 1)
    os.environ[k] = v
os.environ["PBGPU_TIMING"] = "1"
ctx = GpuContext(0, lib_path=lib)
seq = Sequence.from_config(pc.get(cfg))
ctx.load_sequence(0, seq, pc.SEED_BASE)
fb = ctx.alloc_frames(*ctx.build_size(0, n))
for s in range(4):
    ctx.build(0, s * n, n, fb)
    ctx.sync()
fb.free()
ctx.close()
