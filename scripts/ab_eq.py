"""Bitwise equality of a compile-time variant of libpbgpu.so with the shipped library
(itself parity-tested against the oracle) on every BASELINE / edge config, under a few
shape overrides.  python3 ab_eq.py VARIANT_SO [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
import pb_configs as pc  # noqa: E402
from pbgpu import LIB_PATH, GpuContext, Sequence  # noqa: E402

var = os.path.join(ROOT, sys.argv[1])
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 17
ENVS = [{}, {"PBGPU_STAGE_KB": "16"}, {"PBGPU_FST_G": "16"}, {"PBGPU_FST_G": "32"},
        {"PBGPU_XP_IMG": "2"}, {"PBGPU_XP_IMG": "0"}, {"PBGPU_ALLOC": "malloc"}]
ctxs = [GpuContext(0, lib_path=LIB_PATH), GpuContext(0, lib_path=var)]
bad = 0
for env in ENVS:
    for k in ("PBGPU_STAGE_KB", "PBGPU_FST_G", "PBGPU_XP_IMG", "PBGPU_ALLOC"):
        os.environ.pop(k, None)
    os.environ.update(env)
    for name in pc.ALL:
        seq = Sequence.from_config(pc.get(name))
        n = N if "jumbo" not in name else N // 8
        outs, kn = [], []
        for ctx in ctxs:
            ctx.load_sequence(0, seq, pc.SEED_BASE)
            fb = ctx.alloc_frames(*ctx.build_size(0, n))
            ctx.build(0, 12345, n, fb)
            ctx.sync()
            outs.append((fb.packed(), fb.offsets()))
            kn.append(ctx.kernel_name(0))
            fb.free()
        ok = np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
        bad += not ok
        print(f"{'ok  ' if ok else 'DIFF'} {name:28s} {env} {kn[1]}", flush=True)
for c in ctxs:
    c.close()
print("ALL EQUAL" if not bad else f"{bad} DIFFERENT")
sys.exit(1 if bad else 0)
