"""Diagnostic: variable-length frames landed in registered (mapped) UMEM by the
scatter path, batch after batch, against the oracle."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pb-af-xdp_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import oracle_binding as ob  # noqa: E402
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

cfg = {"eth": {}, "ip": {"dip": pc.DIP, "ranges": ["172.16.0.0/12"], "protocol": "tcp"},
       "tcp": {"dport": 80, "syn": 1}, "payloads": [{"length": {"min": 0, "max": 900}}]}
seq = Sequence.from_config(cfg)
bad = 0
with GpuContext(0) as g:
    g.load_sequence(0, seq, 7)
    print("kernel", g.kernel_name(0))
    fb = g.alloc_frames(*g.build_size(0, 1000))
    umem = np.zeros(4096 * 4096, dtype=np.uint8)
    g.lib.pbgpu_host_register(g.h, umem.ctypes.data, umem.nbytes)
    for b in range(3):
        g.build(0, b * 1000, 1000, fb)
        lens = fb.to_umem(umem, 4096, 0, 1000)
        want = ob.frames(seq, 0, b * 1000, 1000, 7)
        offs = fb.offsets()
        for j in range(1000):
            got = umem[j * 4096:j * 4096 + int(lens[j])].tobytes()
            if got != want[j]:
                bad += 1
                if bad < 6:
                    print(f"batch {b} frame {j}: len {int(lens[j])} want {len(want[j])} "
                          f"off {int(offs[j])}..{int(offs[j + 1])}")
        print("batch", b, "bad so far", bad)
    g.lib.pbgpu_host_unregister(g.h, umem.ctypes.data)
print("BAD" if bad else "OK")
