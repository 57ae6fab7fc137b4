"""Every write-probe shape (pbgpu_fill_probe_ex) over N bytes: GB/s per shape, one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd")]
from pbgpu import GpuContext  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 27_648_000_000
ctx = GpuContext(0)
shapes, best = ctx.fill_probe_shapes(n, 10)
print(json.dumps({"bytes": n, "best": best, "gbps": {k: round(n / (v * 1e-3) / 1e9, 1) for k, v in shapes.items()},
                  "ms": {k: round(v, 4) for k, v in shapes.items()}}))
ctx.close()
