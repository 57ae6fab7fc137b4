"""Generate the committed golden vectors (tests/golden/*.npz + index.json).

Run in the build container:  python tests/golden/make_golden.py
Each fixture = frames of one sequence config for a window of iterations,
built by the CPU oracle (oracle/pb_oracle.c) and cross-checked here against
the independent Python restatement (tests/pyspec.py) before it is written.
The GPU parity tests compare libpbgpu.so against these files byte for byte,
so they also pin the oracle against later edits."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd"), os.path.join(ROOT, "tests")]

import oracle_binding as ob  # noqa: E402
import pb_configs as pc  # noqa: E402
import pyspec  # noqa: E402
from pbgpu import Sequence  # noqa: E402

WINDOWS = [(0, 32), (1 << 40, 8)]


def n_for(cfg):
    mx = 54 + max([p.get("length", {}).get("max", 0) for p in cfg.get("payloads", [])] + [256])
    return max(4, min(32, 60000 // mx))


def main():
    index = []
    cases = [(n, 0, 0) for n in pc.ALL] + list(pc.RULE_CASES)
    for name, lit, sf in cases:
        cfg = pc.get(name)
        seq = Sequence.from_config(cfg)
        for first, n in WINDOWS:
            n = min(n, n_for(cfg))
            data, off = ob.build(seq, 0, first, n, pc.SEED_BASE, payload_rule=lit, iph_fold=sf)
            spec = pyspec.build(cfg, 0, first, n, pc.SEED_BASE, literal=bool(lit), single_fold=bool(sf))
            got = [data[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]
            assert got == spec, name
            fn = f"{name}__r{lit}{sf}__k{first}.npz"
            np.savez_compressed(os.path.join(HERE, fn), data=data, offsets=off)
            index.append({"file": fn, "config": name, "payload_rule": lit, "iph_fold": sf, "seq_idx": 0,
                          "seed_base": pc.SEED_BASE, "first_iter": first, "n_iter": n,
                          "n_frames": int(len(off) - 1), "bytes": int(off[-1])})
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/pb_oracle.c",
                   "configs_module": "pb-af-xdp_amd/pb_configs.py", "fixtures": index}, f, indent=1)
    print(len(index), "fixtures")


if __name__ == "__main__":
    main()
