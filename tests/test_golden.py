"""The oracle reproduces the committed golden vectors (regression pin)."""
import json
import os

import numpy as np
import pytest

import oracle_binding as ob
import pb_configs as pc
from pbgpu import Sequence

GOLD = os.path.join(os.path.dirname(__file__), "golden")
INDEX = json.load(open(os.path.join(GOLD, "index.json")))["fixtures"]


@pytest.mark.parametrize("fx", INDEX, ids=[f["file"] for f in INDEX])
def test_oracle_reproduces_golden(fx):
    z = np.load(os.path.join(GOLD, fx["file"]), allow_pickle=False)
    seq = Sequence.from_config(pc.get(fx["config"]))
    data, off = ob.build(seq, fx["seq_idx"], fx["first_iter"], fx["n_iter"], fx["seed_base"],
                         payload_rule=fx["payload_rule"], iph_fold=fx["iph_fold"])
    assert np.array_equal(off, z["offsets"])
    assert np.array_equal(data, z["data"])


def test_multithreaded_oracle_matches_single_thread():
    """pbo_build_mt (the CPU baseline) emits the same frames as pbo_build."""
    seq = Sequence.from_config(pc.get("c3_udp_var"))
    n = 300
    want = ob.frames(seq, 1, 50, n, pc.SEED_BASE)
    out, tot = ob.build_slots_mt(seq, 1, 50, n, pc.SEED_BASE, 4, slot=2048, faithful=True)
    assert tot == sum(len(w) for w in want)
    for i, w in enumerate(want):
        assert out[i * 2048:i * 2048 + len(w)].tobytes() == w
    ring, _ = ob.build_slots_mt(seq, 1, 50, n, pc.SEED_BASE, 3, slot=2048, faithful=False, ring=8)
    # thread t's last frame lands in its ring slot (frames_of_t - 1) % 8
    per = [n * (t + 1) // 3 - n * t // 3 for t in range(3)]
    first = [n * t // 3 for t in range(3)]
    for t in range(3):
        k = per[t] - 1
        w = want[first[t] + k]
        at = (t * 8 + k % 8) * 2048
        assert ring[at:at + len(w)].tobytes() == w
