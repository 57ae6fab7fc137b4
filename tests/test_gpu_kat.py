"""The reference's own known-answer frames through the HIP kernels directly.

images/test1.gif (README.md:23) shows two receiver-side captures, `udp sum ok`,
of 46-B static UDP frames (TTL 0, 4-B exact payload) built by pcktbatch; the
transcription is the fixture tests/golden/kat_test1_gif.json (SURVEY.md
Appendix C).  Every field is static, so every iteration the GPU builds must be
that frame byte for byte: this pins the IPv4 header checksum (sequence.c:596-602)
and the UDP pseudo-header checksum composition (sequence.c:563-572) on the
device path, through every kernel shape that can build it.  Run on the MI355X
box: pytest -m gpu."""
import json
import os

import pytest

import pb_configs as pc
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_test1_gif.json")))

# the default kernel for 46-B static frames, and the other shapes the library can select
SHAPES = [("default", {}), ("linear", {"PBGPU_KERNEL": "linear"}), ("stage", {"PBGPU_KERNEL": "stage"}),
          ("gpf", {"PBGPU_KERNEL": "gpf"})]


@pytest.fixture(scope="module")
def ctx():
    c = GpuContext(0)
    yield c
    c.close()


@pytest.mark.parametrize("shape,env", SHAPES, ids=[s for s, _ in SHAPES])
@pytest.mark.parametrize("frame", [0, 1])
def test_gpu_builds_reference_captured_frame(ctx, monkeypatch, shape, env, frame):
    fr = KAT["frames"][frame]
    cfg = json.loads(json.dumps(KAT["config"]))
    cfg["udp"]["sport"] = fr["sport"]
    want = bytes.fromhex(fr["hex"].replace(" ", ""))
    assert len(want) == 46
    for k in ("PBGPU_KERNEL", "PBGPU_G", "PBGPU_WGF", "PBGPU_STAGE_KB"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx.load_sequence(0, Sequence.from_config(cfg), pc.SEED_BASE)
    n = 3000  # several workgroups, odd first iteration
    got = ctx.build_frames(0, 12345, n)
    assert len(got) == n
    lo, hi = KAT["covered_bytes"]
    for g in got:
        assert g[lo:hi] == want[lo:hi]  # the bytes the receiver checked (udp sum ok)
        assert g == want  # Ethernet bytes from the command line / sender MAC as well
