"""Frame-length / alignment probe: kernel write rate of the build for UDP frames
of several lengths (16-B aligned, 128-B aligned and unaligned strides) plus the
variable-length config and the plain write-peak probe.  GPU only."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pb-af-xdp_amd"))
import pb_configs as pc  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

TARGET = 3 << 30


def rate(ctx, cfg, n, reps=10):
    ctx.load_sequence(0, Sequence.from_config(cfg), pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(0, n))
    for r in range(2):
        ctx.build(0, r * n, n, fb)
    ctx.sync()
    ctx.kernel_time()
    p0, b0 = ctx.counters(1)
    for r in range(reps):
        ctx.build(0, (r + 2) * n, n, fb)
    ctx.sync()
    ms, k = ctx.kernel_time()
    p1, b1 = ctx.counters(1)
    nbytes = (b1[0] - b0[0]) / reps
    name = ctx.kernel_name(0)
    fb.free()
    return {"kernel": name, "frames": n, "bytes": int(nbytes), "ms": round(ms / k, 4),
            "gbps": round(nbytes / (ms / k * 1e-3) / 1e9, 1)}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    lens = [int(x) for x in os.environ.get("LENS", "64,100,1500,1504,1536,1472,1408,1024,512").split(",")]
    out = {"tag": tag}
    with GpuContext(0) as ctx:
        out["fill_gbps"] = round(TARGET / (ctx.fill_probe(TARGET, 20) * 1e-3) / 1e9, 1)
        for flen in lens:
            cfg = json.loads(json.dumps(pc.get("c2_udp_1500")))
            cfg["payloads"][0]["length"] = {"min": flen - 42, "max": flen - 42}
            out[f"udp{flen}"] = rate(ctx, cfg, TARGET // flen)
        out["c3_udp_var"] = rate(ctx, pc.get("c3_udp_var"), 1 << 22)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
