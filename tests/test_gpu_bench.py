"""bench.py keeps the driver's contract: one JSON line with the BASELINE metric,
the roofline and CPU-baseline objects, and numbers that add up.  Short runs of
the real script (small launches) on the MI355X box: the default configs[1]
line, the configs[4] three-sequence mix under torchrun (the RCCL process group,
barrier and counter all-reduce at world size 1, the path the driver's N-GPU
scaling run takes), and the configs[3] line."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:] + out.stderr[-3000:]
    return json.loads(lines[0])


def test_bench_json_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "1", "--packets",
           str(1 << 20), "--ramp-seconds", "0.05", "--cpu-seconds", "0.4"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    d = _line(out)
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["vs_baseline"] is None
    # value = packets per second of the timed launches (Mpps), ms_per_step their wall time
    assert abs(d["value"] - (1 << 20) / (d["ms_per_step"] * 1e-3) / 1e6) < 0.01 * d["value"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["algorithmic_bytes_per_launch"] == (1 << 20) * 64
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert 0.05 < r["frac"] < 1.0
    assert r["traffic_source"].startswith("profiles/")
    assert d["config"]["workload"].startswith("c2_udp_64")
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    # the threads actually usable: the affinity mask capped by the cgroup CPU quota
    q = cb["host"]["cgroup_cpu_quota"]
    assert cb["cores"] == min(cb["host"]["affinity"], -(-q // 1) if q else cb["host"]["affinity"])
    assert cb["host"]["model"] and d["cpu_baseline_variants"]["faithful_16_threads"]["cores"] == 16
    # each launch timed on its own in a separate pass; the 1500-B leg >= 20 timed steps
    for pl in (r["per_launch_ms"], d["udp_1500"]["per_launch_ms"]):
        assert pl["n"] == 20 and 0 < pl["min"] <= pl["median"] <= pl["max"]
    assert d["udp_1500"]["steps"] >= 20
    assert "not measured" in d["cpu_baseline_variants"]["configs0_c1_udp_static_64_1_thread"]["af_xdp_send"]
    assert d["udp_1500"]["kernel"].startswith("pb_fstage_kernel")
    # the write-roofline probe: every shape reported, the fastest named
    shapes = d["write_peak_probe_shapes_gbps"]
    assert len(shapes) == 15 and d["write_peak_probe_shape"] in shapes
    assert d["write_peak_probe_gbps"] == max(shapes.values())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_mix_under_torchrun_reduces_counters():
    """configs[4]: three sequences per step, the global counters all-reduced over
    RCCL equal packets x steps per sequence (world size 1: the path itself)."""
    n, steps = 1 << 19, 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps",
           str(steps), "--warmup", "1", "--packets", str(n), "--ramp-seconds", "0.05", "--cpu-seconds", "0",
           "--config", "c5_mix"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    gc = d["global_counters"]
    assert gc["sequences"] == ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"]
    assert gc["packets"] == [n * steps] * 3
    assert gc["bytes"] == [n * steps * 64, n * steps * 60, n * steps * 98]
    assert d["config"]["bytes_per_step_per_gpu"] == n * (64 + 60 + 98)
    assert abs(d["value"] - 3 * n / (d["ms_per_step"] * 1e-3) / 1e6) < 0.01 * d["value"]
    # one fused launch per step (pbgpu_build_batch), then the three sequences' kernel bodies
    k = d["roofline"]["kernel"]
    assert len(k) == 4 and k[0].startswith("pb_batch_kernel<") and all(x.startswith("(part) pb_x") for x in k[1:]), k


def test_bench_two_ranks_share_the_gpu_over_gloo():
    """The N-rank path with real builds: two ranks on one GPU (PB_DIST_BACKEND=gloo), each
    building its own shard of every step; the reduced counters cover both ranks' frames."""
    n, steps, world = 1 << 19, 3, 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus",
           str(world), "--steps", str(steps), "--warmup", "1", "--packets", str(n), "--ramp-seconds", "0.05",
           "--cpu-seconds", "0", "--config", "c5_mix"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PB_DIST_BACKEND="gloo")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_gpus"] == world
    gc = d["global_counters"]
    assert gc["packets"] == [n * steps * world] * 3
    assert gc["bytes"] == [n * steps * world * 64, n * steps * world * 60, n * steps * world * 98]
    assert abs(d["value"] - world * 3 * n / (d["ms_per_step"] * 1e-3) / 1e6) < 0.01 * d["value"]


def test_bench_tcp_syn_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--packets",
           str(1 << 20), "--ramp-seconds", "0.05", "--cpu-seconds", "0", "--config", "c4_tcp_syn"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    d = _line(out)
    assert d["config"]["frame_bytes"] == 60 and d["roofline"]["algorithmic_bytes_per_launch"] == 60 << 20
    assert d["roofline"]["kernel"].startswith("pb_xpage_kernel")
    assert "cpu_baseline" not in d and "global_counters" not in d
