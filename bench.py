"""bench.py — device-resident packet-build throughput on MI355X.

BASELINE.json metric: "device-resident Mpps & GB/s, 64B and 1500B UDP, L3+L4
checksums on".  One step = one launch building 2^25 packets of configs[1]
(UDP 64-B frame, random /16 source + source port, 22-B random payload, both
checksums) into HBM.  Multi-GPU: one process per GPU, each
rank builds its own disjoint iteration range (weak scaling, no data-path
collective); the global packet / byte counters are all-reduced over RCCL once
at the end of the timed region (the reference's total_pckts/total_bytes,
sequence.c:12-14).

Prints ONE JSON line on rank 0.  The 1500-B variant, the D2H-inclusive rate
into 4 KiB UMEM slots and the measured write-only peak ride along as extra
keys.  The CPU oracle (oracle/, the checker) is timed beside it on the host
cores as cpu_baseline — it is never the thing measured.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "pb-af-xdp_amd")
for _p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

import pb_configs as pc  # noqa: E402
import pb_dist  # noqa: E402
from pbgpu import GpuContext, Sequence  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
HBM_ACHIEVABLE_GBPS = 6300.0  # the same guide's "≈6.3 TB/s achievable" (HBM section)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--ramp-seconds", type=float, default=0.5,
                    help="untimed build launches before the warm-up steps, until the GPU clock has ramped")
    ap.add_argument("--packets", type=int, default=1 << 25, help="packets per launch (per GPU)")
    ap.add_argument("--config", default="c2_udp_64")
    ap.add_argument("--no-variants", action="store_true", help="skip the 1500-B / D2H / fill extras")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_r01.json"),
                    help="committed rocprofv3 --pmc summary giving HBM bytes per launch")
    return ap.parse_args()


def init_dist(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist  # noqa: F811

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return dist, world, rank, local


def barrier(dist, local):
    if dist is not None:
        import torch

        dist.barrier()
        torch.cuda.synchronize(local)


def run_config(ctx, name, seq_idx, n_pkts, steps, warmup, rank, world, dist, local, ramp_s=0.0):
    """Warm up, then time exactly `steps` launches; returns per-rank timings.

    The GPU starts a run below its sustained clock: the same 2-GiB launch took
    0.36-0.37 ms for the first ~10 ms of back-to-back launches and 0.30-0.31 ms
    after (scripts/alloc_probe.py), so untimed launches run for `ramp_s` seconds
    before the warm-up steps and the timed region sees the steady state a
    continuously sending generator runs in."""
    seq = Sequence.from_config(pc.get(name))
    ctx.load_sequence(seq_idx, seq, pc.SEED_BASE)
    fb = ctx.alloc_frames(*ctx.build_size(seq_idx, n_pkts))
    # span timing: one HIP-event pair around the timed launches, none per launch
    # (a per-launch pair writes back the L2 twice per launch: ~9 us gaps)
    ctx.set_timing(ctx.TIMING_SPAN)
    step_iter = lambda s: pb_dist.step_first_iter(s, rank, world, n_pkts)  # noqa: E731
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < ramp_s:
        for s in range(8):
            ctx.build(seq_idx, step_iter(s), n_pkts, fb)
        ctx.sync()
    for s in range(warmup):
        ctx.build(seq_idx, step_iter(s), n_pkts, fb)
    ctx.sync()
    ctx.kernel_time()  # drop warm-up launches
    p0, b0 = ctx.counters(seq_idx + 1)
    barrier(dist, local)
    t0 = time.perf_counter()
    for s in range(steps):
        ctx.build(seq_idx, step_iter(warmup + s), n_pkts, fb)
    ctx.sync()
    counters = None
    if dist is not None:
        p, b = ctx.counters(seq_idx + 1)
        # RCCL over xGMI: the global sent-packet / byte counter
        gp, gb = pb_dist.allreduce_counters([p[seq_idx]], [b[seq_idx]], device=f"cuda:{local}")
        counters = [gp[0], gb[0]]
    barrier(dist, local)
    wall = time.perf_counter() - t0
    k_ms, k_n = ctx.kernel_time()
    flen = int(fb.f.fixed_len)
    p1, b1 = ctx.counters(seq_idx + 1)
    bytes_per_launch = int(b1[seq_idx] - b0[seq_idx]) // steps  # this rank's frame bytes per launch
    kernel = ctx.kernel_name(seq_idx)
    fb.free()
    if dist is not None:
        import torch

        w = torch.tensor([wall], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    return {"wall_s": wall, "kernel_ms_avg": k_ms / max(k_n, 1), "kernel_launches": k_n, "flen": flen,
            "counters": counters, "bytes_per_launch": bytes_per_launch, "kernel": kernel}


def d2h_rate(ctx, seq_idx, n_pkts):
    """Build + land into 4 KiB UMEM slots in pinned host memory (af_xdp.c:200-214)."""
    n = min(n_pkts, 1 << 18)
    umem = np.zeros(n * 4096, dtype=np.uint8)
    ctx.lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes)
    fb = ctx.alloc_frames(*ctx.build_size(seq_idx, n))
    ctx.build(seq_idx, 0, n, fb)
    fb.to_umem(umem, 4096, 0, n)
    t0 = time.perf_counter()
    reps = 5
    for r in range(reps):
        ctx.build(seq_idx, r * n, n, fb)
        fb.to_umem(umem, 4096, 0, n)
    dt = (time.perf_counter() - t0) / reps
    frame_bytes = fb.total_bytes()
    fb.free()
    ctx.kernel_time()
    ctx.lib.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
    return {"packets": n, "mpps": n / dt / 1e6, "ms_per_batch": dt * 1e3, "slot": 4096,
            "frame_gbps": frame_bytes / dt / 1e9}


def cpu_baseline(name, budget_s, threads=None, faithful=True):
    """The CPU oracle on the host cores, frames copied into 4 KiB UMEM slots.
    faithful: a clock read and the rand_ip dotted-string round trip per
    iteration, as sequence.c:434-497 does; lean: integer only."""
    import oracle_binding as ob

    if threads is None:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
    seq = Sequence.from_config(pc.get(name))
    n = 20000 * threads
    ring = 4096  # NUM_FRAMES slots per socket, af_xdp.h:23
    out = np.zeros(threads * ring * 4096, dtype=np.uint8)
    while True:
        t0 = time.perf_counter()
        _, tot = ob.build_slots_mt(seq, 0, 0, n, pc.SEED_BASE, threads, out=out, ring=ring, faithful=faithful)
        dt = time.perf_counter() - t0
        if dt >= budget_s / 2 or n >= (1 << 28):
            break
        n = min(1 << 28, int(n * max(2.0, budget_s / max(dt, 1e-3))))
    mode = ("faithful mode: clock_gettime + rand_ip string round trip per iteration" if faithful
            else "lean mode: integer only")
    return {"value": n / dt / 1e6, "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": f"{n} iterations of {name} (oracle {mode}, frames into a per-thread ring of "
                      f"4096 x 4096-B UMEM slots), {threads} pthreads, {dt:.2f} s", "gbps": tot / dt / 1e9}


def pmc_traffic(path, name):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("per_launch_hbm_bytes", {}).get(name)
    except (OSError, ValueError):
        return None


def main():
    a = parse()
    dist, world, rank, local = init_dist(a.gpus)
    ctx = GpuContext(local)
    res = run_config(ctx, a.config, 0, a.packets, a.steps, a.warmup, rank, world, dist, local, a.ramp_seconds)
    flen = res["flen"]
    bpl = res["bytes_per_launch"]  # frame bytes one launch builds on one GPU
    pkts_total = a.packets * a.steps * world
    wall = res["wall_s"]
    mpps = pkts_total / wall / 1e6
    gbps = bpl * a.steps * world / wall / 1e9
    k_s = res["kernel_ms_avg"] * 1e-3
    achieved = bpl / k_s / 1e9
    extra = {}
    peak_probe = None
    if rank == 0:
        fill_ms = ctx.fill_probe(bpl, 20)
        peak_probe = bpl / (fill_ms * 1e-3) / 1e9
        extra["write_peak_probe_gbps"] = round(peak_probe, 1)
    if not a.no_variants:
        steps15 = max(3, a.steps // 4)
        v = run_config(ctx, "c2_udp_1500", 1, a.packets, steps15, 1, rank, world, dist, local, a.ramp_seconds / 2)
        n1500 = a.packets * steps15 * world
        ach15 = v["bytes_per_launch"] / (v["kernel_ms_avg"] * 1e-3) / 1e9
        extra["udp_1500"] = {
            "mpps": round(n1500 / v["wall_s"] / 1e6, 3),
            "gbps": round(v["bytes_per_launch"] * steps15 * world / v["wall_s"] / 1e9, 2),
            "kernel": v["kernel"], "kernel_ms_avg": round(v["kernel_ms_avg"], 4),
            "roofline_achieved_gbps": round(ach15, 1), "roofline_frac": round(ach15 / HBM_PEAK_GBPS, 4),
            "frac_of_guide_achievable": round(ach15 / HBM_ACHIEVABLE_GBPS, 4),
            "traffic": pmc_traffic(a.pmc, "c2_udp_1500"), "algorithmic_bytes_per_launch": v["bytes_per_launch"],
            "packets_per_launch": a.packets}
        if rank == 0:
            extra["d2h_umem_64B"] = d2h_rate(ctx, 0, a.packets)
            extra["d2h_umem_1500B"] = d2h_rate(ctx, 1, a.packets)
    ctx.close()
    if rank != 0:
        return
    line = {
        "metric": "device-resident Mpps & GB/s, 64B and 1500B UDP, L3+L4 checksums on",
        "value": round(mpps, 3),
        "unit": "Mpps",
        "gbps": round(gbps, 3),
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ramp_seconds": a.ramp_seconds,
        "ms_per_step": round(wall / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seed stream splitmix64(0x5EEDBA5E ^ (seq<<48) + k); SURVEY.md §8d C2)",
        "config": {"workload": f"{a.config}: " + " ".join((pc.BASELINE.get(a.config) or pc.c2_udp_64).__doc__.split()),
                   "packets_per_launch_per_gpu": a.packets,
                   "frame_bytes": flen or None, "bytes_per_launch_per_gpu": bpl,
                   "parallelism": f"shard-by-iteration x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac_of_guide_achievable": round(achieved / HBM_ACHIEVABLE_GBPS, 4),
                     "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": pmc_traffic(a.pmc, a.config), "kernel": res["kernel"],
                     "kernel_ms_avg": round(res["kernel_ms_avg"], 5),
                     "algorithmic_bytes_per_launch": bpl,
                     "frac_of_measured_write_peak": round(achieved / peak_probe, 4) if peak_probe else None},
    }
    if res["counters"] is not None:
        line["global_counters"] = {"packets": res["counters"][0], "bytes": res["counters"][1]}
    line.update(extra)
    if world == 1 and a.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_baseline(a.config, a.cpu_seconds)
        # the other CPU-path points SURVEY.md §8d names: one thread, and the integer-only form
        short = max(1.0, a.cpu_seconds / 4)
        line["cpu_baseline_variants"] = {
            "faithful_1_thread": cpu_baseline(a.config, short, threads=1),
            "lean_all_threads": cpu_baseline(a.config, short, faithful=False)}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
