"""bench.py — device-resident packet-build throughput on MI355X.

BASELINE.json metric: "device-resident Mpps & GB/s, 64B and 1500B UDP, L3+L4
checksums on".  One step = one launch building 2^25 packets of configs[1]
(UDP 64-B frame, random /16 source + source port, 22-B random payload, both
checksums) into HBM.  --config picks another BASELINE
workload for the same line shape: c2_udp_1500, c3_udp_var (configs[2]),
c4_tcp_syn (configs[3]) and c5_mix (configs[4]: three sequences — UDP 64 B, TCP
SYN 60 B, ICMP 98 B — built per step, 2^24 iterations each per GPU).

Multi-GPU: one process per GPU, each rank builds its own disjoint iteration
range (weak scaling, no data-path collective).  The only exchange is the
reference's global counter (total_pckts / total_bytes, sequence.c:12-14,
633-642): per-sequence {packets, bytes} of the timed steps, all-reduced once
over RCCL at the end of the timed region.  Under torchrun the process group is
created at every world size, 1 included, so the RCCL path runs on one GPU too.

Prints ONE JSON line on rank 0.  The 1500-B variant, the D2H-inclusive rate
into 4 KiB UMEM slots and the write-roofline probe ride along as extra keys.
The CPU oracle (oracle/, the checker) is timed beside it on the host cores as
cpu_baseline — it is never the thing measured.
"""
import argparse
import json
import os
import platform
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
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_r06.json")
MIX = ("c2_udp_64", "c4_tcp_syn", "c5_icmp_echo")  # configs[4]'s three sequences (pb_configs.c5_mix)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--ramp-seconds", type=float, default=0.5,
                    help="untimed build launches before the warm-up steps, until the GPU clock has ramped")
    ap.add_argument("--packets", type=int, default=None,
                    help="iterations per launch per GPU (default 2^25; 2^24 per sequence for c5_mix)")
    ap.add_argument("--config", default="c2_udp_64",
                    choices=["c2_udp_64", "c2_udp_1500", "c3_udp_var", "c4_tcp_syn", "c5_icmp_echo", "c5_mix"])
    ap.add_argument("--no-variants", action="store_true", help="skip the 1500-B / D2H extras")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--pmc", default=PMC_FILE, help="committed rocprofv3 --pmc summary giving HBM bytes per launch")
    a = ap.parse_args()
    if a.packets is None:
        a.packets = (1 << 24) if a.config == "c5_mix" else (1 << 25)
    return a


def init_dist(n_gpus):
    """torchrun (WORLD_SIZE in the environment): RCCL process group at any world
    size; a plain `python bench.py` run is one rank without a process group."""
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    if n_gpus > 1 and not launched:
        raise SystemExit("--gpus N > 1 runs under torch.distributed.run (one process per GPU)")
    dist = None
    if launched:
        import torch
        import torch.distributed as dist  # noqa: F811

        # PB_DIST_BACKEND=gloo: a rehearsal of the N-rank path on fewer GPUs (ranks share a GPU
        # round-robin, counters and timings reduce over gloo); the bench itself is RCCL
        backend = os.environ.get("PB_DIST_BACKEND", "nccl")
        if backend == "gloo":
            if torch.cuda.is_available():
                local %= max(1, torch.cuda.device_count())
                torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return dist, world, rank, local


def reduce_device(local):
    """Where the collectives' tensors live: the rank's GPU under RCCL, host memory under gloo."""
    return "cpu" if os.environ.get("PB_DIST_BACKEND", "nccl") == "gloo" else f"cuda:{local}"


def barrier(dist, local):
    if dist is not None:
        import torch

        dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize(local)


def run_configs(ctx, names, n_pkts, steps, warmup, rank, world, dist, local, ramp_s=0.0, launch_reps=0):
    """Warm up, then time exactly `steps` steps; a step builds `n_pkts` iterations
    of every sequence in `names` (one launch each).  Returns per-rank timings and
    the all-reduced counters of the timed steps.

    The GPU starts a run below its sustained clock: the same 2-GiB launch took
    0.36-0.37 ms for the first ~10 ms of back-to-back launches and 0.30-0.31 ms
    after (scripts/alloc_probe.py), so untimed launches run for `ramp_s` seconds
    before the warm-up steps and the timed region sees the steady state a
    continuously sending generator runs in."""
    nseq = len(names)
    bufs = []
    for i, name in enumerate(names):
        seq = Sequence.from_config(pc.get(name))
        ctx.load_sequence(i, seq, pc.SEED_BASE)
        bufs.append(ctx.alloc_frames(*ctx.build_size(i, n_pkts)))
    # span timing: one HIP-event pair around the timed launches, none per launch
    # (a per-launch pair writes back the L2 twice per launch: ~9 us gaps)
    ctx.set_timing(ctx.TIMING_SPAN)
    step_iter = lambda s: pb_dist.step_first_iter(s, rank, world, n_pkts)  # noqa: E731

    # several sequences: one pbgpu_build_batch call per step (configs[4]'s three: one fused
    # launch, pb_batch_kernel; PBGPU_BATCH=0: one launch per sequence on its own stream)
    batch = nseq > 1 and os.environ.get("PBGPU_BATCH", "1") != "0"

    def step(s):
        if batch:
            ctx.build_batch([(i, step_iter(s), n_pkts, bufs[i]) for i in range(nseq)])
            return
        for i in range(nseq):
            ctx.build(i, step_iter(s), n_pkts, bufs[i])

    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < ramp_s:
        for s in range(8):
            step(s)
        ctx.sync()
    for s in range(warmup):
        step(s)
    ctx.sync()
    ctx.kernel_time()  # drop warm-up launches
    p0, b0 = ctx.counters(nseq)
    barrier(dist, local)
    t0 = time.perf_counter()
    for s in range(steps):
        step(warmup + s)
    ctx.sync()
    p1, b1 = ctx.counters(nseq)
    dp = [int(x) for x in (p1 - p0)]
    db = [int(x) for x in (b1 - b0)]
    # the kernels count the frames they built and the bytes they stored, workgroup by
    # workgroup: a short or skipped build fails here instead of inflating the rate
    for i in range(nseq):
        flen = int(bufs[i].f.fixed_len)
        if dp[i] != steps * n_pkts or (flen and db[i] != steps * n_pkts * flen):
            raise SystemExit(f"counter mismatch on {names[i]}: {dp[i]} frames / {db[i]} bytes for "
                             f"{steps} x {n_pkts} iterations")
    counters = None
    if dist is not None:
        # RCCL over xGMI: the global sent-packet / byte counters of the timed steps
        gp, gb = pb_dist.allreduce_counters(dp, db, device=reduce_device(local))
        counters = {"packets": gp, "bytes": gb}
        if gp != [steps * n_pkts * world] * nseq:
            raise SystemExit(f"global counter mismatch: {gp} frames for {world} x {steps} x {n_pkts} per sequence")
    barrier(dist, local)
    wall = time.perf_counter() - t0
    k_ms, k_n = ctx.kernel_time()
    per_step_launches = max(1, k_n // steps)
    # a separate pass with an event pair around every launch: each launch's own device
    # time (median / min / max; the pairs add ~10 us between launches, so `value` and
    # the roofline come from the span above, not from this pass)
    per_launch = None
    if launch_reps:
        ctx.set_timing(ctx.TIMING_LAUNCH)
        for s in range(launch_reps):
            step(warmup + steps + s)
        ctx.sync()
        t = ctx.kernel_times()
        ctx.set_timing(ctx.TIMING_SPAN)
        if len(t):
            per_step = t.reshape(-1, per_step_launches).sum(axis=1) if len(t) % per_step_launches == 0 else t
            per_launch = {"median": round(float(np.median(per_step)), 5), "min": round(float(per_step.min()), 5),
                          "max": round(float(per_step.max()), 5), "n": int(len(per_step)),
                          "mode": "HIP event pair around every launch, separate pass after the timed span"}
    flens = [int(fb.f.fixed_len) for fb in bufs]
    kernels = [ctx.kernel_name(i) for i in range(nseq)]
    if nseq > 1 and per_step_launches == 1:  # the fused launch, running each sequence's kernel body
        wgt = 256 if os.environ.get("PBGPU_BATCH_WGT") == "256" else 512
        kernels = [f"pb_batch_kernel<{wgt}, 1, 2, 3>"] + [f"(part) {k}" for k in kernels]
    for fb in bufs:
        fb.free()
    if dist is not None:
        import torch

        w = torch.tensor([wall], dtype=torch.float64, device=reduce_device(local))
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    return {"wall_s": wall, "span_ms_per_step": k_ms / max(steps, 1), "kernel_launches": k_n, "flens": flens,
            "per_launch_ms": per_launch,
            "counters": counters, "packets_per_step": sum(dp) // steps, "bytes_per_step": sum(db) // steps,
            "per_seq_bytes_per_step": [x // steps for x in db], "kernels": kernels}


def d2h_rate(ctx, seq_idx, n_pkts, slot=4096):
    """Build + land into UMEM slots in pinned host memory: 4 KiB (af_xdp.c:200-214), or the
    smaller slots of --umemslot (64 B: back to back, written whole)."""
    n = min(n_pkts, 1 << 18)
    umem = np.zeros(n * slot, dtype=np.uint8)
    ctx.lib.pbgpu_host_register(ctx.h, umem.ctypes.data, umem.nbytes)
    fb = ctx.alloc_frames(*ctx.build_size(seq_idx, n))
    ctx.build(seq_idx, 0, n, fb)
    fb.to_umem(umem, slot, 0, n)
    t0 = time.perf_counter()
    reps = 5
    for r in range(reps):
        ctx.build(seq_idx, r * n, n, fb)
        fb.to_umem(umem, slot, 0, n)
    dt = (time.perf_counter() - t0) / reps
    frame_bytes = fb.total_bytes()
    fb.free()
    ctx.kernel_time()
    ctx.lib.pbgpu_host_unregister(ctx.h, umem.ctypes.data)
    return {"packets": n, "mpps": n / dt / 1e6, "ms_per_batch": dt * 1e3, "slot": slot,
            "frame_gbps": frame_bytes / dt / 1e9}


def host_cpu():
    """The host the CPU baseline runs on: model, logical CPUs, the CPUs this process
    may use and the cgroup CPU quota (the GPU box shares a large host)."""
    model = platform.processor() or "?"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota}


def usable_cpus():
    """The CPUs this process can actually use: its affinity mask, capped by the
    cgroup CPU quota (the GPU box gives a 16-CPU quota on a 256-CPU host, so 256
    threads would only time-slice 16 CPUs' worth)."""
    n = len(os.sched_getaffinity(0))
    q = host_cpu()["cgroup_cpu_quota"]
    if q:
        n = min(n, int(-(-q // 1)))
    return max(1, n)


def cpu_baseline(name, budget_s, threads=None, faithful=True):
    """The CPU oracle on the host cores, frames copied into 4 KiB UMEM slots.
    faithful: a clock read and the rand_ip dotted-string round trip per
    iteration, as sequence.c:434-497 does; lean: integer only.
    Default threads: the usable CPUs (affinity mask capped by the cgroup quota)."""
    import oracle_binding as ob

    if threads is None:
        threads = usable_cpus()
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


def pmc_traffic(path, names, packets):
    """HBM bytes per step from a committed rocprofv3 --pmc summary (not measured in
    this run), scaled from the PMC pass's packets per launch to `packets`."""
    try:
        with open(path) as f:
            d = json.load(f)
        hbm, pk = d.get("per_launch_hbm_bytes", {}), d.get("packets_per_launch", {})
        vals = [hbm[n] * packets / pk.get(n, packets) for n in names]
        return int(sum(vals))
    except (OSError, ValueError, KeyError):
        return None


def main():
    a = parse()
    dist, world, rank, local = init_dist(a.gpus)
    ctx = GpuContext(local)
    names = list(MIX) if a.config == "c5_mix" else [a.config]
    res = run_configs(ctx, names, a.packets, a.steps, a.warmup, rank, world, dist, local, a.ramp_seconds,
                      launch_reps=20)
    bps = res["bytes_per_step"]  # frame bytes one step builds on one GPU
    pkts_total = res["packets_per_step"] * a.steps * world
    wall = res["wall_s"]
    mpps = pkts_total / wall / 1e6
    gbps = bps * a.steps * world / wall / 1e9
    achieved = bps / (res["span_ms_per_step"] * 1e-3) / 1e9
    extra = {}
    peak_probe = None
    if rank == 0:
        shapes, best = ctx.fill_probe_shapes(bps, 20)
        peak_probe = bps / (shapes[best] * 1e-3) / 1e9
        extra["write_peak_probe_gbps"] = round(peak_probe, 1)
        extra["write_peak_probe_shape"] = best
        extra["write_peak_probe_shapes_gbps"] = {k: round(bps / (v * 1e-3) / 1e9, 1) for k, v in shapes.items()}
    if not a.no_variants and a.config == "c2_udp_64":
        # >= 20 timed steps (~0.15 s of 50-GB launches) after a full clock ramp
        steps15 = max(20, a.steps // 4)
        v = run_configs(ctx, ["c2_udp_1500"], a.packets, steps15, 2, rank, world, dist, local, a.ramp_seconds,
                        launch_reps=20)
        n1500 = v["packets_per_step"] * steps15 * world
        ach15 = v["bytes_per_step"] / (v["span_ms_per_step"] * 1e-3) / 1e9
        extra["udp_1500"] = {
            "mpps": round(n1500 / v["wall_s"] / 1e6, 3),
            "gbps": round(v["bytes_per_step"] * steps15 * world / v["wall_s"] / 1e9, 2),
            "steps": steps15, "kernel": v["kernels"][0], "kernel_ms_avg": round(v["span_ms_per_step"], 4),
            "per_launch_ms": v["per_launch_ms"],
            "roofline_achieved_gbps": round(ach15, 1), "roofline_frac": round(ach15 / HBM_PEAK_GBPS, 4),
            "frac_of_guide_achievable": round(ach15 / HBM_ACHIEVABLE_GBPS, 4),
            "frac_of_measured_write_peak": round(ach15 / peak_probe, 4) if peak_probe else None,
            "traffic": pmc_traffic(a.pmc, ["c2_udp_1500"], a.packets), "traffic_source": os.path.relpath(a.pmc, ROOT),
            "algorithmic_bytes_per_launch": v["bytes_per_step"], "packets_per_launch": a.packets}
        if rank == 0:
            ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
            ctx.load_sequence(1, Sequence.from_config(pc.get("c2_udp_1500")), pc.SEED_BASE)
            extra["d2h_umem_64B"] = d2h_rate(ctx, 0, a.packets)
            extra["d2h_umem_64B_slot64"] = d2h_rate(ctx, 0, a.packets, 64)
            extra["d2h_umem_1500B"] = d2h_rate(ctx, 1, a.packets)
    if not a.no_variants and a.config != "c2_udp_64" and a.config != "c5_mix" and rank == 0:
        # the configured sequence (still loaded at index 0) landed into UMEM slots
        extra["d2h_umem"] = d2h_rate(ctx, 0, a.packets)
    ctx.close()
    if rank != 0:
        return
    doc = " ".join((pc.c5_mix if a.config == "c5_mix" else pc.BASELINE[a.config]).__doc__.split())
    # the fused mix launch's own PMC pass when the summary has one (else the parts' passes summed)
    mix_traffic = pmc_traffic(a.pmc, ["c5_mix"], a.packets) if a.config == "c5_mix" and \
        res["kernels"][0].startswith("pb_batch_kernel") else None
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
        "data": "synthetic (seed stream splitmix64(0x5EEDBA5E ^ (seq<<48) + k); SURVEY.md §8d)",
        "config": {"workload": f"{a.config}: {doc}",
                   "sequences": names,
                   "packets_per_launch_per_gpu": a.packets,
                   "frame_bytes": res["flens"][0] if len(names) == 1 and res["flens"][0] else None,
                   "bytes_per_step_per_gpu": bps,
                   "parallelism": f"shard-by-iteration x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "frac_of_guide_achievable": round(achieved / HBM_ACHIEVABLE_GBPS, 4),
                     "frac_of_measured_write_peak": round(achieved / peak_probe, 4) if peak_probe else None,
                     "traffic": mix_traffic if mix_traffic is not None else pmc_traffic(a.pmc, names, a.packets),
                     "traffic_source": os.path.relpath(a.pmc, ROOT),
                     "kernel": res["kernels"][0] if len(names) == 1 else res["kernels"],
                     "kernel_ms_avg": round(res["span_ms_per_step"], 5),
                     "per_launch_ms": res["per_launch_ms"],
                     "algorithmic_bytes_per_launch": bps},
    }
    if res["counters"] is not None:
        line["global_counters"] = res["counters"]
        line["global_counters"]["sequences"] = names
    line.update(extra)
    if world == 1 and a.cpu_seconds > 0:
        line["cpu_baseline"] = cpu_baseline(names[0], a.cpu_seconds)
        line["cpu_baseline"]["host"] = host_cpu()
        # the other CPU-path points SURVEY.md §8d names: one thread, the integer-only
        # form, and configs[0] (static 64-B UDP, fixed source, one thread)
        short = max(1.0, a.cpu_seconds / 4)
        line["cpu_baseline_variants"] = {
            "faithful_1_thread": cpu_baseline(names[0], short, threads=1),
            "faithful_16_threads": cpu_baseline(names[0], short, threads=16),
            "lean_usable_threads": cpu_baseline(names[0], short, faithful=False),
            "configs0_c1_udp_static_64_1_thread": dict(
                cpu_baseline("c1_udp_static_64", short, threads=1),
                af_xdp_send="not measured: no AF_XDP socket / CAP_NET_RAW on the GPU host (BASELINE.md §3)")}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
