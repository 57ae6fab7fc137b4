"""bench.py's N-rank plumbing on CPU (gloo, world size 2) with a stub build context: the
weak-scaling iteration ranges each rank builds per step (disjoint over ranks and steps,
pb_dist.step_first_iter), the counters all-reduced over the ranks (the reference's global
total_pckts / total_bytes, sequence.c:12-14, 633-642) and the wall time MAX-reduced, for one
sequence and for configs[4]'s three in one batch call.  The GPU side of the same path is
tests/test_gpu_bench.py (torchrun, RCCL at world 1; two ranks sharing one GPU over gloo)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Frames:
    def __init__(self, flen):
        self.fixed_len = flen


class _Buf:
    def __init__(self, flen):
        self.f = _Frames(flen)
        self.freed = False

    def free(self):
        self.freed = True


class StubCtx:
    """The GpuContext calls run_configs makes; builds are recorded, counters follow them."""
    TIMING_LAUNCH, TIMING_SPAN = 0, 1
    FLEN = {"c2_udp_64": 64, "c4_tcp_syn": 60, "c5_icmp_echo": 98}

    def __init__(self, rank, slow_s):
        self.rank, self.slow_s = rank, slow_s
        self.names, self.builds, self.batches = {}, [], 0
        self.p = np.zeros(4, dtype=np.uint64)
        self.b = np.zeros(4, dtype=np.uint64)
        self.launches, self.timed, self.mode = 0, False, None

    def load_sequence(self, i, seq, seed):
        self.names[i] = seq

    def build_size(self, i, n):
        return n, n * 128

    def alloc_frames(self, nf, nb):
        return _Buf(self.flen_of(len(self.names) - 1))

    def flen_of(self, i):
        return self.flens[i]

    def set_timing(self, mode):
        self.mode = mode

    def build(self, i, first, n, buf):
        self.builds.append((i, first, n))
        self.p[i] += n
        self.b[i] += n * buf.f.fixed_len
        self.launches += 1

    def build_batch(self, parts):
        self.batches += 1
        for i, first, n, buf in parts:
            self.builds.append((i, first, n))
            self.p[i] += n
            self.b[i] += n * buf.f.fixed_len
        self.launches += 1

    def sync(self):
        if self.timed:  # the slow rank's timed region ends later
            import time

            time.sleep(self.slow_s)
            self.timed = False

    def kernel_time(self):
        n, self.launches = self.launches, 0
        return 0.5 * n, n

    def kernel_times(self):
        n, self.launches = self.launches, 0
        return np.full(n, 0.5)

    def counters(self, nseq):
        return self.p[:nseq].copy(), self.b[:nseq].copy()

    def kernel_name(self, i):
        return f"stub<{i}>"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, names, q):
    import sys

    sys.path[:0] = [ROOT, os.path.join(ROOT, "pb-af-xdp_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), PB_DIST_BACKEND="gloo")
    import bench
    from test_bench_dist import StubCtx

    dist, w, r, local = bench.init_dist(world)
    ctx = StubCtx(rank, slow_s=0.3 if rank == 1 else 0.0)
    ctx.flens = [StubCtx.FLEN[nm] for nm in names]
    steps, warmup, n = 3, 2, 1000
    # the first counters read opens the timed region; the stub's next sync (after the timed
    # steps) is the one that sleeps on the slow rank
    real_counters = ctx.counters
    calls = {"n": 0}

    def counters(nseq):
        calls["n"] += 1
        if calls["n"] == 1:
            ctx.timed = True  # the next sync (after the timed steps) sleeps on the slow rank
        return real_counters(nseq)

    ctx.counters = counters
    res = bench.run_configs(ctx, names, n, steps, warmup, r, w, dist, local, ramp_s=0.0, launch_reps=2)
    dist.destroy_process_group()
    q.put((rank, ctx.builds, ctx.batches, res["counters"], res["wall_s"], res["kernels"], res["packets_per_step"]))


def _run(names, world=2):
    c = mp.get_context("spawn")
    q = c.Queue()
    port = _free_port()
    procs = [c.Process(target=_worker, args=(r, world, port, names, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _check(res, names, world=2):
    steps, warmup, n = 3, 2, 1000
    nseq = len(names)
    seen = set()
    walls = []
    for rank, builds, batches, counters, wall, kernels, pps in res:
        # warm-up steps, then the timed steps, then the per-launch pass: step s of rank r builds
        # iterations [(s world + r) n, + n) of every sequence
        per_seq = [[(f, m) for i, f, m in builds if i == k] for k in range(nseq)]
        for k in range(nseq):
            want = [((s * world + rank) * n, n) for s in range(warmup + steps + 2)]
            assert per_seq[k] == want, (rank, k, per_seq[k][:4])
            for f, m in per_seq[k]:
                assert (k, f) not in seen
                seen.add((k, f))
        assert counters == {"packets": [steps * n * world] * nseq,
                            "bytes": [steps * n * world * StubCtx.FLEN[nm] for nm in names]}
        assert pps == n * nseq
        walls.append(wall)
        if nseq > 1:
            assert batches == warmup + steps + 2 and kernels[0].startswith("pb_batch_kernel")
    assert len(set(walls)) == 1 and walls[0] >= 0.3  # MAX over ranks: the slow rank's wall
    assert len(seen) == nseq * world * (warmup + steps + 2)


def test_bench_world2_one_sequence():
    names = ["c2_udp_64"]
    _check(_run(names), names)


def test_bench_world2_mix_batch():
    names = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"]
    _check(_run(names), names)


@pytest.mark.parametrize("world", [4, 8])
def test_bench_more_ranks(world):
    """The driver's 4- and 8-GPU runs rehearsed on CPU: every rank's iteration ranges disjoint,
    counters all-reduced to world x steps x n, the wall the slowest rank's."""
    names = ["c2_udp_64", "c4_tcp_syn", "c5_icmp_echo"] if world == 4 else ["c2_udp_64"]
    _check(_run(names, world), names, world)
