"""Multi-rank path on CPU (gloo, world sizes 2 and 8): shard ranges partition the
iteration space, per-rank builds concatenate to the single-rank build, and the
counter all-reduce gives the global totals.  The per-rank builder here is the
oracle (no GPU in this container); the GPU version of the concatenation
invariant is tests/test_gpu_parity.py::test_sharded_builds_concatenate."""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp

import pb_dist


def test_shard_partitions():
    for n in (0, 1, 7, 1000, 2**25 + 3):
        for world in (1, 2, 3, 8):
            got = [pb_dist.shard(5, n, r, world) for r in range(world)]
            assert got[0][0] == 5 and sum(c for _, c in got) == n
            for (a, c), (a2, _) in zip(got, got[1:]):
                assert a + c == a2
    seen = set()
    for s in range(3):
        for r in range(4):
            a = pb_dist.step_first_iter(s, r, 4, 10)
            assert a not in seen
            seen.add(a)
    with pytest.raises(ValueError):
        pb_dist.shard(0, 10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "pb-af-xdp_amd")]
    import torch.distributed as dist

    import oracle_binding as ob
    import pb_configs as pc
    from pbgpu import Sequence

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seq = Sequence.from_config(pc.get("c3_udp_var"))
    first, n = pb_dist.shard(100, 601, rank, world)
    data, off = ob.build(seq, 0, first, n, pc.SEED_BASE)
    gp, gb = pb_dist.allreduce_counters([n], [int(off[-1])])
    objs = [None] * world
    dist.all_gather_object(objs, data.tobytes())
    dist.destroy_process_group()
    q.put((rank, gp[0], gb[0], hashlib.sha256(b"".join(objs)).hexdigest()))


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_world2_shards_concatenate_and_counters_reduce(world):
    """world 2, and the driver's 8-rank case rehearsed (601 iterations: ragged shards)"""
    import oracle_binding as ob
    import pb_configs as pc
    from pbgpu import Sequence

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole, off = ob.build(Sequence.from_config(pc.get("c3_udp_var")), 0, 100, 601, pc.SEED_BASE)
    want = hashlib.sha256(whole.tobytes()).hexdigest()
    for rank, pk, by, digest in res:
        assert pk == 601 and by == int(off[-1]) and digest == want
