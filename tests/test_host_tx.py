"""The host TX path on the CPU (no GPU): the libbpf-free AF_XDP ring protocol
(host/xsk_ring.c: send_packet / complete_tx, af_xdp.c:25-53, 178-241) on the
in-memory loopback, and the seq_send worker loop (host/sequence_gpu.c) with a
CPU stand-in for the GPU builder (tests/host_stub.c): the max_pckts quota across
threads, max_bytes, time, pps / bps / delay pacing (sequence.c:389-431,
655-684), the per-sequence thread fan-out (sequence.c:741), the stop request
and the end-of-run lines (sequence.c:779-815)."""
import ctypes as C
import os
import subprocess
import threading
import time

import numpy as np
import pytest

import pb_configs as pc
from cmdline_binding import OurCmd
from pbgpu import Sequence, SequenceT

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "pb-af-xdp_amd", "lib")
BUILD = os.path.join(ROOT, "tests", "_build")
STUB = os.path.join(BUILD, "libpbhost_stub.so")


@pytest.fixture(scope="module")
def libs():
    os.makedirs(BUILD, exist_ok=True)
    # built under a per-process name and renamed into place, so parallel test workers
    # (pytest -n) never load a half-written library
    tmp = f"{STUB}.{os.getpid()}"
    subprocess.run(["gcc", "-O2", "-Wall", "-shared", "-fPIC", "-pthread", "-o", tmp,
                    os.path.join(ROOT, "tests", "host_stub.c"), "-L" + LIBDIR, "-lpbhost",
                    "-Wl,-rpath," + LIBDIR], check=True)
    os.replace(tmp, STUB)
    host = C.CDLL(os.path.join(LIBDIR, "libpbhost.so"))
    stub = C.CDLL(STUB)
    host.seq_send.argtypes = [C.c_char_p, SequenceT, C.c_uint16, OurCmd]
    host.seq_send.restype = None
    host.pb_shutdown_stats.argtypes = [C.c_void_p]
    host.pb_sequence_totals.argtypes = [C.c_uint16, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    host.pb_sequence_tx_stats.argtypes = [C.c_uint16] + [C.POINTER(C.c_uint64)] * 3
    host.cmd_line_af_xdp_defaults.argtypes = [C.POINTER(OurCmd)]
    stub.ring_stress.argtypes = [C.c_uint32, C.c_uint64, C.POINTER(C.c_uint64)]
    stub.stub_recorded.restype = C.c_uint64
    stub.stub_recorded.argtypes = [C.c_void_p] * 4 + [C.c_uint64]
    stub.stub_record.argtypes = [C.c_uint64]
    stub.stub_times.argtypes = [C.c_void_p, C.c_uint64]
    yield host, stub
    stub.stub_uninstall()
    host.pb_set_tx_hook(None, None)


# ---------------------------------------------------------------- ring protocol


class XdpDesc(C.Structure):
    _fields_ = [("addr", C.c_uint64), ("len", C.c_uint32), ("options", C.c_uint32)]


class Ring(C.Structure):
    _fields_ = [("cached_prod", C.c_uint32), ("cached_cons", C.c_uint32), ("mask", C.c_uint32), ("size", C.c_uint32),
                ("producer", C.POINTER(C.c_uint32)), ("consumer", C.POINTER(C.c_uint32)),
                ("flags", C.POINTER(C.c_uint32)), ("ring", C.c_void_p)]


class Xsk(C.Structure):
    _fields_ = [("fd", C.c_int), ("umem", C.c_void_p), ("n_frames", C.c_uint32), ("frame_size", C.c_uint32),
                ("tx", Ring), ("cq", Ring), ("fq", Ring), ("next_slot", C.c_uint32), ("outstanding_tx", C.c_uint32),
                ("need_wakeup", C.c_uint32), ("wakeups", C.c_uint64), ("completed", C.c_uint64),
                ("maps", C.c_void_p * 3), ("map_len", C.c_size_t * 3), ("loop_mem", C.c_void_p),
                ("loop_auto", C.c_int), ("loop_sink", C.c_void_p), ("loop_ctx", C.c_void_p), ("batch", C.c_uint32),
                ("loop_hold", C.c_uint32), ("slot_base", C.c_uint32), ("scq", C.c_void_p), ("thread", C.c_uint32)]


def _loopback(host, n, fs=4096):
    umem = np.zeros(n * fs + 4096, dtype=np.uint8)
    base = (umem.ctypes.data + 4095) & ~4095
    x = Xsk()
    assert host.pb_xsk_loopback(C.byref(x), C.c_void_p(base), n, fs) == 0
    return x, umem


def test_ring_reserve_submit_consume_complete(libs):
    host, _ = libs
    host.pb_ring_prod_reserve.restype = C.c_uint32
    host.pb_ring_tx_desc.restype = C.POINTER(XdpDesc)
    host.pb_xsk_loop_consume.restype = C.c_uint32
    host.pb_xsk_complete.restype = C.c_uint32
    host.pb_xsk_free_slots.restype = C.c_uint32
    x, _keep = _loopback(host, 8)
    x.loop_auto = 0
    idx = C.c_uint32()
    # the TX ring holds exactly `size` entries
    assert host.pb_ring_prod_reserve(C.byref(x.tx), 5, C.byref(idx)) == 5 and idx.value == 0
    assert host.pb_ring_prod_reserve(C.byref(x.tx), 4, C.byref(idx)) == 0
    assert host.pb_ring_prod_reserve(C.byref(x.tx), 3, C.byref(idx)) == 3 and idx.value == 5
    for i in range(8):
        d = host.pb_ring_tx_desc(C.byref(x.tx), i).contents
        d.addr, d.len = i * 4096, 60 + i
    host.pb_ring_prod_submit(C.byref(x.tx), 8)
    assert x.tx.producer[0] == 8
    # the kernel side takes 3, completes them; the producer sees 3 free entries again
    assert host.pb_xsk_loop_consume(C.byref(x), 3, None, None) == 3
    assert x.tx.consumer[0] == 3 and x.cq.producer[0] == 3
    assert host.pb_ring_prod_reserve(C.byref(x.tx), 3, C.byref(idx)) == 3 and idx.value == 8
    # indices wrap: entry 8 is slot 0 of the ring
    d = host.pb_ring_tx_desc(C.byref(x.tx), 8).contents
    assert C.addressof(d) == x.tx.ring
    host.pb_xsk_close(C.byref(x))


def test_send_fills_descriptors_and_reaps_completions(libs):
    host, _ = libs
    host.pb_xsk_free_slots.restype = C.c_uint32
    x, _keep = _loopback(host, 16)
    lens = (C.c_uint16 * 16)(*range(100, 116))
    # loopback with the kernel side run at every wakeup: each send completes at once
    for rnd in range(5):
        assert host.pb_xsk_send(C.byref(x), lens, 11) == 0
        assert x.outstanding_tx == 0 and x.completed == 11 * (rnd + 1)
        assert x.next_slot == (11 * (rnd + 1)) % 16
    assert x.wakeups == 5
    # without a consumer the UMEM slots run out: the sender is refused, not overwritten
    x.loop_auto = 0
    assert host.pb_xsk_send(C.byref(x), lens, 16) == 0
    assert host.pb_xsk_free_slots(C.byref(x)) == 0
    assert host.pb_xsk_send(C.byref(x), lens, 1) == -28  # -ENOSPC
    host.pb_xsk_close(C.byref(x))


@pytest.mark.parametrize("n_frames,total", [(8, 5000), (64, 40000), (4096, 200000)])
def test_ring_protocol_with_kernel_on_another_thread(libs, n_frames, total):
    """Producer and consumer on different threads: every frame arrives once, in
    order, with its descriptor's length; every descriptor completes."""
    _, stub = libs
    w = C.c_uint64()
    assert stub.ring_stress(n_frames, total, C.byref(w)) == 0
    assert w.value > 0


def test_af_xdp_socket_setup_fails_cleanly_without_privilege(libs):
    host, _ = libs
    x = Xsk()
    umem = np.zeros(4096 * 4096 + 4096, dtype=np.uint8)
    base = (umem.ctypes.data + 4095) & ~4095
    rc = host.pb_xsk_open(C.byref(x), b"lo", 0, C.c_void_p(base), 4096, 4096, 0, 8, -1, 0, 4096, 0, None, 0)
    # a negative errno (no AF_XDP / CAP_NET_RAW in this container), or a bound socket
    assert rc <= 0
    if rc == 0:
        host.pb_xsk_close(C.byref(x))
    assert host.pb_xsk_open(C.byref(x), b"pbnodev0", 0, C.c_void_p(base), 4096, 4096, 0, 8, -1, 0, 4096, 0, None,
                            0) == -19  # -ENODEV
    # a shared-UMEM socket's slot range must lie inside the UMEM
    assert host.pb_xsk_open(C.byref(x), b"lo", 1, C.c_void_p(base), 2048, 4096, 0, 0, 3, 4096, 4096, 0, None, 0) == -22
    # slots that do not divide the registered chunk, or a UMEM that is not whole chunks
    assert host.pb_xsk_open(C.byref(x), b"lo", 0, C.c_void_p(base), 4096, 96, 4096, 8, -1, 0, 4096, 0, None, 0) == -22
    assert host.pb_xsk_open(C.byref(x), b"lo", 0, C.c_void_p(base), 64, 64, 8192, 8, -1, 0, 64, 0, None, 0) == -22


def test_shared_umem_socket_on_the_owners_queue_needs_the_shared_ring(libs):
    """xsk_bind lets an XDP_SHARED_UMEM socket keep its own fill / completion rings only
    on another queue or device; on the owner's queue it must take the owner's rings (a
    shared buffer pool).  pb_xsk_open refuses that combination without a shared completion
    ring (pb_xsk_shared_cq_t) before any socket is made; seq_send now gives --sharedumem
    --queue with several threads that ring, so the sequence gets as far as the socket (which
    this container cannot open: no AF_XDP / CAP_NET_RAW)."""
    host, _ = libs
    x = Xsk()
    umem = np.zeros(4096 * 4096 + 4096, dtype=np.uint8)
    base = (umem.ctypes.data + 4095) & ~4095
    # a valid slot range (2048 slots from 2048 of 4096), shared fd, the owner's queue 5, no ring
    assert host.pb_xsk_open(C.byref(x), b"lo", 5, C.c_void_p(base), 2048, 4096, 0, 0, 3, 2048, 4096, 5, None,
                            1) == -22
    assert x.fd == 0 and x.umem is None  # refused before any socket was made
    r = _run(libs, _cfg(maxpckts=1000, delay=0, threads=2), shared_umem=1, queue=5, queue_set=1, tx=b"xsk")
    assert r["err"] != 0 and r["pckts"] == 0  # the socket open fails here, not a refusal up front


@pytest.mark.parametrize("threads,hold", [(3, 0), (4, 7), (2, 0)])
def test_sharedumem_one_queue_shares_the_completion_ring(libs, monkeypatch, threads, hold):
    """--sharedumem --queue 0 with several threads (af_xdp.c:412-443: every socket on the
    owner's queue): all threads' completions arrive on one ring, reaped under a lock and
    credited to the thread whose slot range holds each address.  On the loopback every frame
    is submitted once, the quota is exact and every descriptor completes; PB_LOOP_HOLD keeps
    some frames in flight so reaps interleave across threads."""
    host = libs[0]
    if hold:
        monkeypatch.setenv("PB_LOOP_HOLD", str(hold))
    r = _run(libs, _cfg(maxpckts=30000, delay=0, threads=threads), gpu_batch=1000, shared_umem=1, queue=0,
             queue_set=1)
    assert r["err"] == 0 and r["pckts"] == 30000 and r["seen"] == 30000
    # (which threads send depends on when each starts: one that starts late may find the quota
    # claimed, as in test_maxpckts_quota_is_exact_across_threads)
    assert len(np.unique(r["k"])) == 30000 and set(np.unique(r["thread"])) <= set(range(threads))
    assert (r["len"] != 0xFFFF).all()  # every descriptor's frame intact in its slot
    d, c, wk = C.c_uint64(), C.c_uint64(), C.c_uint64()
    host.pb_sequence_tx_stats(0, C.byref(d), C.byref(c), C.byref(wk))
    assert d.value == 30000 and c.value == 30000
    u = C.c_uint64()
    host.pb_sequence_umems(0, C.byref(u))
    assert u.value == 1


def test_shared_completion_ring_credits_each_thread(libs):
    """pb_xsk_shared_cq_t on its own, no threads: three queues on one UMEM submit 5, 9 and 3
    frames, the loopback's kernel side posts all 17 to the one shared completion ring, and the
    first queue to reap takes them all off it, crediting each address's slot range: every queue
    then completes exactly its own frames, the later ones from their credits alone."""
    host = libs[0]
    host.pb_xsk_complete.restype = C.c_uint32
    host.pb_xsk_loop_consume.restype = C.c_uint32
    q = (C.c_uint8 * 8192)()  # the C struct (mutex, ring, credits) fits well inside
    slots, fs = 16, 4096
    assert host.pb_xsk_scq_init(q, 3, slots, fs, 1) == 0
    umem = np.zeros(3 * slots * fs + 4096, dtype=np.uint8)
    base = (umem.ctypes.data + 4095) & ~4095
    xs = [Xsk() for _ in range(3)]
    sends = [5, 9, 3]
    lens = (C.c_uint16 * slots)(*([60] * slots))
    for t, x in enumerate(xs):
        assert host.pb_xsk_loopback_shared(C.byref(x), C.c_void_p(base), fs, q, t) == 0
        assert x.slot_base == t * slots
        x.loop_auto = 0  # the kernel side runs below, by hand
        assert host.pb_xsk_send(C.byref(x), lens, sends[t]) == 0
        assert x.outstanding_tx == sends[t] and x.completed == 0
    for x in xs:
        assert host.pb_xsk_loop_consume(C.byref(x), 64, None, None) == sends[xs.index(x)]
    for t, x in enumerate(xs):
        assert host.pb_xsk_complete(C.byref(x), 64) == sends[t]
        assert x.completed == sends[t] and x.outstanding_tx == 0
    for x in xs:
        host.pb_xsk_close(C.byref(x))
    host.pb_xsk_scq_free(q)


def test_gpu_range_past_the_device_count_is_refused_up_front(libs):
    """--gpu I --gpus N names GPUs I..I+N-1: with fewer present, seq_send refuses the sequence
    before it takes a slot or starts a thread (pbgpu_open would fail on the missing ones
    thread by thread); a range that fits runs."""
    cfg = _cfg(maxpckts=64, delay=0, threads=2)
    for gpus, first in ((3, 0), (2, 1), (1, 2)):
        r = _run(libs, cfg, devices=2, gpus=gpus, gpu_first=first)
        assert r["err"] == -19 and r["seen"] == 0 and r["pckts"] == 0, (gpus, first, r["err"])
    r = _run(libs, cfg, devices=2, gpus=2)
    assert r["err"] == 0 and r["pckts"] == 64


# ---------------------------------------------------------------- worker loop


def _cmd(host, **kw):
    c = OurCmd()
    host.cmd_line_af_xdp_defaults(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def _seq(cfg):
    s = Sequence.from_config(cfg)
    return s


def _run(libs, cfg, seqc=1, cap=1 << 20, devices=None, **cmdkw):
    host, stub = libs
    host.pb_reset()
    stub.stub_install()
    if devices is not None:
        stub.stub_set_devices(devices)
    assert stub.stub_record(cap) == 0
    s = _seq(cfg)
    t0 = time.perf_counter()
    host.seq_send(b"lo", s.c, seqc, _cmd(host, **cmdkw))
    err = host.pb_shutdown_stats(None)
    dt = time.perf_counter() - t0
    p, b = C.c_uint64(), C.c_uint64()
    host.pb_sequence_totals(0, C.byref(p), C.byref(b))
    n = min(cap, 1 << 22)
    k = np.zeros(n, dtype=np.uint64)
    i, ln, th = (np.zeros(n, dtype=np.uint16) for _ in range(3))
    seen = stub.stub_recorded(k.ctypes.data, i.ctypes.data, ln.ctypes.data, th.ctypes.data, n)
    m = min(seen, n)
    t = np.zeros(m, dtype=np.float64)
    stub.stub_times(t.ctypes.data, m)
    return {"err": err, "pckts": p.value, "bytes": b.value, "dt": dt, "seen": seen, "k": k[:m], "i": i[:m],
            "len": ln[:m], "thread": th[:m], "t": t, "seq": s}


def _cfg(min_len=22, max_len=22, **kw):
    c = pc.c2_udp_64()
    c["payloads"] = [{"length": {"min": min_len, "max": max_len}}]
    c.update(kw)
    return c


def test_single_thread_sends_iterations_in_order(libs):
    r = _run(libs, _cfg(maxpckts=10000, delay=0), gpu_batch=3000)
    assert r["err"] == 0 and r["pckts"] == 10000 and r["seen"] == 10000
    assert np.array_equal(r["k"], np.arange(10000, dtype=np.uint64))
    assert (r["len"] == 64).all() and r["bytes"] == 64 * 10000


@pytest.mark.parametrize("threads,gpus", [(2, 2), (3, 1), (8, 2)])
def test_maxpckts_quota_is_exact_across_threads(libs, threads, gpus):
    """The max_pckts quota is claimed per batch: the sequence sends exactly
    max_pckts frames over all threads / GPUs, every one a distinct iteration of
    the threads' shards (the reference overshoots by up to a batch per thread)."""
    maxp = 123457
    r = _run(libs, _cfg(0, 900, maxpckts=maxp, delay=0, threads=threads), gpus=gpus, gpu_batch=5000)
    assert r["err"] == 0 and r["pckts"] == maxp and r["seen"] == maxp
    assert len(np.unique(r["k"])) == maxp
    # thread t sends iterations of its shard: (step * threads + t) * batch + j
    assert ((r["k"] // 5000) % threads == r["thread"]).all()
    assert r["bytes"] == int(r["len"].astype(np.int64).sum())
    # (a thread that starts late may find the quota already claimed: no per-thread share is promised)


def test_maxpckts_with_several_payloads_rounds_to_whole_iterations(libs):
    cfg = _cfg(maxpckts=1001, delay=0)
    cfg["payloads"] = [{"length": {"min": 10, "max": 10}}, {"length": {"min": 30, "max": 30}},
                       {"length": {"min": 50, "max": 50}}]
    r = _run(libs, cfg, gpu_batch=100)
    assert r["pckts"] == 1002  # 334 whole iterations of 3 frames
    assert np.array_equal(np.bincount(r["i"].astype(np.int64)), [334, 334, 334])


@pytest.mark.parametrize("threads", [1, 4])
def test_maxbytes_stops_at_the_byte_budget(libs, threads):
    maxb = 3_000_000
    r = _run(libs, _cfg(0, 1400, maxbytes=maxb, delay=0, threads=threads), gpu_batch=2000)
    assert r["err"] == 0
    # sends until the total reaches max_bytes (sequence.c:668-674): at most one frame over per thread
    assert maxb <= r["bytes"] < maxb + threads * 1500
    assert r["bytes"] == int(r["len"].astype(np.int64).sum()) and r["pckts"] == r["seen"]


def test_time_limit(libs):
    r = _run(libs, _cfg(time=1, delay=100), gpu_batch=1000)
    assert r["err"] == 0 and 0.9 < r["dt"] < 3.0
    assert 1000 < r["pckts"] <= 12000  # ~10k frames at one per 100 us


def test_pps_limit_is_global_over_threads(libs):
    """pps limits the sequence, not each thread (sequence.c:389-431: cur_pps is shared)."""
    r = _run(libs, _cfg(maxpckts=3000, pps=4000, delay=0, threads=3), gpu_batch=100000)
    assert r["pckts"] == 3000
    assert 0.55 < r["dt"] < 1.6  # 3000 frames at 4000 pps: 0.75 s


def test_bps_limit(libs):
    # 64-B frames, 128000 bytes per second: 2000 frames per second
    r = _run(libs, _cfg(maxpckts=1500, bps=128000, delay=0), gpu_batch=100000)
    assert r["pckts"] == 1500
    assert 0.55 < r["dt"] < 1.6


@pytest.mark.parametrize("threads,want_s", [(1, 0.8), (2, 0.4)])
def test_delay_is_per_thread_and_per_packet(libs, threads, want_s):
    """delay sleeps after every packet of every thread (sequence.c:655-659)."""
    r = _run(libs, _cfg(maxpckts=400, delay=2000, threads=threads), gpu_batch=100000)
    assert r["pckts"] == 400
    assert want_s * 0.7 < r["dt"] < want_s * 2 + 0.4


@pytest.mark.parametrize("kw,gap_s", [({"delay": 2000}, 0.002), ({"pps": 2000, "delay": 0}, 0.0005),
                                      ({"bps": 128000, "delay": 0}, 0.0005)])
def test_pacing_spreads_the_frames_of_a_batch(libs, kw, gap_s):
    """Inside a landed batch the frames are submitted when due, one at a time at these rates
    (the reference sleeps `delay` after every packet, sequence.c:655-659): no burst of a whole
    batch then an idle gap, as a launch-granular pacer would send."""
    r = _run(libs, _cfg(maxpckts=300, **kw), gpu_batch=100000)
    assert r["err"] == 0 and r["pckts"] == 300
    d = np.diff(r["t"])
    assert 0.4 * gap_s < np.median(d) < 4 * gap_s, np.median(d)
    # most frames leave on their own (a launch-granular pacer sends 50-200 back to back, then
    # waits: under 2% of its gaps are this long); a sender delayed by the scheduler catches up
    # with a few at once, so the bound leaves room for a loaded machine
    assert (d > 0.3 * gap_s).mean() > 0.5, (d > 0.3 * gap_s).mean()


def test_default_delay_sends_one_frame_per_second_per_thread(libs):
    """The README default delay (1,000,000 us) means one packet per second per thread."""
    host, stub = libs
    host.pb_reset()
    stub.stub_install()
    stub.stub_record(100)
    s = _seq(_cfg(delay=1000000, threads=2, block=0))
    t0 = time.perf_counter()
    host.seq_send(b"lo", s.c, 3, _cmd(host))  # not blocking: returns at once
    assert time.perf_counter() - t0 < 0.5
    time.sleep(1.5)
    host.pb_shutdown_stats(None)  # stops and joins the threads
    dt = time.perf_counter() - t0
    p = C.c_uint64()
    host.pb_sequence_totals(0, C.byref(p), None)
    assert 1.4 < dt < 3.0
    assert 2 <= p.value <= 6  # t = 0 and t = 1 s on each of 2 threads


def test_stop_request_ends_an_unbounded_sequence(libs):
    host, stub = libs
    host.pb_reset()
    stub.stub_install()
    stub.stub_record(1 << 16)
    s = _seq(_cfg(delay=0))
    threading.Timer(0.5, host.pb_request_stop).start()
    t0 = time.perf_counter()
    host.seq_send(b"lo", s.c, 1, _cmd(host, gpu_batch=50000))
    dt = time.perf_counter() - t0
    assert dt < 2.5
    p = C.c_uint64()
    host.pb_sequence_totals(0, C.byref(p), None)
    assert p.value > 0


def test_tx_accounting_and_stats_line(libs, capfd):
    host, _ = libs
    cfg = _cfg(maxpckts=9000, delay=0, track=1, threads=2)
    r = _run(libs, cfg, gpu_batch=2500)
    d, c, w = C.c_uint64(), C.c_uint64(), C.c_uint64()
    host.pb_sequence_tx_stats(0, C.byref(d), C.byref(c), C.byref(w))
    assert d.value == 9000 and c.value == 9000 and w.value > 0
    # the reference's end-of-run lines (sequence.c:786-815) through a config
    class Cfg(C.Structure):
        _fields_ = [("interface", C.c_char_p), ("seq", SequenceT * 256)]

    conf = Cfg()
    conf.seq[0] = r["seq"].c
    capfd.readouterr()
    host.pb_shutdown_stats(C.byref(conf))
    out = capfd.readouterr().out
    assert "Completed 1 sequences!" in out
    assert "[1] Completed sequence with a total of 9000 packets and 576000 bytes." in out


def test_non_blocking_sequences_run_concurrently(libs):
    """block = 0: seq_send returns after starting the threads; the reference joins
    only when block is set or for the last sequence (sequence.c:765)."""
    host, stub = libs
    host.pb_reset()
    stub.stub_install()
    stub.stub_record(1 << 16)
    a = _seq(_cfg(maxpckts=5000, delay=200, block=0))
    b = _seq(_cfg(maxpckts=5000, delay=0, block=1))
    t0 = time.perf_counter()
    host.seq_send(b"lo", a.c, 3, _cmd(host, gpu_batch=1000))
    t_first = time.perf_counter() - t0
    host.seq_send(b"lo", b.c, 3, _cmd(host, gpu_batch=1000))
    p0, p1 = C.c_uint64(), C.c_uint64()
    # the paced sequence is still running: wait (bounded) for its first frames, so a
    # loaded machine cannot stop it before its thread has sent anything
    t1 = time.perf_counter() + 10.0
    while time.perf_counter() < t1:
        host.pb_sequence_totals(0, C.byref(p0), None)
        if p0.value:
            break
        time.sleep(0.005)
    host.pb_shutdown_stats(None)
    host.pb_sequence_totals(0, C.byref(p0), None)
    host.pb_sequence_totals(1, C.byref(p1), None)
    assert t_first < 0.5
    assert p1.value == 5000 and 0 < p0.value <= 5000


# ---------------------------------------------------------------- AF_XDP flags (round 3)


def test_send_submits_in_batches_of_batchsize(libs):
    """--batchsize: descriptors per reserve / submit / complete (send_packet,
    af_xdp.c:184-233); 0 (no --batchsize) submits a whole send at once."""
    host, _ = libs
    lens = (C.c_uint16 * 16)(*range(100, 116))
    for batch, want_wakeups in ((0, 1), (4, 3), (1, 11)):
        x, _keep = _loopback(host, 16)
        x.batch = batch
        assert host.pb_xsk_send(C.byref(x), lens, 11) == 0
        assert x.completed == 11 and x.next_slot == 11 and x.wakeups == want_wakeups
        host.pb_xsk_close(C.byref(x))


def test_batchsize_flag_changes_the_worker_submits(libs):
    host = libs[0]
    w = {}
    for kw in ({}, {"batch_size": 1, "batch_set": 1}, {"batch_size": 64, "batch_set": 1}):
        r = _run(libs, _cfg(maxpckts=6000, delay=0), gpu_batch=3000, **kw)
        assert r["pckts"] == 6000 and np.array_equal(r["k"], np.arange(6000, dtype=np.uint64))
        d, c, wk = C.c_uint64(), C.c_uint64(), C.c_uint64()
        host.pb_sequence_tx_stats(0, C.byref(d), C.byref(c), C.byref(wk))
        w[kw.get("batch_size", 0)] = wk.value
    # one wakeup per submit: per landed chunk (<= 1024 frames), per frame, per 64 frames
    # (landed chunks: 1024, 1024, 952 in the first batch; the second also splits at the ring's wrap)
    assert w[1] == 6000 and 94 <= w[64] <= 100 and w[0] <= 12


def test_sharedumem_gives_the_sequence_one_umem(libs):
    """--sharedumem (af_xdp.c:412-428): the sequence's threads share one UMEM, each
    in its own slot range; without it every thread allocates its own."""
    host = libs[0]
    for shared, want in ((0, 4), (1, 1)):
        r = _run(libs, _cfg(maxpckts=20000, delay=0, threads=4), gpu_batch=1000, shared_umem=shared)
        assert r["err"] == 0 and r["pckts"] == 20000 and len(np.unique(r["k"])) == 20000
        assert (r["len"] != 0xFFFF).all()  # every descriptor's frame intact in its slot
        u = C.c_uint64()
        host.pb_sequence_umems(0, C.byref(u))
        assert u.value == want


def test_maxbytes_cut_never_rewrites_frames_in_flight(libs, monkeypatch):
    """A max_bytes budget that ends inside a landed chunk stops the thread there:
    no further landing may reuse the slots of frames still owned by the NIC (the
    loopback holds PB_LOOP_HOLD descriptors unconsumed, as a slow NIC would)."""
    monkeypatch.setenv("PB_LOOP_HOLD", "3000")
    for maxb in (1_234_567, 3_000_001, 5_432_109):
        r = _run(libs, _cfg(0, 1400, maxbytes=maxb, delay=0), gpu_batch=2000)
        assert r["err"] == 0
        n = r["seen"]
        # every frame the NIC side consumed is the one its descriptor named, in order
        assert np.array_equal(r["k"], np.arange(n, dtype=np.uint64))
        assert (r["len"] != 0xFFFF).all()
        assert maxb <= r["bytes"] < maxb + 1500 and r["pckts"] == n


def test_skb_mode_is_copy_mode_and_refuses_zerocopy(libs):
    host = libs[0]
    host.pb_bind_flags.restype = C.c_uint16
    host.pb_bind_flags.argtypes = [C.POINTER(OurCmd)]
    host.pb_af_xdp_setup.argtypes = [C.POINTER(OurCmd), C.c_int]
    XDP_COPY, XDP_ZEROCOPY, XDP_USE_NEED_WAKEUP = 2, 4, 8
    assert host.pb_bind_flags(C.byref(_cmd(host))) == XDP_USE_NEED_WAKEUP
    assert host.pb_bind_flags(C.byref(_cmd(host, skb_mode=1))) == XDP_COPY | XDP_USE_NEED_WAKEUP
    assert host.pb_bind_flags(C.byref(_cmd(host, skb_mode=1, no_wake_up=1))) == XDP_COPY
    assert host.pb_bind_flags(C.byref(_cmd(host, zero_copy=1))) == XDP_ZEROCOPY | XDP_USE_NEED_WAKEUP
    assert host.pb_af_xdp_setup(C.byref(_cmd(host, skb_mode=1)), 0) == 0
    assert host.pb_af_xdp_setup(C.byref(_cmd(host, skb_mode=1, zero_copy=1)), 0) == -22
    assert host.pb_af_xdp_setup(C.byref(_cmd(host, batch_size=0, batch_set=1)), 0) == -22
    binp = os.path.join(ROOT, "pb-af-xdp_amd", "bin", "pcktbatch-gpu")
    r = subprocess.run([binp, "-z", "--dip", "10.0.0.2", "--skb", "--zerocopy"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "--skb and --zerocopy" in r.stderr


def test_seed_is_drawn_per_run_unless_given(libs):
    """Without --seed every run draws its seed base (CLOCK_BOOTTIME ns, or getrandom
    with --veryrandom), as the reference seeds every iteration from the clock
    (sequence.c:434-441); --seed S replays the same stream."""
    host = libs[0]
    host.pb_resolve_seed.restype = C.c_uint64
    host.pb_resolve_seed.argtypes = [C.POINTER(OurCmd)]
    a, b = _cmd(host), _cmd(host)
    sa = host.pb_resolve_seed(C.byref(a))
    time.sleep(0.001)
    sb = host.pb_resolve_seed(C.byref(b))
    assert sa != sb and a.seed_base == sa and b.seed_base == sb
    r1, r2 = _cmd(host, very_random=1), _cmd(host, very_random=1)
    assert host.pb_resolve_seed(C.byref(r1)) != host.pb_resolve_seed(C.byref(r2))
    s1, s2 = _cmd(host, seed_base=1234, seed_set=1), _cmd(host, seed_base=1234, seed_set=1)
    assert host.pb_resolve_seed(C.byref(s1)) == host.pb_resolve_seed(C.byref(s2)) == 1234


@pytest.mark.parametrize("umem_frames,shared,threads", [(64, 0, 1), (16384, 0, 2), (16384, 1, 4)])
def test_umemframes_sizes_each_umem(libs, umem_frames, shared, threads):
    """--umemframes N: UMEM slots per socket (the reference's NUM_FRAMES, af_xdp.h:23, is
    4096); landings take half of them at a time.  Exact quota, every frame once and intact,
    with private and shared UMEMs."""
    r = _run(libs, _cfg(0, 900, maxpckts=60000, delay=0, threads=threads), gpu_batch=20000,
             umem_frames=umem_frames, shared_umem=shared)
    assert r["err"] == 0 and r["pckts"] == 60000 and r["seen"] == 60000
    assert len(np.unique(r["k"])) == 60000 and (r["len"] != 0xFFFF).all()


def test_umemframes_must_be_a_power_of_two(libs):
    host = libs[0]
    host.pb_af_xdp_setup.argtypes = [C.POINTER(OurCmd), C.c_int]
    for n, ok in ((4096, True), (64, True), (1 << 20, True), (1000, False), (32, False), (1 << 21, False)):
        assert (host.pb_af_xdp_setup(C.byref(_cmd(host, umem_frames=n)), 0) == 0) == ok, n


@pytest.mark.parametrize("slot,shared,threads,lo,hi", [(64, 0, 1, 22, 22), (64, 1, 4, 22, 22), (1024, 0, 2, 0, 900),
                                                       (128, 1, 3, 40, 80)])
def test_umemslot_cuts_the_umem_into_smaller_slots(libs, slot, shared, threads, lo, hi):
    """--umemslot S: the UMEM's 4-KiB chunks cut into slots of S bytes (4096 / S frames per chunk,
    descriptors at slot * S): exact quota, every frame once and intact in its slot, private and
    shared UMEMs (the shared ring credits completions by slot * S)."""
    r = _run(libs, _cfg(lo, hi, maxpckts=70000, delay=0, threads=threads), gpu_batch=20000, umem_slot=slot,
             shared_umem=shared)
    assert r["err"] == 0 and r["pckts"] == 70000 and r["seen"] == 70000
    assert len(np.unique(r["k"])) == 70000 and (r["len"] != 0xFFFF).all()
    assert r["len"].max() <= slot


def test_umemslot_one_queue_shared_ring(libs):
    r = _run(libs, _cfg(maxpckts=40000, delay=0, threads=3), gpu_batch=5000, umem_slot=64, shared_umem=1, queue=0,
             queue_set=1)
    assert r["err"] == 0 and r["pckts"] == 40000 and len(np.unique(r["k"])) == 40000
    assert (r["len"] != 0xFFFF).all()


def test_umemslot_refusals(libs, capfd):
    host = libs[0]
    host.pb_af_xdp_setup.argtypes = [C.POINTER(OurCmd), C.c_int]
    for s, ok in ((0, True), (64, True), (4096, True), (2048, True), (32, False), (96, False), (8192, False)):
        assert (host.pb_af_xdp_setup(C.byref(_cmd(host, umem_slot=s)), 0) == 0) == ok, s
    # at most 2^22 slots per UMEM
    assert host.pb_af_xdp_setup(C.byref(_cmd(host, umem_slot=64, umem_frames=1 << 16)), 0) == 0
    assert host.pb_af_xdp_setup(C.byref(_cmd(host, umem_slot=64, umem_frames=1 << 17)), 0) == -22
    # seq_send refuses a bad slot before the sequence takes a slot; frames longer than the slot
    # fail their landing
    for kw in ({"umem_slot": 96}, {"umem_slot": 64, "umem_frames": 1 << 17}):
        r = _run(libs, _cfg(maxpckts=100, delay=0), **kw)
        assert r["err"] == -22 and r["seen"] == 0
    capfd.readouterr()
    r = _run(libs, _cfg(0, 900, maxpckts=1000, delay=0), umem_slot=256)
    assert r["err"] == -22 and r["pckts"] < 1000
    assert "--umemslot" in capfd.readouterr().err
