"""pbgpu — Python binding of libpbgpu.so (include/pbgpu.h) and of the
sequence/config surface (include/pb_config.h).

`Sequence.from_config(dict)` accepts a sequence object in the reference's JSON
schema (README.md:216-575: "eth", "ip", "udp", "tcp", "icmp", "payloads", ...)
with the reference's documented defaults, so a PB-AF-XDP config drives the GPU
build unchanged.  `GpuContext` wraps one device context.

The frame builder only exists on the GPU: if libpbgpu.so is missing, or was
built without a usable device at run time, every build call raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, Optional, Sequence as Seq

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libpbgpu.so")

MAX_PAYLOADS = 64
MAX_RANGES = 64
MAX_SEQUENCES = 256

PAYLOAD_STREAM = 0
PAYLOAD_LITERAL = 1
FOLD_FULL = 0
FOLD_SINGLE = 1

ERRORS = {
    0: "ok",
    -2: "ENOENT",
    -5: "EIO",
    -12: "ENOMEM",
    -19: "ENODEV",
    -22: "EINVAL",
    -28: "ENOSPC",
    -95: "ENOTSUP",
}


class PbError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {ERRORS.get(code, code)} ({code})")
        self.code = code


# ---------------------------------------------------------------- ABI types
class PayloadOpt(C.Structure):
    _fields_ = [
        ("exact", C.c_char_p),
        ("is_static", C.c_uint8),
        ("is_file", C.c_uint8),
        ("is_string", C.c_uint8),
        ("min_len", C.c_uint16),
        ("max_len", C.c_uint16),
    ]


class _Eth(C.Structure):
    _fields_ = [("src_mac", C.c_char_p), ("dst_mac", C.c_char_p)]


class _Ip(C.Structure):
    _fields_ = [
        ("src_ip", C.c_char_p),
        ("dst_ip", C.c_char_p),
        ("protocol", C.c_char_p),
        ("tos", C.c_uint8),
        ("csum", C.c_uint8),
        ("min_ttl", C.c_uint8),
        ("max_ttl", C.c_uint8),
        ("min_id", C.c_uint16),
        ("max_id", C.c_uint16),
        ("ranges", C.c_char_p * MAX_RANGES),
        ("range_count", C.c_uint16),
    ]


class _Udp(C.Structure):
    _fields_ = [("src_port", C.c_uint16), ("dst_port", C.c_uint16)]


class _Tcp(C.Structure):
    _fields_ = [("src_port", C.c_uint16), ("dst_port", C.c_uint16)] + [
        (n, C.c_uint8) for n in ("syn", "ack", "psh", "fin", "rst", "urg", "ece", "cwr")
    ]


class _Icmp(C.Structure):
    _fields_ = [("code", C.c_uint8), ("type", C.c_uint8)]


class SequenceT(C.Structure):
    """pb_sequence_t (include/pb_config.h)."""

    _fields_ = [
        ("interface", C.c_char_p),
        ("block", C.c_uint8),
        ("track", C.c_uint8),
        ("max_pckts", C.c_uint64),
        ("max_bytes", C.c_uint64),
        ("pps", C.c_uint64),
        ("bps", C.c_uint64),
        ("time", C.c_uint64),
        ("threads", C.c_uint16),
        ("delay", C.c_uint64),
        ("l4_csum", C.c_uint8),
        ("eth", _Eth),
        ("ip", _Ip),
        ("udp", _Udp),
        ("tcp", _Tcp),
        ("icmp", _Icmp),
        ("pls", PayloadOpt * MAX_PAYLOADS),
        ("pl_cnt", C.c_uint16),
    ]


class Rules(C.Structure):
    _fields_ = [("payload_rule", C.c_uint8), ("iph_fold", C.c_uint8)]


class Frames(C.Structure):
    """pbgpu_frames (include/pbgpu.h)."""

    _fields_ = [
        ("data", C.c_void_p),
        ("offsets", C.c_void_p),
        ("reserved", C.c_void_p),
        ("scan_tmp", C.c_void_p),
        ("capacity_frames", C.c_uint64),
        ("capacity_bytes", C.c_uint64),
        ("seq_idx", C.c_uint16),
        ("first_iter", C.c_uint64),
        ("n_frames", C.c_uint64),
        ("fixed_len", C.c_uint32),
        ("total_bytes", C.c_uint64),
    ]


# ------------------------------------------------------------- sequences
def _b(s: Optional[str]) -> Optional[bytes]:
    return None if s is None else s.encode()


class Sequence:
    """Owns a SequenceT plus the byte strings its char* fields point at."""

    def __init__(self) -> None:
        self.c = SequenceT()
        self._keep: list = []
        self.set_defaults()

    def _str(self, s: Optional[str]) -> Optional[bytes]:
        b = _b(s)
        if b is not None:
            self._keep.append(b)
        return b

    def set_defaults(self) -> None:
        """Defaults documented in README.md:216-575 (PB-Common clear_sequence)."""
        c = self.c
        c.block = 1
        c.track = 0
        c.delay = 1000000
        c.l4_csum = 1
        c.ip.csum = 1
        c.ip.min_ttl = 64
        c.ip.max_ttl = 64
        c.ip.min_id = 0
        c.ip.max_id = 64000

    @classmethod
    def from_config(cls, cfg: dict) -> "Sequence":
        """A sequence object in the reference's JSON schema (README.md:216-575)."""
        s = cls()
        c = s.c
        c.interface = s._str(cfg.get("interface"))
        for key, field in (("block", "block"), ("track", "track"), ("maxpckts", "max_pckts"),
                           ("maxbytes", "max_bytes"), ("pps", "pps"), ("bps", "bps"), ("time", "time"),
                           ("threads", "threads"), ("delay", "delay"), ("l4csum", "l4_csum")):
            if key in cfg and cfg[key] is not None:
                setattr(c, field, int(cfg[key]))
        eth = cfg.get("eth", {}) or {}
        c.eth.src_mac = s._str(eth.get("smac"))
        c.eth.dst_mac = s._str(eth.get("dmac"))
        ip = cfg.get("ip", {}) or {}
        c.ip.src_ip = s._str(ip.get("sip"))
        c.ip.dst_ip = s._str(ip.get("dip"))
        c.ip.protocol = s._str(ip.get("protocol"))
        if "tos" in ip:
            c.ip.tos = int(ip["tos"])
        if "csum" in ip:
            c.ip.csum = int(ip["csum"])
        ttl = ip.get("ttl", {}) or {}
        if "min" in ttl:
            c.ip.min_ttl = int(ttl["min"])
        if "max" in ttl:
            c.ip.max_ttl = int(ttl["max"])
        idd = ip.get("id", {}) or {}
        if "min" in idd:
            c.ip.min_id = int(idd["min"])
        if "max" in idd:
            c.ip.max_id = int(idd["max"])
        ranges = ip.get("ranges", []) or []
        if len(ranges) > MAX_RANGES:
            raise ValueError("too many ranges")
        for i, r in enumerate(ranges):
            c.ip.ranges[i] = s._str(r)
        c.ip.range_count = len(ranges)
        udp = cfg.get("udp", {}) or {}
        c.udp.src_port = int(udp.get("sport", 0))
        c.udp.dst_port = int(udp.get("dport", 0))
        tcp = cfg.get("tcp", {}) or {}
        c.tcp.src_port = int(tcp.get("sport", 0))
        c.tcp.dst_port = int(tcp.get("dport", 0))
        for fl in ("syn", "ack", "psh", "fin", "rst", "urg", "ece", "cwr"):
            setattr(c.tcp, fl, int(tcp.get(fl, 0)))
        icmp = cfg.get("icmp", {}) or {}
        c.icmp.code = int(icmp.get("code", 0))
        c.icmp.type = int(icmp.get("type", 0))
        pls = cfg.get("payloads", []) or []
        if len(pls) > MAX_PAYLOADS:
            raise ValueError("too many payloads")
        for i, p in enumerate(pls):
            po = c.pls[i]
            po.exact = s._str(p.get("exact"))
            po.is_static = int(p.get("isstatic", 0))
            po.is_file = int(p.get("isfile", 0))
            po.is_string = int(p.get("isstring", 0))
            ln = p.get("length", {}) or {}
            po.min_len = int(ln.get("min", 0))
            po.max_len = int(ln.get("max", 0))
        c.pl_cnt = len(pls)
        return s

    @property
    def frames_per_iter(self) -> int:
        return max(1, int(self.c.pl_cnt))


def parse_mac(s: Optional[str]) -> bytes:
    if not s:
        return bytes(6)
    return bytes(int(x, 16) for x in s.split(":"))


# --------------------------------------------------------------- library
_libs = {}


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libpbgpu.so (raises if it is absent: there is no CPU fallback).
    Other paths load other builds side by side (compile-time A/B probes)."""
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run `make -C pb-af-xdp_amd`): the GPU path has no fallback")
    lib = C.CDLL(path)
    P, U8P, U64P = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)
    FP = C.POINTER(Frames)
    sig = {
        "pbgpu_open": (C.c_int, [C.c_int, C.POINTER(P)]),
        "pbgpu_close": (None, [P]),
        "pbgpu_strerror": (C.c_char_p, [C.c_int]),
        "pbgpu_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "pbgpu_load_sequence": (C.c_int, [P, C.c_uint16, C.POINTER(SequenceT), U8P, U8P, C.POINTER(Rules),
                                          C.c_uint64]),
        "pbgpu_build_size": (C.c_int, [P, C.c_uint16, C.c_uint64, U64P, U64P]),
        "pbgpu_frames_alloc": (C.c_int, [P, C.c_uint64, C.c_uint64, C.POINTER(FP)]),
        "pbgpu_frames_free": (None, [P, FP]),
        "pbgpu_build": (C.c_int, [P, C.c_uint16, C.c_uint64, C.c_uint64, FP]),
        "pbgpu_build_batch": (C.c_int, [P, C.c_uint32, C.POINTER(C.c_uint16), U64P, U64P, C.POINTER(FP)]),
        "pbgpu_sync": (C.c_int, [P]),
        "pbgpu_frames_total": (C.c_int, [P, FP, U64P]),
        "pbgpu_frames_offsets": (C.c_int, [P, FP]),
        "pbgpu_copy_packed": (C.c_int, [P, FP, P, C.c_uint64, C.c_uint64]),
        "pbgpu_copy_offsets": (C.c_int, [P, FP, U64P]),
        "pbgpu_copy_to_umem": (C.c_int, [P, FP, P, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32,
                                         C.POINTER(C.c_uint16)]),
        "pbgpu_host_register": (C.c_int, [P, P, C.c_size_t]),
        "pbgpu_host_unregister": (C.c_int, [P, P]),
        "pbgpu_counters": (C.c_int, [P, U64P, U64P, C.c_int]),
        "pbgpu_kernel_time": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]),
        "pbgpu_set_timing": (C.c_int, [P, C.c_int]),
        "pbgpu_kernel_times": (C.c_int, [P, C.POINTER(C.c_double), C.c_uint32, C.POINTER(C.c_uint32)]),
        "pbgpu_fill_probe": (C.c_int, [P, C.c_uint64, C.c_uint32, C.POINTER(C.c_double)]),
        "pbgpu_fill_probe_ex": (C.c_int, [P, C.c_uint64, C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
        "pbgpu_fill_probe_at": (C.c_int, [P, C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_double)]),
        "pbgpu_fill_shape_name": (C.c_char_p, [C.c_int]),
        "pbgpu_abi_size": (C.c_size_t, [C.c_int]),
        "pbgpu_kernel_name": (C.c_int, [P, C.c_uint16, C.c_char_p, C.c_size_t]),
    }
    for name, (res, args) in sig.items():
        if path != LIB_PATH and not hasattr(lib, name):
            continue  # an older build loaded for an A/B lacks the newer entry points
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _libs[path] = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise PbError(rc, what)


def _u8(b: Optional[bytes]):
    if b is None:
        return None
    return (C.c_uint8 * 6).from_buffer_copy(b)


class FrameBuffer:
    """A device-resident pbgpu_frames allocation."""

    def __init__(self, ctx: "GpuContext", ptr):
        self.ctx = ctx
        self.ptr = ptr

    @property
    def f(self) -> Frames:
        return self.ptr.contents

    def total_bytes(self) -> int:
        t = C.c_uint64()
        _check(self.ctx.lib.pbgpu_frames_total(self.ctx.h, self.ptr, C.byref(t)), "frames_total")
        return int(t.value)

    def fill_offsets(self) -> None:
        """offsets[] on the device (variable length: expanded from the 4-B form on first use)."""
        _check(self.ctx.lib.pbgpu_frames_offsets(self.ctx.h, self.ptr), "frames_offsets")

    def offsets(self) -> np.ndarray:
        n = int(self.f.n_frames)
        out = np.empty(n + 1, dtype=np.uint64)
        _check(self.ctx.lib.pbgpu_copy_offsets(self.ctx.h, self.ptr, out.ctypes.data_as(C.POINTER(C.c_uint64))),
               "copy_offsets")
        return out

    def packed(self) -> np.ndarray:
        total = self.total_bytes()
        out = np.empty(total, dtype=np.uint8)
        if total:
            _check(self.ctx.lib.pbgpu_copy_packed(self.ctx.h, self.ptr, out.ctypes.data, 0, total), "copy_packed")
        return out

    def frames(self) -> list:
        data = self.packed()
        off = self.offsets()
        return [data[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]

    def to_umem(self, umem: np.ndarray, slot: int, first_frame: int, n: int, first_slot: int = 0) -> np.ndarray:
        lens = np.empty(n, dtype=np.uint16)
        _check(self.ctx.lib.pbgpu_copy_to_umem(self.ctx.h, self.ptr, umem.ctypes.data, slot, first_slot,
                                               first_frame, n, lens.ctypes.data_as(C.POINTER(C.c_uint16))),
               "copy_to_umem")
        return lens

    def free(self) -> None:
        if self.ptr is not None:
            self.ctx.lib.pbgpu_frames_free(self.ctx.h, self.ptr)
            self.ptr = None


class GpuContext:
    """One pbgpu_ctx (one GPU)."""

    def __init__(self, device: int = 0, lib_path: str = LIB_PATH):
        self.lib = load_library(lib_path)
        h = C.c_void_p()
        _check(self.lib.pbgpu_open(device, C.byref(h)), f"pbgpu_open({device})")
        self.h = h
        self._seqs = {}

    def close(self) -> None:
        if self.h:
            self.lib.pbgpu_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load_sequence(self, idx: int, seq: Sequence, seed_base: int, smac: Optional[bytes] = None,
                      dmac: Optional[bytes] = None, payload_rule: int = PAYLOAD_STREAM,
                      iph_fold: int = FOLD_FULL) -> None:
        rules = Rules(payload_rule, iph_fold)
        _check(self.lib.pbgpu_load_sequence(self.h, idx, C.byref(seq.c), _u8(smac), _u8(dmac), C.byref(rules),
                                            C.c_uint64(seed_base)), "load_sequence")
        self._seqs[idx] = seq

    def build_size(self, idx: int, n_iter: int):
        mf, mb = C.c_uint64(), C.c_uint64()
        _check(self.lib.pbgpu_build_size(self.h, idx, n_iter, C.byref(mf), C.byref(mb)), "build_size")
        return int(mf.value), int(mb.value)

    def alloc_frames(self, capacity_frames: int, capacity_bytes: int) -> FrameBuffer:
        p = C.POINTER(Frames)()
        _check(self.lib.pbgpu_frames_alloc(self.h, capacity_frames, capacity_bytes, C.byref(p)), "frames_alloc")
        return FrameBuffer(self, p)

    def build(self, idx: int, first_iter: int, n_iter: int, fb: FrameBuffer) -> None:
        _check(self.lib.pbgpu_build(self.h, idx, first_iter, n_iter, fb.ptr), "build")

    def build_batch(self, parts) -> None:
        """parts: (idx, first_iter, n_iter, FrameBuffer) tuples, built as one pbgpu_build_batch
        call (configs[4]'s three sequences: one fused launch)."""
        n = len(parts)
        idx = (C.c_uint16 * n)(*[p[0] for p in parts])
        fi = (C.c_uint64 * n)(*[p[1] for p in parts])
        ni = (C.c_uint64 * n)(*[p[2] for p in parts])
        outs = (C.POINTER(Frames) * n)(*[p[3].ptr for p in parts])
        _check(self.lib.pbgpu_build_batch(self.h, n, idx, fi, ni, outs), "build_batch")

    def sync(self) -> None:
        _check(self.lib.pbgpu_sync(self.h), "sync")

    def counters(self, n_seq: int):
        p = np.zeros(n_seq, dtype=np.uint64)
        b = np.zeros(n_seq, dtype=np.uint64)
        _check(self.lib.pbgpu_counters(self.h, p.ctypes.data_as(C.POINTER(C.c_uint64)),
                                       b.ctypes.data_as(C.POINTER(C.c_uint64)), n_seq), "counters")
        return p, b

    TIMING_LAUNCH, TIMING_SPAN = 0, 1

    def set_timing(self, mode: int) -> None:
        """PBGPU_TIMING_LAUNCH: an event pair per launch; PBGPU_TIMING_SPAN: one
        span per kernel_time() call (no per-launch events)."""
        _check(self.lib.pbgpu_set_timing(self.h, mode), "set_timing")

    def kernel_time(self):
        ms, n = C.c_double(), C.c_uint32()
        _check(self.lib.pbgpu_kernel_time(self.h, C.byref(ms), C.byref(n)), "kernel_time")
        return float(ms.value), int(n.value)

    def kernel_times(self, cap: int = 4096) -> np.ndarray:
        """TIMING_LAUNCH: each launch's device time (ms) since the last call."""
        ms = np.zeros(cap, dtype=np.float64)
        n = C.c_uint32()
        _check(self.lib.pbgpu_kernel_times(self.h, ms.ctypes.data_as(C.POINTER(C.c_double)), cap, C.byref(n)),
               "kernel_times")
        return ms[:min(cap, int(n.value))]

    def fill_probe(self, nbytes: int, reps: int) -> float:
        ms = C.c_double()
        _check(self.lib.pbgpu_fill_probe(self.h, nbytes, reps, C.byref(ms)), "fill_probe")
        return float(ms.value)

    FILL_SHAPES = 15  # PBGPU_FILL_SHAPES

    def fill_probe_shapes(self, nbytes: int, reps: int):
        """Every write-probe shape's mean ms per launch {name: ms} and the fastest's name."""
        ms = (C.c_double * self.FILL_SHAPES)()
        best = C.c_int()
        _check(self.lib.pbgpu_fill_probe_ex(self.h, nbytes, reps, ms, C.byref(best)), "fill_probe_ex")
        names = [self.lib.pbgpu_fill_shape_name(i).decode() for i in range(self.FILL_SHAPES)]
        return {names[i]: float(ms[i]) for i in range(self.FILL_SHAPES)}, names[best.value]

    def fill_probe_at(self, fb: "FrameBuffer", nbytes: int, reps: int):
        """Every write-probe shape's mean ms per launch over a frame buffer's own memory."""
        ms = (C.c_double * self.FILL_SHAPES)()
        _check(self.lib.pbgpu_fill_probe_at(self.h, fb.f.data, nbytes, reps, ms), "fill_probe_at")
        names = [self.lib.pbgpu_fill_shape_name(i).decode() for i in range(self.FILL_SHAPES)]
        return {names[i]: float(ms[i]) for i in range(self.FILL_SHAPES)}

    def kernel_name(self, idx: int) -> str:
        buf = C.create_string_buffer(96)
        _check(self.lib.pbgpu_kernel_name(self.h, idx, buf, 96), "kernel_name")
        return buf.value.decode()

    def build_frames(self, idx: int, first_iter: int, n_iter: int) -> list:
        """Convenience: build into a fresh buffer and return the frames as bytes."""
        mf, mb = self.build_size(idx, n_iter)
        fb = self.alloc_frames(mf, mb)
        try:
            self.build(idx, first_iter, n_iter, fb)
            self.sync()
            return fb.frames()
        finally:
            fb.free()


def device_count() -> int:
    lib = load_library()
    n = C.c_int()
    lib.pbgpu_device_count(C.byref(n))
    return int(n.value)
