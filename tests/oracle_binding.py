"""ctypes binding of the CPU oracle (oracle/libpb_oracle.so) — TEST
INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker, never by the product path."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "libpb_oracle.so")

_lib = None


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return ORACLE_LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            build_oracle()
        from pbgpu import SequenceT, Rules  # noqa: E402  (shared ABI types)
        L = C.CDLL(ORACLE_LIB)
        L.pbo_rand_r.restype = C.c_int
        L.pbo_rand_r.argtypes = [C.POINTER(C.c_uint)]
        L.pbo_rand_num.restype = C.c_int
        L.pbo_rand_num.argtypes = [C.c_int, C.c_int, C.c_uint]
        L.pbo_seed.restype = C.c_uint32
        L.pbo_seed.argtypes = [C.c_uint64, C.c_uint16, C.c_uint64]
        L.pbo_build.restype = C.c_int
        L.pbo_build.argtypes = [C.POINTER(SequenceT), C.c_void_p, C.c_void_p, C.c_uint16, C.c_uint64, C.c_uint64,
                                C.c_uint64, C.POINTER(Rules), C.c_int, C.c_void_p, C.c_uint64, C.c_uint32,
                                C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.pbo_build_mt.restype = C.c_int
        L.pbo_build_mt.argtypes = [C.POINTER(SequenceT), C.c_void_p, C.c_void_p, C.c_uint16, C.c_uint64,
                                   C.c_uint64, C.c_uint64, C.POINTER(Rules), C.c_int, C.c_int, C.c_void_p,
                                   C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)]
        L.pbo_iph_csum.restype = C.c_uint16
        L.pbo_iph_csum.argtypes = [C.c_char_p, C.c_int]
        L.pbo_l4_csum.restype = C.c_uint16
        L.pbo_l4_csum.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint8]
        L.pbo_verify_frames.restype = C.c_uint64
        L.pbo_verify_frames.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int]
        _lib = L
    return _lib


def rand_r(seed: int):
    s = C.c_uint(seed)
    r = lib().pbo_rand_r(C.byref(s))
    return r, s.value


def rand_num(lo: int, hi: int, seed: int) -> int:
    return lib().pbo_rand_num(lo, hi, seed)


def seed(seed_base: int, seq_idx: int, k: int) -> int:
    return lib().pbo_seed(seed_base, seq_idx, k)


def _mac(b):
    return None if b is None else (C.c_uint8 * 6).from_buffer_copy(b)


def build(seq, seq_idx: int, first_iter: int, n_iter: int, seed_base: int, payload_rule: int = 0,
          iph_fold: int = 0, faithful: bool = False, smac=None, dmac=None):
    """Oracle frames for iterations [first_iter, first_iter+n_iter): (packed uint8 array, offsets)."""
    from pbgpu import Rules
    fpi = seq.frames_per_iter
    nf = n_iter * fpi
    cap = nf * 65600 if nf * 65600 < (1 << 28) else None
    if cap is None:
        # bounded by the sequence's own maximum frame length
        mx = 54 + max([int(p.max_len) for p in seq.c.pls[:max(1, seq.c.pl_cnt)]] + [0]) + 65536
        cap = nf * mx
    out = np.zeros(cap, dtype=np.uint8)
    offs = np.zeros(nf + 1, dtype=np.uint64)
    n = C.c_uint64()
    tot = C.c_uint64()
    rules = Rules(payload_rule, iph_fold)
    rc = lib().pbo_build(C.byref(seq.c), _mac(smac), _mac(dmac), seq_idx, first_iter, n_iter, seed_base,
                         C.byref(rules), int(faithful), out.ctypes.data, cap, 0, offs.ctypes.data, C.byref(n),
                         C.byref(tot))
    if rc != 0:
        raise RuntimeError(f"pbo_build -> {rc}")
    assert n.value == nf
    return out[: tot.value].copy(), offs


def frames(seq, seq_idx, first_iter, n_iter, seed_base, **kw):
    data, off = build(seq, seq_idx, first_iter, n_iter, seed_base, **kw)
    return [data[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]


def build_slots_mt(seq, seq_idx, first_iter, n_iter, seed_base, nthreads, slot=4096, faithful=True,
                   payload_rule=0, iph_fold=0, out=None, ring=0):
    """Frames into UMEM-geometry slots; ring > 0: each thread reuses its own ring
    of `ring` slots (the reference's per-socket UMEM of NUM_FRAMES frames)."""
    from pbgpu import Rules
    nf = n_iter * seq.frames_per_iter
    if out is None:
        out = np.zeros((nthreads * ring if ring else nf) * slot, dtype=np.uint8)
    tot = C.c_uint64()
    rules = Rules(payload_rule, iph_fold)
    rc = lib().pbo_build_mt(C.byref(seq.c), None, None, seq_idx, first_iter, n_iter, seed_base, C.byref(rules),
                            int(faithful), nthreads, out.ctypes.data, out.nbytes, slot, ring, C.byref(tot))
    if rc != 0:
        raise RuntimeError(f"pbo_build_mt -> {rc}")
    return out, int(tot.value)


def verify_frames(data: np.ndarray, offsets, fixed_len: int, n: int, nthreads: int = 16) -> int:
    """Frames among n whose IPv4 checksum, tot_len or L4 checksum fails (C checker)."""
    off = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    return int(lib().pbo_verify_frames(data.ctypes.data, None if off is None else off.ctypes.data, fixed_len, n,
                                       nthreads))
