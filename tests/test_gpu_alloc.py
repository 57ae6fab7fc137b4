"""Frame buffers of >= 64 MiB are physical chunks mapped in order into one reserved address range
(fb_alloc, csrc/pbgpu.cpp): builds into them equal builds into a hipMalloc'ed
buffer (PBGPU_ALLOC=malloc) byte for byte, for a fixed-length and a packed variable-length
sequence (the latter also writes its offsets into a chunk-mapped array), UMEM landing reads them,
and freeing returns the memory (repeated 3-GiB allocations do not accumulate)."""
import hashlib

import numpy as np
import pytest

import pb_configs as pc
from pbgpu import GpuContext, Sequence

pytestmark = pytest.mark.gpu


def _build(monkeypatch, name, n, malloc):
    if malloc:
        monkeypatch.setenv("PBGPU_ALLOC", "malloc")
    else:
        monkeypatch.delenv("PBGPU_ALLOC", raising=False)
    with GpuContext(0) as ctx:
        ctx.load_sequence(0, Sequence.from_config(pc.get(name)), pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(0, n))
        ctx.build(0, 777, n, fb)
        ctx.sync()
        data = fb.packed()
        off = fb.offsets()
        umem = np.zeros(64 * 4096, dtype=np.uint8)
        lens = fb.to_umem(umem, 4096, n - 64, 64)
        p, b = ctx.counters(1)
        fb.free()
    return (hashlib.sha256(data.tobytes()).hexdigest(), hashlib.sha256(off.tobytes()).hexdigest(),
            umem.tobytes(), lens.tobytes(), int(p[0]), int(b[0]))


@pytest.mark.parametrize("chunk_mb,dma", [(None, False), (2, False), (None, True)])
@pytest.mark.parametrize("name,n", [("c2_udp_64", 1 << 22), ("c3_udp_var", 1 << 19)])
def test_chunk_mapped_buffer_matches_hipmalloc(monkeypatch, name, n, chunk_mb, dma):
    """The default 64-MiB chunks, 2-MiB ones (PBGPU_ALLOC_CHUNK_MB), and UMEM landing through DMA
    copies from them (PBGPU_UMEM_DMA=1) instead of the mapped scatter kernel."""
    if chunk_mb:
        monkeypatch.setenv("PBGPU_ALLOC_CHUNK_MB", str(chunk_mb))
    if dma:
        monkeypatch.setenv("PBGPU_UMEM_DMA", "1")
    a = _build(monkeypatch, name, n, malloc=False)
    b = _build(monkeypatch, name, n, malloc=True)
    assert a == b
    assert a[4] == n


def _free_bytes():
    """hipMemGetInfo of the HIP runtime libpbgpu.so uses (torch brings a runtime of its own)."""
    import ctypes as C

    hip = C.CDLL("libamdhip64.so", mode=C.RTLD_GLOBAL)
    free, total = C.c_size_t(), C.c_size_t()
    assert hip.hipMemGetInfo(C.byref(free), C.byref(total)) == 0
    return int(free.value)


def test_chunk_mapped_buffers_are_released(monkeypatch):
    monkeypatch.delenv("PBGPU_ALLOC", raising=False)
    n = 3 * (1 << 30) // 64
    with GpuContext(0) as ctx:
        ctx.load_sequence(0, Sequence.from_config(pc.get("c2_udp_64")), pc.SEED_BASE)
        fb = ctx.alloc_frames(*ctx.build_size(0, n))
        fb.free()
        free0 = _free_bytes()
        for k in range(6):
            fb = ctx.alloc_frames(*ctx.build_size(0, n))
            ctx.build(0, k * n, n, fb)
            ctx.sync()
            fb.free()
        free1 = _free_bytes()
    assert abs(free0 - free1) < (256 << 20), (free0, free1)
