"""The C-ABI library (CPU-side checks, no compute): it loads, exports every
entry point include/pbgpu.h declares, the ctypes mirror of the structs matches
the C layout, and without a usable GPU it refuses to run (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

import pbgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("pbgpu.h",):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(pbgpu_[a-z_0-9]+)\s*\(", text))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = pbgpu.load_library()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n


def test_struct_layout_matches_c():
    lib = pbgpu.load_library()
    assert lib.pbgpu_abi_size(0) == C.sizeof(pbgpu.SequenceT)
    assert lib.pbgpu_abi_size(1) == C.sizeof(pbgpu.PayloadOpt)
    assert lib.pbgpu_abi_size(2) == C.sizeof(pbgpu.Frames)
    assert lib.pbgpu_abi_size(3) == pbgpu.SequenceT.ip.offset + pbgpu._Ip.ranges.offset
    assert lib.pbgpu_abi_size(4) == pbgpu.SequenceT.pls.offset
    assert lib.pbgpu_abi_size(5) == pbgpu.SequenceT.pl_cnt.offset
    assert lib.pbgpu_abi_size(6) == pbgpu.Frames.total_bytes.offset
    assert lib.pbgpu_abi_size(99) == 0


def test_error_strings():
    lib = pbgpu.load_library()
    for code in (0, -2, -5, -12, -19, -22, -28, -95):
        assert lib.pbgpu_strerror(code)


def test_open_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pbgpu.PbError) as e:
        pbgpu.GpuContext(0)
    assert e.value.code == -19


def test_null_arguments_rejected():
    lib = pbgpu.load_library()
    assert lib.pbgpu_open(0, None) == -22
    assert lib.pbgpu_build(None, 0, 0, 1, None) == -22
    assert lib.pbgpu_load_sequence(None, 0, None, None, None, None, 0) == -22
    assert lib.pbgpu_build_batch(None, 0, None, None, None, None) == -22
