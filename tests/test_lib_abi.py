"""CPU checks of the C-ABI library: it builds for gfx950, loads, and exports every entry
point declared in include/snrse.h (no kernel is launched here)."""
import ctypes
import os
import re

from conftest import ROOT


def test_header_symbols_exported():
    from snrse import _lib, build
    path = build.build_library()
    lib = ctypes.CDLL(path)
    with open(os.path.join(ROOT, "include", "snrse.h")) as f:
        hdr = f.read()
    declared = sorted(set(re.findall(r"\b(snrse_\w+)\s*\(", hdr)))
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib.exported_symbols())
    _lib.load(path)
    assert _lib.load().snrse_abi_version() == 1
    assert _lib.load().snrse_error_string(1)


def test_no_cpu_fallback():
    import pytest
    import torch
    from snrse import ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.gn_stats(torch.zeros(1, 4, 4, 128))
