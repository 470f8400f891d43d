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
    assert _lib.load().snrse_abi_version() == 2
    assert _lib.load().snrse_error_string(1)


def test_no_cpu_fallback():
    import pytest
    import torch
    from snrse import ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.gn_stats(torch.zeros(1, 4, 4, 128))


def _prototypes(hdr):
    """name -> parameter count of every prototype in the header."""
    body = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(snrse_\w+)\s*\(([^;{]*?)\)\s*;", body):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_header_prototypes_match_bindings():
    """Every prototype's parameter count equals its ctypes binding's (a stale binding would pass
    arguments shifted by one, e.g. after the snrse_ctx arguments were added)."""
    from snrse import _lib
    with open(os.path.join(ROOT, "include", "snrse.h")) as f:
        protos = _prototypes(f.read())
    sigs = {k: len(v) for k, v in _lib.SIGNATURES.items()}
    sigs.update({k: len(v[0]) for k, v in _lib.HOUSEKEEPING.items()})
    assert set(protos) == set(sigs)
    bad = {k: (protos[k], sigs[k]) for k in protos if protos[k] != sigs[k]}
    assert not bad, bad


def test_launch_context_host_api():
    """snrse_ctx (host memory only, no GPU call): a new context copies the process default switches,
    has its own values afterwards, reports read-back defaults, rejects unknown names."""
    from snrse import _lib
    lib = _lib.load()
    v = ctypes.c_int(0)
    _lib.call("snrse_set_option", b"splitk_target", 192)
    a = lib.snrse_ctx_create()
    b = lib.snrse_ctx_create()
    try:
        assert a and b and a != b
        _lib.call("snrse_ctx_get_option", a, b"splitk_target", ctypes.addressof(v))
        assert v.value == 192
        _lib.call("snrse_ctx_set_option", a, b"conv_variant", 2)
        _lib.call("snrse_ctx_get_option", b, b"conv_variant", ctypes.addressof(v))
        assert v.value == 0
        _lib.call("snrse_ctx_get_option", a, b"conv_variant", ctypes.addressof(v))
        assert v.value == 2
        _lib.call("snrse_get_option", b"conv_variant", ctypes.addressof(v))
        assert v.value == 0
        for name, want in ((b"last_kernel", 0), (b"last_ksplit", 1), (b"last_chunks", 1), (b"halo_kernel", 5)):
            _lib.call("snrse_ctx_get_option", a, name, ctypes.addressof(v))
            assert v.value == want, name
        assert lib.snrse_ctx_set_option(a, b"no_such_switch", 1) != 0
        assert lib.snrse_ctx_set_workspace(a, None, 16) != 0  # NULL with a size
        assert lib.snrse_ctx_set_workspace(a, None, 0) == 0
    finally:
        lib.snrse_ctx_destroy(a)
        lib.snrse_ctx_destroy(b)
        _lib.call("snrse_set_option", b"splitk_target", 256)
