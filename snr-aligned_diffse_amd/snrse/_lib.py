"""ctypes binding of libsnrse_hip.so (include/snrse.h) — the only route to the kernels.

There is deliberately no CPU fallback: if the library or a HIP device is missing, every
op raises.  Tensors cross the boundary as raw device pointers (`data_ptr()`); launches go
on torch's current HIP stream so torch events / graphs see them.
"""
from __future__ import annotations

import ctypes as C
import os

# torch bundles its own libamdhip64.so.7; importing it first makes our library bind to that
# same HIP runtime (same SONAME) instead of pulling /opt/rocm's copy into the process as a
# second runtime whose device pointers and streams torch could not use.
import torch  # noqa: F401

from .build import LIB

F32, BF16, F16, F64, F32X3 = 0, 1, 2, 3, 4

_vp, _i, _f, _u64, _ll = C.c_void_p, C.c_int, C.c_float, C.c_uint64, C.c_longlong

# name -> argtypes (all return int status except the housekeeping ones)
SIGNATURES = {
    "snrse_upfirdn2d": [_vp, _vp, _vp] + [_i] * 15 + [_vp],
    "snrse_conv2d": [_vp, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _i, _vp, _i, _f,
                     _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _i, _i, _i, _vp],
    "snrse_gn_scale_shift": [_vp, _i, _vp, _i, _i, _i, _vp, _vp, _i, _f, _vp, _vp, _vp],
    "snrse_gn_stats": [_vp, _vp, _i, _vp, _i, _i, _i, _vp, _vp, _i, _vp],
    "snrse_gn_apply": [_vp, _i, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _f, _i, _i, _vp, _i, _vp],
    "snrse_set_option": [C.c_char_p, _i],
    "snrse_get_option": [C.c_char_p, _vp],
    "snrse_attention": [_vp, _vp, _i, _i, _i, _i, _vp],
    "snrse_temb_mlp": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp],
    "snrse_temb_dense": [_vp, _vp, _vp, _vp, _i, _i, _i, _vp],
    "snrse_temb_gfp_dense": [_vp, _vp, _vp, _vp, _vp, _i, _i, _vp],
    "snrse_input_pack": [_vp, _vp, _i, _i, _i, _vp, _vp, _i, _vp],
    "snrse_score_update": [_vp, _i, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp],
    "snrse_sde_update": [_vp, _vp, _vp, _vp, _u64, _u64, _vp, _i, _i, _vp, _vp, _vp],
    "snrse_axpby_noise": [_vp, _vp, _vp, _u64, _u64, _vp, _i, _i, _vp, _vp],
    "snrse_stft": [_vp, _i, _i, _vp, _f, _i, _i, _vp, _vp],
    "snrse_absmax": [_vp, _i, _i, _vp, _vp],
    "snrse_energy_ratios": [_vp, _vp, _vp, _i, _i, _vp, _vp],
    "snrse_input_conv": [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp],
    "snrse_input_conv_x3": [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp],
    "snrse_spec_transform": [_vp, _vp, C.c_longlong, _i, _vp],
    "snrse_snrnet": [_vp, _i, _i] + [_vp] * 17 + [_vp, _vp, _vp],
    "snrse_istft": [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp],
    "snrse_gn_resample": [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _i, _vp],
    "snrse_gn_act": [_vp, _i, _vp, _i, _i, _i, _vp, _vp, _i, _vp, _i, _vp],
    "snrse_set_workspace": [_vp, C.c_size_t],
    # caller-owned launch contexts (snrse_ctx: switches, split-K workspace, read-backs)
    "snrse_ctx_set_workspace": [_vp, _vp, C.c_size_t],
    "snrse_ctx_set_option": [_vp, C.c_char_p, _i],
    "snrse_ctx_get_option": [_vp, C.c_char_p, _vp],
    "snrse_ctx_probe_begin": [_vp, _i],
    "snrse_ctx_probe_read": [_vp, _vp, _vp, _i, _vp],
    # consistency-training step (csrc/train.hip)
    "snrse_conv_wgrad": [_vp, _i, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp],
    "snrse_conv_wgrad_x3": [_vp, _i, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp],
    "snrse_chan_sum": [_vp, _i, _i, _i, _vp, _vp, _f, _vp],
    "snrse_gn_moments": [_vp, _i, _vp, _i, _i, _i, _i, _f, _vp, _vp, _vp],
    "snrse_gn_backward": [_vp, _i, _vp, _i, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp],
    "snrse_bgemm": [_vp, _ll, _ll, _ll, _vp, _ll, _ll, _ll, _vp, _ll, _ll, _ll, _vp, _i, _i, _i, _i, _f, _f, _vp],
    "snrse_softmax_rows": [_vp, _vp, _ll, _i, _f, _vp],
    "snrse_softmax_bwd_rows": [_vp, _vp, _vp, _ll, _i, _f, _vp],
    "snrse_silu": [_vp, _vp, _ll, _vp],
    "snrse_silu_bwd": [_vp, _vp, _vp, _ll, _i, _vp],
    "snrse_axpby": [_vp, _vp, _ll, _f, _f, _vp],
    "snrse_scale_rows": [_vp, _vp, _vp, _i, _ll, _i, _vp],
    "snrse_gfp": [_vp, _vp, _i, _i, _vp, _vp],
    "snrse_ct_perturb": [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp],
    "snrse_ct_loss": [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp],
    "snrse_adam_ema": [_vp, _vp, _vp, _i, _f, _f, _f, _f, _f, _f, _f, _vp],
}
HOUSEKEEPING = {"snrse_abi_version": ([], _i), "snrse_build_id": ([], C.c_char_p), "snrse_error_string": ([_i], C.c_char_p),
                "snrse_device_name": ([C.c_char_p, _i], _i), "snrse_snrnet_workspace": ([_i, _i], C.c_size_t),
                "snrse_ctx_create": ([], _vp), "snrse_ctx_destroy": ([_vp], None)}

_lib = None


def load(path: str | None = None) -> C.CDLL:
    """Load (once) and type the library.  Raises OSError when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("SNRSE_LIB", LIB)
    if not os.path.exists(path):
        raise OSError(f"libsnrse_hip.so not found at {path}: run __graft_entry__.build() "
                      "(or python -m snrse.build) first; there is no CPU fallback")
    lib = C.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _i
    for name, (args, res) in HOUSEKEEPING.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    # SNRSE_OPTS="name=value,..." sets library options at load time (A/B runs of bench.py / tools)
    for kv in filter(None, os.environ.get("SNRSE_OPTS", "").split(",")):
        k, v = kv.split("=")
        check(lib.snrse_set_option(k.strip().encode(), int(v)), f"snrse_set_option({k})")
    return lib


def exported_symbols():
    return list(SIGNATURES) + list(HOUSEKEEPING)


def check(rc: int, what: str):
    if rc != 0:
        msg = load().snrse_error_string(rc)
        raise RuntimeError(f"{what} failed: {msg.decode() if msg else rc} (code {rc})")


def call(name: str, *args):
    lib = load()
    n = len(SIGNATURES[name])
    if len(args) != n:  # ctypes would silently pass surplus arguments as C ints
        raise TypeError(f"{name} takes {n} arguments, {len(args)} given")
    check(getattr(lib, name)(*args), name)
