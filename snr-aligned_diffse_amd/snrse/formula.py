"""Deterministic "formula" tensors: weights, test inputs and injected noise.

The reference's trained checkpoints are not available offline (README.md:53 of the
reference), and its default init zeroes most of the network (`init_scale=0` makes
Conv_1 / NIN_3 / pyramid convs ~1e-10, layers.py:88-91).  Parity and benchmarks
therefore run on weights produced by a counter-hash formula: any process (the
golden-vector generator that drives the reference modules, the CPU oracle, the HIP
path on the GPU box) regenerates bit-identical float32 values from a parameter's
name and shape, so no weights are committed.

Value of element j of tensor `name`:  u = splitmix64(crc32(name) * C1 + j) mapped to
[-1, 1) with 24 bits of mantissa, then scaled by a per-kind rule (`param_scale`).
"""
from __future__ import annotations

import math
import zlib

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + _GOLD
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
        x = x ^ (x >> np.uint64(31))
    return x


def _seed(name: str) -> np.uint64:
    return np.uint64(zlib.crc32(name.encode("utf-8")) & 0xFFFFFFFF)


def uniform(name: str, n: int) -> np.ndarray:
    """n float64 values in [-1, 1), exactly representable in float32."""
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64) + _seed(name) * np.uint64(0x100000001B3)
    bits = _splitmix(idx) >> np.uint64(40)  # 24 random bits
    return bits.astype(np.float64) * (2.0 / 16777216.0) - 1.0


def normal(name: str, n: int) -> np.ndarray:
    """n float64 standard normals (Box-Muller on two formula streams)."""
    u1 = (uniform(name + "#u1", n) + 1.0) * 0.5  # [0, 1)
    u2 = (uniform(name + "#u2", n) + 1.0) * 0.5
    u1 = 1.0 - u1  # (0, 1]
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)


def normal_tensor(name: str, shape, complex_: bool = False):
    """float32 (or complex64 with each part ~ N(0, 1/2), like torch.randn_like on
    a complex tensor) formula normals as a numpy array."""
    n = int(np.prod(shape))
    if complex_:
        re = normal(name + "#re", n)
        im = normal(name + "#im", n)
        z = (re + 1j * im) / math.sqrt(2.0)
        return z.astype(np.complex64).reshape(shape)
    return normal(name, n).astype(np.float32).reshape(shape)


def param_scale_kind(name: str, shape, siblings: dict) -> tuple[str, float]:
    """Scale rule for one state-dict entry (kind, bound)."""
    leaf = name.rsplit(".", 1)[-1]
    nd = len(shape)
    if leaf == "W" and nd == 1:  # GaussianFourierProjection.W  (layerspp.py:37)
        return "gfp", 16.0
    if "blstm" in name:  # torch LSTM default init bound 1/sqrt(hidden)
        return "lstm", 1.0 / math.sqrt(128.0)
    if leaf == "weight" and nd == 1:  # GroupNorm gamma
        return "gn_gamma", 0.1
    if leaf == "bias" and nd == 1:
        sib = name[: -len("bias")] + "weight"
        if sib in siblings and len(siblings[sib]) == 1:
            return "gn_beta", 0.1
        return "bias", 0.05
    if leaf == "b" and nd == 1:  # NIN bias
        return "bias", 0.05
    if leaf == "W" and nd == 2:  # NIN weight stored (in, out)  (layers.py:546-551)
        fan_in, fan_out = shape[0], shape[1]
    elif nd == 2:  # Linear (out, in)
        fan_in, fan_out = shape[1], shape[0]
    else:  # Conv2d (out, in, kh, kw)
        rf = int(np.prod(shape[2:]))
        fan_in, fan_out = shape[1] * rf, shape[0] * rf
    # variance_scaling(1, 'fan_avg', 'uniform') of layers.py:59-91, at scale 1
    return "weight", math.sqrt(3.0 / ((fan_in + fan_out) / 2.0))


def formula_param(name: str, shape, siblings: dict) -> np.ndarray:
    kind, s = param_scale_kind(name, shape, siblings)
    u = uniform(name, int(np.prod(shape))).reshape(shape)
    if kind == "gn_gamma":
        v = 1.0 + s * u
    else:
        v = s * u
    return v.astype(np.float32)


def formula_state_dict(shapes: dict) -> dict:
    """{name: shape} -> {name: float32 numpy array} (ordering preserved)."""
    return {k: formula_param(k, tuple(v), shapes) for k, v in shapes.items()}
