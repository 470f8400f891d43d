"""WAV decoding for the Specs front-end (the reference reads clips with `torchaudio.load`,
data_module.py:48-49; torchaudio is not part of this build).

`load(path)` -> (float32 tensor [channels, frames], sample_rate) with torchaudio's default
normalisation (`normalize=True`): signed 16/24/32-bit PCM divided by 2^(bits-1), unsigned
8-bit PCM as (v - 128) / 128, IEEE float 32/64 passed through (as float32).  RIFF/RIFX-free
little-endian WAVE only (PCM = 1, IEEE_FLOAT = 3, EXTENSIBLE = 0xFFFE with either sub-format);
anything else raises ValueError.  The file is memory-mapped and decoded with one numpy view.
"""
from __future__ import annotations

import struct

import numpy as np
import torch

_PCM, _FLOAT, _EXT = 1, 3, 0xFFFE


def _chunks(buf: memoryview):
    off = 12
    while off + 8 <= len(buf):
        cid, size = struct.unpack_from("<4sI", buf, off)
        yield cid, off + 8, size
        off += 8 + size + (size & 1)


def read_wav(path: str):
    """-> (numpy float32 [frames, channels], sample_rate)."""
    raw = np.memmap(path, dtype=np.uint8, mode="r")
    buf = memoryview(raw)
    if len(buf) < 12 or bytes(buf[0:4]) != b"RIFF" or bytes(buf[8:12]) != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    fmt = data = None
    for cid, off, size in _chunks(buf):
        if cid == b"fmt ":
            fmt = struct.unpack_from("<HHIIHH", buf, off)
            if fmt[0] == _EXT and size >= 40:
                sub = struct.unpack_from("<H", buf, off + 24)[0]
                fmt = (sub,) + fmt[1:]
        elif cid == b"data":
            data = (off, min(size, len(buf) - off))
    if fmt is None or data is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, sr, _, align, bits = fmt
    if ch < 1 or align != ch * ((bits + 7) // 8):
        raise ValueError(f"{path}: inconsistent fmt chunk")
    off, size = data
    n = size // align
    b = raw[off:off + n * align]
    if tag == _PCM and bits == 16:
        x = b.view("<i2").astype(np.float32) / 32768.0
    elif tag == _PCM and bits == 32:
        x = (b.view("<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    elif tag == _PCM and bits == 24:
        t = b.reshape(-1, 3).astype(np.int32)
        v = t[:, 0] | (t[:, 1] << 8) | (t[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / 8388608.0
    elif tag == _PCM and bits == 8:
        x = (b.astype(np.float32) - 128.0) / 128.0
    elif tag == _FLOAT and bits == 32:
        x = b.view("<f4").astype(np.float32)
    elif tag == _FLOAT and bits == 64:
        x = b.view("<f8").astype(np.float32)
    else:
        raise ValueError(f"{path}: unsupported WAVE format tag {tag} / {bits} bit")
    return x.reshape(n, ch), sr


def load(path: str):
    """torchaudio.load(path) equivalent -> (float32 tensor [channels, frames], sample_rate)."""
    x, sr = read_wav(path)
    return torch.from_numpy(np.ascontiguousarray(x.T)), sr


def write_wav(path: str, x: np.ndarray, sr: int = 16000, bits: int = 16):
    """Write [frames] or [frames, channels] float audio as PCM16 or float32 (test fixtures, outputs)."""
    x = np.asarray(x)
    x = x[:, None] if x.ndim == 1 else x
    ch = x.shape[1]
    if bits == 16:
        data = np.clip(np.round(x * 32768.0), -32768, 32767).astype("<i2").tobytes()
        tag = _PCM
    elif bits == 32:
        data = x.astype("<f4").tobytes()
        tag = _FLOAT
    else:
        raise ValueError("bits must be 16 (PCM) or 32 (float)")
    align = ch * bits // 8
    hdr = struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + len(data), b"WAVE", b"fmt ", 16, tag, ch, sr, sr * align,
                      align, bits, b"data", len(data))
    with open(path, "wb") as f:
        f.write(hdr + data)
