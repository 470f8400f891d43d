"""Torch-tensor wrappers over the C-ABI (device pointers + torch's current stream).

Every op requires HIP device tensors and raises otherwise — there is no CPU fallback.

Concurrency contract.  The library's stateful entries (snrse_conv2d, snrse_gn_stats, snrse_input_conv,
snrse_gn_resample) take a caller-owned launch context (snrse_ctx: switches, split-K workspace, read-backs
of the latest launch), so calls through distinct contexts are independent.  Here every host thread has
its own context per device (LaunchContext, thread-local, with its own split-K workspace), the StatsArena
stack is thread-local, and each network keeps one arena per launch stream.  So evaluations issued by
different host threads on different streams run concurrently without sharing mutable state, and one
thread interleaving several streams (snrse.sampler.pc_sample_lockstep) switches to a per-lane context
with use_workspace_lane(lane) before issuing each lane's launches.  set_option() is process-wide policy:
it edits the library's process default and every live context; get_option() reads the calling thread's
current context (so "last_kernel" etc. describe that thread's latest launch).
"""
from __future__ import annotations

import ctypes as C
import itertools
import math
import os
import threading
import weakref

import torch

from . import _lib

F32, BF16, F16 = _lib.F32, _lib.BF16, _lib.F16
INV_SQRT2 = 1.0 / math.sqrt(2.0)
# the 16-bit activation / weight formats of the fast path: fp16 (round 6 default) and bf16 (the same kernels)
H16 = (torch.float16, torch.bfloat16)


def conv_code(act_dtype: torch.dtype, wgt_dtype: torch.dtype) -> int:
    """snrse_conv2d dtype: fp32 activations with bf16 weights are the split-bf16 fp32 GEMM (weights from
    split_weight), else the activations' dtype (weights of the same dtype)."""
    if act_dtype == torch.float32 and wgt_dtype == torch.bfloat16:
        return _lib.F32X3
    if wgt_dtype != act_dtype:
        raise TypeError(f"snrse: conv weights {wgt_dtype} for {act_dtype} activations")
    return code(act_dtype)


def split_weight(w: torch.Tensor) -> torch.Tensor:
    """fp32 packed conv weights [N][K] (K % 32 == 0) -> the SNRSE_F32X3 layout [N][2K] bf16: per 32-element
    K-tile, 32 hi = bf16(w) then 32 lo = bf16(w - hi)."""
    n, k = w.shape
    if k % 32:
        raise ValueError(f"snrse: split weights need K % 32 == 0, got {k}")
    w = w.float().reshape(n, k // 32, 1, 32)
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], 2).reshape(n, 2 * k).contiguous()


def code(dtype: torch.dtype) -> int:
    if dtype == torch.float32:
        return F32
    if dtype == torch.float16:
        return F16
    if dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"snrse: unsupported dtype {dtype}")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _ws_alloc(dev):
    mb = int(os.environ.get("SNRSE_WORKSPACE_MB", "128"))
    return (torch.empty(mb << 18, dtype=torch.float32, device=dev) if mb > 0 else None), mb


_CONTEXTS = weakref.WeakSet()  # every live LaunchContext (set_option reaches all of them)
_CTX_SEQ = itertools.count()
_TLS = threading.local()       # per thread: {device: {lane: LaunchContext}}, current lane per device, arenas


class LaunchContext:
    """A caller-owned snrse_ctx (include/snrse.h) on one device: the library's switches (copied from the
    process default at creation), a split-K workspace of SNRSE_WORKSPACE_MB (default 128; 0 disables K
    splitting) and the read-backs of the latest launch issued through it."""

    def __init__(self, device):
        lib = _lib.load()
        self.device = torch.device(device)
        self.ptr = lib.snrse_ctx_create()
        if not self.ptr:
            raise MemoryError("snrse_ctx_create failed")
        self._lib = lib
        self.ws, mb = _ws_alloc(self.device)
        _lib.call("snrse_ctx_set_workspace", self.ptr, None if self.ws is None else self.ws.data_ptr(),
                  0 if self.ws is None else mb << 20)
        # mirror of the context's "stats_zeroed" switch; snrse_ctx_create copies it from the process default
        self.zeroed = int(bool(self.get_option("stats_zeroed")))
        self.seq = next(_CTX_SEQ)  # creation order (probe_read over several threads' contexts)
        _CONTEXTS.add(self)

    def set_option(self, name, value):
        _lib.call("snrse_ctx_set_option", self.ptr, name.encode(), int(value))
        if name == "stats_zeroed":
            self.zeroed = int(bool(value))

    def get_option(self, name):
        v = C.c_int(0)
        _lib.call("snrse_ctx_get_option", self.ptr, name.encode(), C.addressof(v))
        return v.value

    def __del__(self):
        try:
            self._lib.snrse_ctx_destroy(self.ptr)
        except Exception:
            pass


def _tls_contexts(dev):
    d = getattr(_TLS, "ctx", None)
    if d is None:
        d = _TLS.ctx = {}
        _TLS.lane = {}
    return d.setdefault(torch.device(dev), {})


def context(dev=None, lane=None):
    """The calling thread's current LaunchContext on `dev` (lane: that lane's context, created on first
    use; default: the lane selected by use_workspace_lane, initially 0)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if dev is None else torch.device(dev)
    ctxs = _tls_contexts(dev)
    if lane is None:
        lane = _TLS.lane.get(dev, 0)
    c = ctxs.get(lane)
    if c is None:
        c = ctxs[lane] = LaunchContext(dev)
    return c


def _cx(dev):
    return context(dev).ptr


def use_workspace_lane(lane, dev):
    """Make lane `lane`'s own context (and so its own split-K workspace and read-backs) the calling
    thread's current one on `dev`.  The two-stream sampler (snrse.sampler.pc_sample_lockstep) issues each
    half-batch's launches behind its lane's context, so concurrent split-K GEMMs never share a workspace."""
    dev = torch.device(dev)
    _tls_contexts(dev)
    _TLS.lane[dev] = lane
    context(dev, lane)


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("snrse: HIP device tensor required (no CPU fallback)")
        if t is not None and not t.is_contiguous():
            raise RuntimeError("snrse: contiguous tensor required")


def conv2d(src0, wgt, ksize, cout, bias=None, src1=None, sc=None, sc1=None, sc_wgt=None, temb=None,
           temb_off=0, res=None, out_scale=1.0, comb=None, comb_w=None, comb_b=None, out=None,
           out_f32=False, stats=None, gn=None, gn_act=True):
    """NHWC conv (see snrse_conv2d).  src0 [B,H,W,C0]; returns out [B,H,W,cout].
    temb: [B, R] f32 table of all Dense_0 outputs, this layer's columns start at temb_off.
    stats: optional new_stats() buffer receiving the output's per-channel (sum, sumsq).
    gn: optional (scale, shift) [B, C0+C1] f32 — consume SiLU(GN(x)) (halo path only, see halo_ok)."""
    _dev(src0, src1, wgt, sc, sc1, sc_wgt, bias, res, comb, comb_w, comb_b, temb)
    cx = context(src0.device)
    B, H, W, C0 = src0.shape
    C1 = 0 if src1 is None else src1.shape[3]
    Csc = 0 if sc is None else sc.shape[3]
    Csc1 = 0 if sc1 is None else sc1.shape[3]
    odt = torch.float32 if out_f32 else src0.dtype
    if sc_wgt is not None and sc_wgt.dtype != wgt.dtype:
        raise TypeError("snrse: conv2d wgt and sc_wgt must share one layout (both split or neither)")
    if out is None:
        out = torch.empty(B, H, W, cout, device=src0.device, dtype=odt)
    _stats_zeroed(cx, stats)
    _lib.call("snrse_conv2d", cx.ptr, _ptr(src0), C0, _ptr(src1), C1, B, H, W, ksize, _ptr(wgt), _ptr(sc), Csc,
              _ptr(sc1), Csc1, _ptr(sc_wgt), _ptr(bias), None if temb is None else temb.data_ptr() + 4 * temb_off,
              0 if temb is None else temb.shape[1], _ptr(res), 0 if res is None else res.shape[-1], float(out_scale), _ptr(comb),
              _ptr(comb_w), _ptr(comb_b), out.data_ptr(), cout, out.shape[-1], _ptr(stats),
              None if gn is None else gn[0].data_ptr(), None if gn is None else gn[1].data_ptr(), int(bool(gn_act)),
              conv_code(src0.dtype, wgt.dtype), int(out_f32), _stream())
    return out


def _opt(x, name):
    """A library switch as the launch context of x's device sees it (set_option, SNRSE_OPTS or a
    per-context setting): the shape predicates below mirror the library's own dispatch."""
    return context(x.device).get_option(name)


def get_option(name):
    """A switch or read-back of the calling thread's current context on the current device."""
    return context().get_option(name)


def _probe_contexts(dev, all_threads):
    """This thread's context first, then (all_threads) every other live context on the device by creation."""
    own = context(dev)
    if not all_threads:
        return [own]
    others = sorted((c for c in list(_CONTEXTS) if c is not own and c.device == own.device), key=lambda c: c.seq)
    return [own] + others


def probe_begin(capacity, dev=None, all_threads=False):
    """Bracket the next `capacity` conv2d calls of this thread's current context (all_threads: of every
    context on the device, e.g. the autograd engine's worker thread during a backward) with library-recorded
    HIP events (snrse_ctx_probe_begin; created without the system-scope fence).  capacity 0 stops probing."""
    for cx in _probe_contexts(dev, all_threads):
        _lib.call("snrse_ctx_probe_begin", cx.ptr, int(capacity))


def probe_read(max_calls, dev=None, all_threads=False):
    """(ms per probed conv2d call, kernel generation per call) (snrse_ctx_probe_read): in call order for one
    context; with all_threads, this thread's calls followed by each other context's (the order of a
    training step: forward on the calling thread, then the backward on the autograd worker)."""
    out_ms, out_k = [], []
    for cx in _probe_contexts(dev, all_threads):
        ms = (C.c_float * max_calls)()
        kern = (C.c_int * max_calls)()
        n = C.c_int(0)
        _lib.call("snrse_ctx_probe_read", cx.ptr, C.addressof(ms), C.addressof(kern), int(max_calls),
                  C.addressof(n))
        out_ms += list(ms[:n.value])
        out_k += list(kern[:n.value])
    return out_ms, out_k


KERNELS = {1: "conv_mfma_kernel", 2: "conv_glds_kernel", 3: "conv_x3_kernel", 4: "conv_x3h_kernel",
           5: "conv_halo5_kernel",
           10: "conv_head_kernel", 11: "conv_head_x3_kernel", 14: "conv_head_small_kernel",
           15: "conv_head_part_kernel"}


def kernel_name(gen):
    """Kernel symbol of a conv generation code (snrse_get_option "last_kernel" / "halo_kernel")."""
    return KERNELS.get(gen, f"conv_kernel_{gen}")


def conv_kernel_name():
    """Kernel symbol the halo-eligible convs dispatch to under the current setting."""
    return kernel_name(get_option("halo_kernel"))


def halo_ok(x, ksize, cout):
    """True when snrse_conv2d takes the halo path (and so accepts a fused GroupNorm).  Any batch size
    qualifies: sources beyond 2 GiB run as consecutive launches over image ranges (snrse_conv2d)."""
    B, H, W, C = x.shape
    # images tileable by 4 x 64 (the kernel then uses 8 x 32 tiles where H % 8 == 0); W = 32 alone stays on
    # the split-K GEMM (faster there: profiles/r03v_level4_halo_vs_glds.jsonl)
    return (x.dtype in H16 and ksize == 3 and cout % 128 == 0 and H % 4 == 0 and W % 64 == 0
            and _opt(x, "conv_variant") in (0, 5))


def x3h_ok(x, ksize, cout):
    """True when a split-bf16 fp32 conv (fp32 x, ops.split_weight weights) takes the halo kernel
    (conv_x3h_kernel) under the current x3_tile setting -- the one form that accepts a fused GroupNorm
    (gn=).  Mirrors snrse_conv2d's dispatch: 3x3, H % 4 == 0 and >= 256 tiles of 4 x 64 px x 128 couts
    (the last tile column cut by the image edge; x3_tile 0), or wherever legal (x3_tile 4)."""
    B, H, W, C = x.shape
    if x.dtype != torch.float32 or ksize != 3 or cout % 128 or H % 4:
        return False
    t = _opt(x, "x3_tile")
    return t == 4 or (t == 0 and B * (H // 4) * (-(-W // 64)) * (cout // 128) >= 256)


def head_ok(x, split=False):
    """True when a 3x3 conv of x with Cout = 4 and f32 output (the pyramid heads) takes a head kernel that
    accepts a fused GroupNorm (gn=): the halo-staged head (16-bit x, C <= 1024; or f32 x with split weights:
    split=True, the fp32x3 mode's conv_head_x3_kernel; H % 8 == 0, W % 32 == 0), or with C % 256 == 0 the
    wave-per-8-pixels head of the other image sizes (16-bit, or the fp32x3 form; option head_small, snrse_conv2d)."""
    B, H, W, C = x.shape
    if _opt(x, "conv_variant") == 1:
        return False
    h16 = x.dtype in H16
    dt_ok = h16 or (split and x.dtype == torch.float32)
    # channels: the C-ABI's K-tile (64 16-bit / 32 f32 channels, snrse_conv2d); the 16-bit tiled heads stage the
    # image's GroupNorm affine in an LDS table of 1024 channels
    if dt_ok and H % 8 == 0 and W % 32 == 0 and C % (64 if h16 else 32) == 0 and (not h16 or C <= 1024):
        return True
    return dt_ok and C % 256 == 0 and _opt(x, "head_small") != 0


def gn_scale_shift(sums0, gamma, beta, HW, sums1=None, groups=None, eps=1e-6):
    """Per-(b, c) GroupNorm affine [B, C] x 2 from per-channel sums."""
    _dev(sums0, sums1, gamma, beta)
    B, C0 = sums0.shape[0], sums0.shape[2]
    C1 = 0 if sums1 is None else sums1.shape[2]
    C = C0 + C1
    g = groups if groups is not None else min(C // 4, 32)
    # one [2, B, C] allocation: the persistent halo GEMM fetches scale and shift through a single
    # buffer resource (shift == scale + B*C)
    ss = torch.empty(2, B, C, device=sums0.device, dtype=torch.float32)
    scale, shift = ss[0], ss[1]
    _lib.call("snrse_gn_scale_shift", sums0.data_ptr(), C0, _ptr(sums1), C1, B, HW, gamma.data_ptr(), beta.data_ptr(),
              g, float(eps), scale.data_ptr(), shift.data_ptr(), _stream())
    return scale, shift


STAT_SLOTS = 16  # SNRSE_STAT_SLOTS (include/snrse.h)


def _arena_stack():
    """The calling thread's active StatsArena stack (innermost last)."""
    st = getattr(_TLS, "arenas", None)
    if st is None:
        st = _TLS.arenas = []
    return st


class StatsArena:
    """One f64 buffer per network evaluation, zeroed by a single fill, from which new_stats()
    carves the GroupNorm statistics buffers; the producers are told (option "stats_zeroed") to
    skip their per-call memset.  The first evaluation inside an arena only measures the size
    (its buffers come from torch.empty and are cleared by the producers as usual)."""

    ALIGN = 32  # doubles (256 B)

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf, self.off, self.need = None, 0, 0

    def __enter__(self):
        if self.buf is not None:
            self.buf.zero_()
        self.off, self.need = 0, 0
        _arena_stack().append(self)
        return self

    def __exit__(self, *exc):
        _arena_stack().remove(self)
        if self.buf is None or self.need > self.buf.numel():
            self.buf = torch.empty(self.need, dtype=torch.float64, device=self.device)
        return False

    def take(self, n):
        na = (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.need += na
        if self.buf is None or self.off + na > self.buf.numel():
            return None
        t = self.buf[self.off:self.off + n]
        self.off += na
        return t


def _stats_zeroed(cx, *bufs):
    """Set context cx's "stats_zeroed" switch for a producer writing into `bufs`."""
    bufs = [b for b in bufs if b is not None]
    if not bufs:
        return
    z = int(all(getattr(b, "_snrse_zeroed", False) for b in bufs))
    if cx.zeroed != z:
        cx.set_option("stats_zeroed", z)


def new_stats(x_or_shape, C=None):
    """[B, STAT_SLOTS, C, 2] f64 per-channel statistics buffer for an NHWC tensor (producers
    spread their atomics over the slots; consumers fold them).  Inside a StatsArena on the same
    device the buffer is a pre-zeroed arena slice."""
    if C is None:
        B, C, dev = x_or_shape.shape[0], x_or_shape.shape[-1], x_or_shape.device
    else:
        B, dev = x_or_shape, torch.device("cuda", torch.cuda.current_device())
    st = _arena_stack()
    if st and st[-1].device == torch.device(dev):
        t = st[-1].take(B * STAT_SLOTS * C * 2)
        if t is not None:
            t = t.view(B, STAT_SLOTS, C, 2)
            t._snrse_zeroed = True
            return t
    return torch.empty(B, STAT_SLOTS, C, 2, device=dev, dtype=torch.float64)


def fold_stats(st):
    """[B, STAT_SLOTS, C, 2] -> [B, C, 2] per-channel (sum, sumsq) (inspection / tests)."""
    return st.sum(1)


def gn_stats(src0, src1=None):
    """Per-channel (sum, sumsq) of each source: returns (sums0, sums1 or None)."""
    _dev(src0, src1)
    B, H, W, C0 = src0.shape
    C1 = 0 if src1 is None else src1.shape[3]
    s0 = new_stats(src0)
    s1 = None if src1 is None else new_stats(src1)
    cx = context(src0.device)
    _stats_zeroed(cx, s0, s1)
    _lib.call("snrse_gn_stats", cx.ptr, _ptr(src0), C0, _ptr(src1), C1, B, H * W, s0.data_ptr(), _ptr(s1),
              code(src0.dtype), _stream())
    return s0, s1


MODES = {"none": 0, "down": 1, "up": 2}
GN_FUSED_MAX_HW = 512  # gn_apply: images up to this many pixels take the single fold + apply launch


def gn_apply(src0, src1=None, sums=None, gamma=None, beta=None, act=True, mode="none", groups=None, eps=1e-6,
             sums1=None):
    """sums: new_stats() buffer of src0 or a (sums0, sums1) pair; None = no norm."""
    if isinstance(sums, tuple):
        sums, sums1 = sums
    _dev(src0, src1, sums, sums1, gamma, beta)
    B, H, W, C0 = src0.shape
    C1 = 0 if src1 is None else src1.shape[3]
    C = C0 + C1
    m = MODES[mode]
    # small images (the 16 x 32 .. 4 x 8 levels of C2): ONE launch that folds the statistics per block (at most
    # 4 blocks per image) and applies, instead of gn_scale_shift + gn_act -- two launch-floor kernels
    small = m == 0 and H * W <= GN_FUSED_MAX_HW
    if sums is not None and (m == 0 or resample_ok(src0)) and not small:
        # the per-(b, c) affine once (snrse_gn_scale_shift), then the elementwise / LDS-tiled apply: no
        # per-block re-fold of the slotted statistics (the fp32 gn_apply pass ran at ~0.2 of HBM peak that way)
        scale, shift = gn_scale_shift(sums, gamma, beta, H * W, sums1=sums1, groups=groups, eps=eps)
        if m == 0:
            return gn_act(src0, src1, scale, shift, act=act)
        if src1 is None and resample_ok(src0):
            return gn_resample(src0, scale, shift, act=act, mode=mode)[0]
    Ho, Wo = (H // 2, W // 2) if m == 1 else ((2 * H, 2 * W) if m == 2 else (H, W))
    out = torch.empty(B, Ho, Wo, C, device=src0.device, dtype=src0.dtype)
    g = groups if groups is not None else min(C // 4, 32)
    _lib.call("snrse_gn_apply", _ptr(src0), C0, _ptr(src1), C1, B, H, W, _ptr(sums), _ptr(sums1), _ptr(gamma),
              _ptr(beta), g, float(eps), int(bool(act)), m, out.data_ptr(), code(src0.dtype), _stream())
    return out


def resample_ok(x):
    """True when snrse_gn_resample takes x (NHWC): 16-bit with C % 16 == 0, or f32 with C / 4 dividing 64."""
    C = x.shape[3]
    if x.dtype in H16:
        return C % 16 == 0
    return x.dtype == torch.float32 and C % 4 == 0 and 64 % (C // 4) == 0


def gn_resample(x, scale=None, shift=None, act=True, mode="down", want_raw=False):
    """act(x*scale+shift) FIR-resampled x2 ('down' / 'up': upfirdn2d with [1,3,3,1]) and, with
    want_raw, the FIR of x itself (the ResBlock shortcut input) from one LDS-tiled pass over x
    (snrse_gn_resample; 16-bit: C % 8 == 0 with C / 8 dividing 64, or C % 16 == 0; f32: C / 4 dividing 64).
    Returns (activated, raw or None)."""
    _dev(x, scale, shift)
    if x.dtype not in (torch.float16, torch.bfloat16, torch.float32):
        raise TypeError("snrse: gn_resample takes fp16, bf16 or f32 activations")
    B, H, W, C = x.shape
    m = MODES[mode]
    if m == 0:
        raise ValueError("snrse: gn_resample mode must be 'down' or 'up'")
    Ho, Wo = (H // 2, W // 2) if m == 1 else (2 * H, 2 * W)
    oa = torch.empty(B, Ho, Wo, C, device=x.device, dtype=x.dtype)
    orw = torch.empty_like(oa) if want_raw else None
    _lib.call("snrse_gn_resample", _cx(x.device), x.data_ptr(), C, B, H, W, _ptr(scale), _ptr(shift), int(bool(act)), m,
              oa.data_ptr(), _ptr(orw), code(x.dtype), _stream())
    return oa, orw


def gn_act(src0, src1=None, scale=None, shift=None, act=True):
    """act(x*scale+shift) of the channel concatenation (src0 | src1), NHWC fp16, bf16 or f32 (snrse_gn_act)."""
    _dev(src0, src1, scale, shift)
    B, H, W, C0 = src0.shape
    C1 = 0 if src1 is None else src1.shape[3]
    out = torch.empty(B, H, W, C0 + C1, device=src0.device, dtype=src0.dtype)
    _lib.call("snrse_gn_act", src0.data_ptr(), C0, _ptr(src1), C1, B, H * W, _ptr(scale), _ptr(shift),
              int(bool(act)), out.data_ptr(), code(src0.dtype), _stream())
    return out


def fir(x, mode):
    """FIR [1,3,3,1] down/up x2 of an NHWC tensor (no normalisation)."""
    return gn_apply(x, act=False, mode=mode)


def attention(qkv, C=256, split=False):
    """softmax(q k^T / sqrt(C)) v (layerspp.py:84-88) of qkv [B, L(, W), 3C]; split=True (fp32 only): the fp32x3
    mode's split-bf16 products (snrse_attention with SNRSE_F32X3) instead of exact fp32 MFMAs."""
    _dev(qkv)
    B, L = qkv.shape[0], qkv.shape[1] * (qkv.shape[2] if qkv.dim() == 4 else 1)
    out = torch.empty(*qkv.shape[:-1], C, device=qkv.device, dtype=qkv.dtype)
    if split and qkv.dtype != torch.float32:
        raise TypeError("snrse: split attention takes fp32 q, k, v")
    _lib.call("snrse_attention", qkv.data_ptr(), out.data_ptr(), B, L, C, _lib.F32X3 if split else code(qkv.dtype),
              _stream())
    return out


def temb_mlp(t, Wg, W1, b1, W2, b2, fused=False):
    """temb [B, 4 nf] (ncsnpp.py:256-275): two row-parallel launches, snrse_temb_gfp_dense (W1 gfp(t) + b1) then
    snrse_temb_dense (W2 silu(.) + b2); fused=True: the one-launch snrse_temb_mlp (a block per utterance)."""
    _dev(t, Wg, W1, b1, W2, b2)
    B = t.shape[0]
    out = torch.empty(B, W2.shape[0], device=t.device, dtype=torch.float32)
    if fused:
        _lib.call("snrse_temb_mlp", t.data_ptr(), Wg.data_ptr(), W1.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                  b2.data_ptr(), out.data_ptr(), B, Wg.shape[0], _stream())
        return out
    a = torch.empty(B, W1.shape[0], device=t.device, dtype=torch.float32)
    _lib.call("snrse_temb_gfp_dense", t.data_ptr(), Wg.data_ptr(), W1.data_ptr(), b1.data_ptr(), a.data_ptr(), B,
              Wg.shape[0], _stream())
    _lib.call("snrse_temb_dense", a.data_ptr(), W2.data_ptr(), b2.data_ptr(), out.data_ptr(), B, W2.shape[0],
              W2.shape[1], _stream())
    return out


def temb_dense(temb, W, bias):
    _dev(temb, W, bias)
    B, D = temb.shape
    R = W.shape[0]
    out = torch.empty(B, R, device=temb.device, dtype=torch.float32)
    _lib.call("snrse_temb_dense", temb.data_ptr(), W.data_ptr(), bias.data_ptr(), out.data_ptr(), B, R, D,
              _stream())
    return out


def input_conv_ok(x):
    B, F, T = x.shape[0], x.shape[-2], x.shape[-1]
    return T % 64 == 0 and (F * T // 64) % 16 == 0


def input_conv(x, y, wgt, bias):
    """16-bit fused input conv: x, y complex64 [B,F,T], wgt [128][64] fp16 or bf16 -> (h [B,F,T,128] in wgt's
    format, stats, pyramid f32)."""
    _dev(x, y, wgt, bias)
    if wgt.dtype not in H16:
        raise TypeError(f"snrse: input_conv takes fp16 / bf16 weights, got {wgt.dtype}")
    B, F, T = x.shape[0], x.shape[-2], x.shape[-1]
    h = torch.empty(B, F, T, 128, device=x.device, dtype=wgt.dtype)
    pyr = torch.empty(B, F, T, 4, device=x.device, dtype=torch.float32)
    st = new_stats(B, 128)
    cx = context(x.device)
    _stats_zeroed(cx, st)
    _lib.call("snrse_input_conv", cx.ptr, x.data_ptr(), y.data_ptr(), B, F, T, wgt.data_ptr(), bias.data_ptr(),
              h.data_ptr(), pyr.data_ptr(), st.data_ptr(), code(wgt.dtype), _stream())
    return h, st, pyr


def input_conv_x3_ok(x):
    return input_conv_ok(x) and x.shape[-1] <= 1024


def input_conv_x3(x, y, wgt_split, bias):
    """fp32x3 fused input conv: x, y complex64 [B,F,T], split weights [128][128] bf16 -> (h [B,F,T,128] f32,
    stats, pyramid f32)."""
    _dev(x, y, wgt_split, bias)
    B, F, T = x.shape[0], x.shape[-2], x.shape[-1]
    h = torch.empty(B, F, T, 128, device=x.device, dtype=torch.float32)
    pyr = torch.empty(B, F, T, 4, device=x.device, dtype=torch.float32)
    st = new_stats(B, 128)
    cx = context(x.device)
    _stats_zeroed(cx, st)
    _lib.call("snrse_input_conv_x3", cx.ptr, x.data_ptr(), y.data_ptr(), B, F, T, wgt_split.data_ptr(),
              bias.data_ptr(), h.data_ptr(), pyr.data_ptr(), st.data_ptr(), _stream())
    return h, st, pyr


def input_pack(x, y, dtype):
    """x, y complex64 [B,F,T] -> (im2col [B,F,T,64] dtype, pyramid [B,F,T,4] f32)."""
    _dev(x, y)
    B, F, T = x.shape[0], x.shape[-2], x.shape[-1]
    col = torch.empty(B, F, T, 64, device=x.device, dtype=dtype)
    pyr = torch.empty(B, F, T, 4, device=x.device, dtype=torch.float32)
    _lib.call("snrse_input_pack", x.data_ptr(), y.data_ptr(), B, F, T, col.data_ptr(), pyr.data_ptr(),
              code(dtype), _stream())
    return col, pyr


def score_update(pyr, out_w, out_b, t, score_mode, x, y=None, coef=None, noise=None, seed=0, offset=0,
                 want_score=False, x_out=None, xmean_out=None):
    """Output head + score + optional SDE step.  Returns (x_out, x_mean, score)."""
    _dev(pyr, out_w, out_b, t, x, y, coef, noise)
    B = x.shape[0]
    HW = x.shape[-2] * x.shape[-1]
    score = torch.empty_like(x) if want_score else None
    if coef is not None:
        x_out = torch.empty_like(x) if x_out is None else x_out
        xmean_out = torch.empty_like(x) if xmean_out is None else xmean_out
    else:
        x_out = xmean_out = None
    _lib.call("snrse_score_update", pyr.data_ptr(), int(pyr.dtype == torch.float32), out_w.data_ptr(),
              out_b.data_ptr(), t.data_ptr(), int(score_mode), B, HW, x.data_ptr(), _ptr(y), _ptr(noise),
              int(seed) & (2**64 - 1), int(offset), _ptr(coef), _ptr(x_out), _ptr(xmean_out), _ptr(score),
              _stream())
    return x_out, xmean_out, score


def sde_update(x, coef, y=None, score=None, noise=None, seed=0, offset=0, x_out=None, xmean_out=None):
    _dev(x, coef, y, score, noise)
    B = x.shape[0]
    HW = x.shape[-2] * x.shape[-1]
    x_out = torch.empty_like(x) if x_out is None else x_out
    xmean_out = torch.empty_like(x) if xmean_out is None else xmean_out
    _lib.call("snrse_sde_update", x.data_ptr(), _ptr(y), _ptr(score), _ptr(noise), int(seed) & (2**64 - 1),
              int(offset), coef.data_ptr(), B, HW, x_out.data_ptr(), xmean_out.data_ptr(), _stream())
    return x_out, xmean_out


def axpby_noise(coef, x=None, y=None, noise=None, seed=0, offset=0, like=None):
    ref = x if x is not None else (y if y is not None else like)
    _dev(coef, x, y, noise)
    B = ref.shape[0]
    HW = ref.shape[-2] * ref.shape[-1]
    out = torch.empty_like(ref)
    _lib.call("snrse_axpby_noise", _ptr(x), _ptr(y), _ptr(noise), int(seed) & (2**64 - 1), int(offset),
              coef.data_ptr(), B, HW, out.data_ptr(), _stream())
    return out


def energy_ratios(s_hat, s, n=None):
    """[B, L] f32 device waveforms -> [B, 3] f64 (SI-SDR, SI-SIR, SI-SAR) dB (utils.py:10-35);
    without n only SI-SDR (column 0) is defined (sgmse/util/other.py:71-75)."""
    B, L = s_hat.shape
    if s.shape != s_hat.shape or (n is not None and n.shape != s_hat.shape):
        raise ValueError("energy_ratios: s_hat, s, n must share one [B, L] shape")
    a = [t.to(torch.float32).contiguous() for t in (s_hat, s)]
    nn = None if n is None else n.to(torch.float32).contiguous()
    _dev(a[0], a[1], nn)
    out = torch.empty(B, 3, device=s_hat.device, dtype=torch.float64)
    _lib.call("snrse_energy_ratios", a[0].data_ptr(), a[1].data_ptr(), _ptr(nn), B, L, out.data_ptr(), _stream())
    return out


def absmax(sig):
    """[B, L] f32 -> [B] max |sig| per row."""
    _dev(sig)
    B, L = sig.shape
    out = torch.empty(B, device=sig.device, dtype=torch.float32)
    _lib.call("snrse_absmax", sig.data_ptr(), B, L, out.data_ptr(), _stream())
    return out


def stft(sig, in_scale=1.0, tpad=None, mode=1, in_div=None):
    """sig [B, L] f32 -> complex64 [B, 256, Tpad] of sig * in_scale / in_div[b]."""
    _dev(sig, in_div)
    B, L = sig.shape
    T = 1 + L // 128
    tpad = T if tpad is None else tpad
    out = torch.empty(B, 256, tpad, device=sig.device, dtype=torch.complex64)
    _lib.call("snrse_stft", sig.data_ptr(), B, L, _ptr(in_div), float(in_scale), tpad, int(mode), out.data_ptr(),
              _stream())
    return out


def istft(spec, length, mode=1, out_scale=None):
    """spec complex64 [B, 256, T] -> [B, length] f32 (* out_scale[b])."""
    _dev(spec, out_scale)
    B, Fq, T = spec.shape
    frames = torch.empty(B, T, 510, device=spec.device, dtype=torch.float32)
    out = torch.empty(B, length, device=spec.device, dtype=torch.float32)
    _lib.call("snrse_istft", spec.data_ptr(), B, T, length, int(mode), _ptr(out_scale), frames.data_ptr(),
              out.data_ptr(), _stream())
    return out


UPFIRDN_DTYPES = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: _lib.F16, torch.float64: _lib.F64}


def upfirdn2d(inp, kernel, up=1, down=1, pad=(0, 0)):
    """Reference-signature upfirdn2d (op/upfirdn2d.py:145-156) on [N, C, H, W]."""
    _dev(inp, kernel)
    N, Cc, H, W = inp.shape
    kh, kw = kernel.shape
    x = inp.reshape(N * Cc, H, W, 1).contiguous()
    oh = (H * up + pad[0] + pad[1] - kh) // down + 1
    ow = (W * up + pad[0] + pad[1] - kw) // down + 1
    out = torch.empty(N * Cc, oh, ow, 1, device=inp.device, dtype=inp.dtype)
    k = kernel.to(torch.float32).contiguous()
    dt = UPFIRDN_DTYPES.get(inp.dtype)
    if dt is None:
        raise TypeError(f"upfirdn2d: unsupported dtype {inp.dtype} (float, double, half, bfloat16)")
    _lib.call("snrse_upfirdn2d", x.data_ptr(), out.data_ptr(), k.data_ptr(), N * Cc, H, W, 1, kh, kw, up, up,
              down, down, pad[0], pad[1], pad[0], pad[1], dt, _stream())
    return out.view(N, Cc, oh, ow)


def _upfirdn_raw(x4, k, upx, upy, dnx, dny, px0, px1, py0, py1):
    """snrse_upfirdn2d on [major, H, W, minor] with per-axis factors and pads."""
    major, H, W, minor = x4.shape
    kh, kw = k.shape
    oh = (H * upy + py0 + py1 - kh) // dny + 1
    ow = (W * upx + px0 + px1 - kw) // dnx + 1
    out = torch.empty(major, oh, ow, minor, device=x4.device, dtype=x4.dtype)
    dt = UPFIRDN_DTYPES.get(x4.dtype)
    if dt is None:
        raise TypeError(f"upfirdn2d: unsupported dtype {x4.dtype} (float, double, half, bfloat16)")
    _lib.call("snrse_upfirdn2d", x4.contiguous().data_ptr(), out.data_ptr(), k.to(torch.float32).contiguous().data_ptr(),
              major, H, W, minor, kh, kw, upx, upy, dnx, dny, px0, px1, py0, py1, dt, _stream())
    return out


class _UpFirDn2d(torch.autograd.Function):
    """upfirdn2d with gradients, every direction through snrse_upfirdn2d -- the call pattern of the
    reference's UpFirDn2d / UpFirDn2dBackward (op/upfirdn2d.py:19-142): the input gradient is the op on
    the output gradient with the flipped kernel, up and down swapped and the transposed pads
    (kw - pad_x0 - 1, in_w up - out_w down + pad_x0 - up + 1, likewise in y); its own gradient is the
    forward op again."""

    @staticmethod
    def forward(ctx, x, kernel, up, down, pad):
        (upx, upy), (dnx, dny), (px0, px1, py0, py1) = up, down, pad
        N, C, H, W = x.shape
        kh, kw = kernel.shape
        out = _upfirdn_raw(x.reshape(N * C, H, W, 1), kernel, upx, upy, dnx, dny, px0, px1, py0, py1)
        oh, ow = out.shape[1], out.shape[2]
        ctx.save_for_backward(kernel)
        ctx.geom = (up, down, pad, (N, C, H, W), (oh, ow),
                    (kw - px0 - 1, W * upx - ow * dnx + px0 - upx + 1, kh - py0 - 1, H * upy - oh * dny + py0 - upy + 1))
        return out.view(N, C, oh, ow)

    @staticmethod
    def backward(ctx, g):
        (kernel,) = ctx.saved_tensors
        return _UpFirDn2dGrad.apply(g, kernel, ctx.geom), None, None, None, None


class _UpFirDn2dGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, kernel, geom):
        (upx, upy), (dnx, dny), _, (N, C, H, W), (oh, ow), (gx0, gx1, gy0, gy1) = geom
        gi = _upfirdn_raw(g.contiguous().reshape(N * C, oh, ow, 1), torch.flip(kernel, [0, 1]), dnx, dny, upx, upy,
                          gx0, gx1, gy0, gy1)
        ctx.save_for_backward(kernel)
        ctx.geom = geom
        return gi.view(N, C, H, W)

    @staticmethod
    def backward(ctx, gg):
        (kernel,) = ctx.saved_tensors
        (upx, upy), (dnx, dny), (px0, px1, py0, py1), (N, C, H, W), (oh, ow), _ = ctx.geom
        go = _upfirdn_raw(gg.contiguous().reshape(N * C, H, W, 1), kernel, upx, upy, dnx, dny, px0, px1, py0, py1)
        return go.view(N, C, oh, ow), None, None


def upfirdn2d_autograd(inp, kernel, up=1, down=1, pad=(0, 0)):
    """The reference's upfirdn2d(input, kernel, up, down, pad) (op/upfirdn2d.py:145-156) with its autograd
    (first and second derivatives w.r.t. the input), on the HIP op."""
    _dev(inp, kernel)
    return _UpFirDn2d.apply(inp, kernel, (up, up), (down, down), (pad[0], pad[1], pad[0], pad[1]))


def set_option(name: str, value: int):
    """Process-wide switch: the library's process default context and every live LaunchContext."""
    _lib.call("snrse_set_option", name.encode(), int(value))
    for c in list(_CONTEXTS):
        c.set_option(name, value)


def spec_transform(spec, direction):
    """'exponent' spec_fwd (direction 0) / spec_back (1) on a complex64 device tensor."""
    _dev(spec)
    out = torch.empty_like(spec)
    _lib.call("snrse_spec_transform", spec.data_ptr(), out.data_ptr(), spec.numel(), int(direction), _stream())
    return out


SNRNET_KEYS = ["conv5x5_1.weight", "conv5x5_1.bias", "conv3x3_1.weight", "conv3x3_1.bias", "convt_1.weight",
               "convt_2.weight", "convt_3.weight", "convt_4.weight", "convt_1.bias", "convt_2.bias", "convt_3.bias",
               "convt_4.bias"]


def pack_snrnet(sd, device):
    f = lambda k: sd[k].detach().to(device, torch.float32).contiguous()  # noqa: E731
    w = [f(k) for k in SNRNET_KEYS]
    wih = torch.stack([f("blstm.weight_ih_l0"), f("blstm.weight_ih_l0_reverse")]).contiguous()
    whh = torch.stack([f("blstm.weight_hh_l0"), f("blstm.weight_hh_l0_reverse")]).contiguous()
    bsum = torch.stack([f("blstm.bias_ih_l0") + f("blstm.bias_hh_l0"),
                        f("blstm.bias_ih_l0_reverse") + f("blstm.bias_hh_l0_reverse")]).contiguous()
    return w + [wih, bsum, whh, f("fc.weight").reshape(-1).contiguous(), f("fc.bias")]


def snrnet(spec, packed):
    """SNRNet on the raw complex STFT [B, 256, T] (T % 16 == 0) -> [B] in (0, 1)."""
    _dev(spec)
    B, _, T = spec.shape
    ws = torch.empty(int(_lib.load().snrse_snrnet_workspace(B, T)) // 4 + 1, device=spec.device, dtype=torch.float32)
    out = torch.empty(B, device=spec.device, dtype=torch.float32)
    _lib.call("snrse_snrnet", spec.data_ptr(), B, T, *[p.data_ptr() for p in packed], ws.data_ptr(), out.data_ptr(),
              _stream())
    return out
