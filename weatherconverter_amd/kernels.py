"""Thin typed wrappers over the C ABI (``include/wc_kernels.h``) taking torch device tensors.

All launches go on the current torch stream (so torch ops, HIP graphs captured through
``torch.cuda.graph`` and these kernels are ordered).  Shapes are validated here before a pointer
ever reaches a kernel; the C layer re-validates and returns a status that is turned into a
RuntimeError.
"""
import contextlib
import ctypes
import functools
import os
import threading
from dataclasses import dataclass
from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple

import torch

from . import _native
from ._native import ConvArgs, ConvSeg


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


# Optional per-launch instrumentation for bench.py's roofline leg: when a list is installed here,
# conv_igemm records a (tile, algorithmic_flops, start_event, end_event) tuple around each launch.
PROFILE = None
REPLAY = None  # {'name': instantiation, 'reps': R, 'events': []}: see replay_timing


def profile_conv(enable: bool):
    """Record (name, algorithmic work, start event, end event, algorithmic bytes, issued MFMA FLOPs or
    None) for every conv / attention / GN launch until disabled."""
    global PROFILE
    if enable:
        _native.last_kernel_name()  # drop a name left by a launch outside the measurement
    PROFILE = [] if enable else None
    return PROFILE
STAMPS = None  # {'slots': int64 device tensor, 'launches': [(name, flops, nbytes, mfma)]}: see stamp_timing


def stamp_timing(slots: Optional[torch.Tensor]):
    """While set (an int64 device tensor), every named launch is bracketed by two wc_stamp launches that
    write the GPU wall clock to slots[2 i], slots[2 i + 1] (launch i in STAMPS['launches'] order).
    Captured into a HIP graph, the stamps time each launch as the replayed graph runs it.  None ends
    it; returns the state dict."""
    global STAMPS
    if slots is None:
        STAMPS = None
    else:
        _req(slots.is_cuda and slots.dtype == torch.int64 and slots.is_contiguous(), 'stamp slots: int64 device tensor')
        _native.last_kernel_name()  # drop a name left by a launch outside the measurement
        STAMPS = {'slots': slots, 'launches': []}
    return STAMPS


def _measuring() -> bool:
    """A timing mode that records the launches' algorithmic work is active."""
    return PROFILE is not None or REPLAY is not None or STAMPS is not None


def wall_clock_hz() -> float:
    """Rate of the clock wc_stamp reads (hipDeviceAttributeWallClockRate)."""
    khz = ctypes.c_int()
    _native.call('wc_wall_clock_khz', ctypes.byref(khz))
    return khz.value * 1e3


def replay_timing(name: Optional[str], reps: int = 5):
    """While set, every launch of instantiation `name` whose output does not alias its inputs is
    re-issued `reps` times back to back right after itself, between ONE pair of events (no per-launch
    event gaps; operands alive, the results rewritten unchanged).  Returns the state dict; the
    mean launch duration is sum(elapsed) / (reps * len(events))."""
    global REPLAY
    if name is not None:
        _native.last_kernel_name()  # drop a name left by a launch outside the measurement
    REPLAY = {'name': name, 'reps': reps, 'events': []} if name is not None else None
    return REPLAY


def _idempotent(fn_name: str, args) -> bool:
    """A conv launch can be re-run without changing its own inputs (output not aliased)."""
    if not fn_name.startswith('wc_conv'):
        return fn_name.startswith(('wc_attention', 'wc_wino_vsplit'))
    a = args[0]._obj
    ins = {a.seg[i].src for i in range(a.nseg)} | {a.res}
    return a.out not in ins


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _req(cond: bool, msg: str):
    if not cond:
        raise RuntimeError(f'weatherconverter_amd: {msg}')


@dataclass
class View:
    """NHWC fp32 channel slice ``t[..., c0:c0+C]`` of a contiguous (B, H, W, Ctot) tensor."""
    t: torch.Tensor
    c0: int
    C: int

    @staticmethod
    def full(t: torch.Tensor) -> 'View':
        return View(t, 0, t.shape[-1])

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + 4 * self.c0

    @property
    def ldc(self) -> int:
        return self.t.shape[-1]

    @property
    def B(self) -> int:
        return self.t.shape[0]

    @property
    def H(self) -> int:
        return self.t.shape[1]

    @property
    def W(self) -> int:
        return self.t.shape[2]

    def check(self):
        _req(self.t.is_cuda and self.t.dtype == torch.float32 and self.t.is_contiguous() and self.t.dim() == 4,
             'views must be contiguous fp32 NHWC device tensors')
        _req(0 <= self.c0 and self.c0 + self.C <= self.t.shape[-1], 'view channel range out of bounds')

    def tensor(self) -> torch.Tensor:
        return self.t[..., self.c0:self.c0 + self.C]


@dataclass
class Seg:
    view: View
    taps: Sequence[Tuple[int, int]]
    stride: int = 1
    scale: Optional[torch.Tensor] = None
    shift: Optional[torch.Tensor] = None
    silu: bool = False
    kbase: int = 0


TAPS3 = [(dy, dx) for dy in (-1, 0, 1) for dx in (-1, 0, 1)]


@dataclass
class GnPart:
    """GroupNorm tile partials of one NHWC tensor (B, H, W, 32*ncb), attached to it as
    ``t._wc_gn``: float32 [B][HW/64][ncb][32/sw][2] (mean, M2) per 64-pixel block x sw-channel
    sub-slot.  Written by the split-precision conv epilogues (wc_conv_args.gn_part) or
    wc_gn_partials; read by wc_gn_finalize_part for any channel range whose groups are whole
    sub-slots, instead of another pass over the tensor."""
    part: torch.Tensor
    sw: int
    ncb: int
    np64: int

    @staticmethod
    def eligible(t: torch.Tensor) -> bool:
        return t.dim() == 4 and (t.shape[1] * t.shape[2]) % 64 == 0 and t.shape[-1] % 32 == 0

    @staticmethod
    def attach(t: torch.Tensor, sw: int) -> 'GnPart':
        _req(GnPart.eligible(t) and sw in (4, 8, 16, 32), 'GN tile partials: HW % 64 == 0, C % 32 == 0')
        B, H, W, C = t.shape
        gp = GnPart(torch.empty((B, H * W // 64, C // 32, 32 // sw, 2), dtype=torch.float32, device=t.device), sw,
                    C // 32, H * W // 64)
        t._wc_gn = gp
        return gp

    @staticmethod
    def of(v: Optional['View']) -> Optional['GnPart']:
        gp = getattr(v.t, '_wc_gn', None) if v is not None else None
        return gp if (gp is not None and gp.covers(v)) else None

    def covers(self, v: 'View') -> bool:
        return getattr(v.t, '_wc_gn', None) is self and v.c0 % 32 == 0 and v.C % 32 == 0


def _conv_args(segs: Sequence[Seg], N: int, bias: Optional[torch.Tensor], out: Optional[View], Hm: int, Wm: int,
               temb: Optional[torch.Tensor], temb_ld: int, res: Optional[View], out_map,
               out_nchw: Optional[torch.Tensor], act: int, absmax: Optional[torch.Tensor] = None,
               act_param: Optional[torch.Tensor] = None, gn: Optional[GnPart] = None, gn_p64: int = 0,
               out_dummy: bool = False) -> ConvArgs:
    a = ConvArgs()
    _req(1 <= len(segs) <= 2, 'conv takes 1 or 2 K segments')
    B = segs[0].view.B
    for i, s in enumerate(segs):
        v = s.view
        v.check()
        _req(v.B == B, 'segment batch mismatch')
        _req(len(s.taps) <= _native.MAX_TAPS, 'too many taps')
        cs = a.seg[i]
        cs.src = v.ptr
        cs.C = v.C
        cs.ldc = v.ldc
        cs.H = v.H
        cs.W = v.W
        cs.sy = cs.sx = s.stride
        cs.ntaps = len(s.taps)
        for j, (dy, dx) in enumerate(s.taps):
            cs.dy[j] = dy
            cs.dx[j] = dx
        if s.scale is not None:
            _req(s.scale.shape == (B, v.C) and s.shift.shape == (B, v.C), 'GN affine shape')
            cs.scale = s.scale.data_ptr()
            cs.shift = s.shift.data_ptr()
        cs.silu = int(s.silu)
        cs.kbase = s.kbase
    a.nseg = len(segs)
    a.B, a.Hm, a.Wm, a.N = B, Hm, Wm, N
    a.bias = _ptr(bias)
    a.temb, a.temb_ld = _ptr(temb), temb_ld
    if res is not None:
        res.check()
        a.res, a.ldres = res.ptr, res.ldc
    a.osy, a.osx, a.ooy, a.oox = out_map
    a.act = act
    if act == _native.ACT_PRELU:
        _req(act_param is not None and act_param.is_cuda and act_param.dtype == torch.float32
             and act_param.numel() >= N, 'PReLU slopes: float32[N] on the device')
        a.act_param = act_param.data_ptr()
    if absmax is not None:
        _req(absmax.is_cuda and absmax.dtype == torch.float32 and absmax.is_contiguous() and absmax.numel() == B,
             'absmax output: float32[B] on the device')
        a.absmax_out = absmax.data_ptr()
    if gn is not None:
        _req(out is not None and gn.covers(out) and N == out.C, 'GN partials: output view of the partials tensor')
        a.gn_part, a.gn_ncb, a.gn_sw = gn.part.data_ptr(), gn.ncb, gn.sw
        a.gn_c0, a.gn_p64, a.gn_np64 = out.c0, gn_p64, gn.np64
    if out_nchw is not None:
        _req(out_nchw.is_contiguous() and out_nchw.shape[0] == B and out_nchw.shape[1] == N, 'NCHW output shape')
        a.out = out_nchw.data_ptr()
        a.ldo = 0
        a.Ho, a.Wo = out_nchw.shape[2], out_nchw.shape[3]
        a.out_nchw = 1
    elif out_dummy:  # the kernel writes its own output format (e.g. the pre-split qkv)
        a.out, a.ldo, a.Ho, a.Wo = None, N, Hm, Wm
    else:
        out.check()
        _req(out.C == N and out.B == B, 'output view shape')
        a.out, a.ldo, a.Ho, a.Wo = out.ptr, out.ldc, out.H, out.W
    return a


def _timed(name: str, fn_name: str, flops: float, *args, nbytes: float = 0.0, mfma: Optional[float] = None):
    """Launch; while profiling, record timing under the launched kernel's exact instantiation name
    (the library reports it, in rocprofv3's form; ``name`` is the fallback for unnamed kernels).

    REPLAY with name '*' (or this instantiation's name): an idempotent launch is re-issued
    REPLAY['reps'] times back to back right after itself between one event pair and recorded as
    (name, flops, e0, e1, reps, nbytes, mfma) in REPLAY['events'] — per-launch durations free of event
    gaps; a launch that rewrites its own input runs once between its own events (reps 1).  nbytes =
    the launch's algorithmic HBM bytes (each input and output element once) where the wrapper
    states it; mfma = the dense 16-bit MFMA FLOPs the launch issues where they are not the
    algorithmic FLOPs times its arithmetic mode's pieces (the Winograd conv: 2/3 of the direct form's
    products on its 3x3 segment), else None."""
    if STAMPS is not None:
        i = len(STAMPS['launches'])
        _req(2 * i + 1 < STAMPS['slots'].numel(), 'stamp slots exhausted')
        sp = STAMPS['slots'].data_ptr()
        _native.call('wc_stamp', sp, 2 * i, _stream())
        _native.call(fn_name, *args)
        exact = _native.last_kernel_name() or name
        _native.call('wc_stamp', sp, 2 * i + 1, _stream())
        STAMPS['launches'].append((exact, flops, nbytes, mfma))
        return
    if PROFILE is None and REPLAY is None:
        _native.call(fn_name, *args)
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _native.call(fn_name, *args)
    e1.record()
    exact = _native.last_kernel_name() or name
    if PROFILE is not None:
        PROFILE.append((exact, flops, e0, e1, nbytes, mfma))
    if REPLAY is not None and REPLAY['name'] in ('*', exact):
        reps = REPLAY['reps'] if _idempotent(fn_name, args) else 0
        if reps:
            r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            r0.record()
            for _ in range(reps):
                _native.call(fn_name, *args)
            r1.record()
            _native.last_kernel_name()
            REPLAY['events'].append((exact, flops, r0, r1, reps, nbytes, mfma))
        else:
            REPLAY['events'].append((exact, flops, e0, e1, 1, nbytes, mfma))


def _flops(segs: Sequence[Seg], Hm: int, Wm: int, N: int) -> float:
    return 2.0 * segs[0].view.B * Hm * Wm * N * sum(len(sg.taps) * sg.view.C for sg in segs)


def _abytes(segs: Sequence[Seg], N: int, out_pixels: int, res: Optional[View] = None, B: int = 0) -> float:
    """Algorithmic HBM bytes of a conv launch: every input element of every segment, the output and
    the residual view once (fp32).  (B: the batch when segs may be empty.)"""
    if not _measuring():
        return 0.0
    b = sum(4.0 * sg.view.B * sg.view.H * sg.view.W * sg.view.C for sg in segs)
    b += 4.0 * (segs[0].view.B if segs else B) * out_pixels * N * (2 if res is not None else 1)
    return b


def conv_igemm(segs: Sequence[Seg], w: torch.Tensor, bias: Optional[torch.Tensor], out: View, *, Hm: int, Wm: int,
               temb: Optional[torch.Tensor] = None, temb_ld: int = 0, res: Optional[View] = None,
               out_map=(1, 1, 0, 0), out_nchw: Optional[torch.Tensor] = None, act: int = 0,
               act_param: Optional[torch.Tensor] = None):
    """Implicit-GEMM conv on fp32 MFMA:
    out[b, my*osy+ooy, mx*osx+oox, n] = act(sum_k A[m, k] W[n, k] + bias (+ temb)) (+ res)."""
    _req(w.is_cuda and w.dtype == torch.float32 and w.is_contiguous() and w.dim() == 2, 'packed weight')
    N, ldw = w.shape
    a = _conv_args(segs, N, bias, out, Hm, Wm, temb, temb_ld, res, out_map, out_nchw, act, act_param=act_param)
    a.w, a.ldw = w.data_ptr(), ldw
    # the kernel symbol wc_conv_igemm dispatches to (mirrors dispatch() in csrc/wc_conv.hip)
    bm, bn = (256, 64) if N <= 64 else (128, 128)
    s0 = segs[0]
    pro = 0 if s0.scale is None else (2 if s0.silu else 1)
    unib = 'true' if (Hm * Wm) % bm == 0 else 'false'
    _timed(f'conv_igemm_kernel<{bm}, {bn}, {pro}, {unib}, {act}>', 'wc_conv_igemm',
           _flops(segs, Hm, Wm, N) if _measuring() else 0.0, ctypes.byref(a), _stream())


# ---- bf16x6 split-precision 3x3 conv (csrc/wc_conv6.hip) ----

CONV_PRECISIONS = ('f16x3', 'bf16x6', 'fp32')


def default_conv_precision() -> str:
    """Conv / attention arithmetic: 'f16x3' (the GN-prologue 3x3 convs on two-piece fp16 with a
    provable range bound, everything else bf16x6), 'bf16x6' (exact 3-piece bf16 split on bf16 MFMA
    everywhere) or 'fp32' (fp32 MFMA).  All three are fp32-class.  Overridable with
    WC_CONV_PRECISION."""
    p = os.environ.get('WC_CONV_PRECISION', 'f16x3')
    _req(p in CONV_PRECISIONS, f'WC_CONV_PRECISION must be one of {CONV_PRECISIONS}, got {p!r}')
    return p


def _piece_dtype() -> torch.dtype:
    """16-bit piece format of the f16x3 packs for the active library variant: fp16, or bf16 on the bf16
    single-piece build (the bf16 training line), whose kernels read their operands as bf16."""
    return torch.bfloat16 if _native.active_variant() == 'bf16' else torch.float16


def _split2(v: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(h, l) 16-bit pieces of an fp32 tensor: h = piece(v), l = piece(v - h) (round to nearest even).
    On the bf16 single-piece line l = 0, as the device packs write it (wc_x6.hpp split2_one / split2_pair
    under WC_SINGLE16=2: that line has no correction products)."""
    dt = _piece_dtype()
    h = v.to(dt)
    if dt == torch.bfloat16:
        return h, torch.zeros_like(h)
    return h, (v - h.float()).to(dt)


@dataclass
class X6Weight:
    """A conv weight re-packed for the bf16x6 kernels: its three exact bf16 pieces, laid out as
    [N tile][step][piece][k-half][BN][8] (bit patterns in an int16 tensor).  order 'halo':
    steps are (16-channel chunk, tap) for wc_conv3x3_x6; 'natural': K/16 in K order for
    wc_conv_igemm_x6."""
    data: torch.Tensor
    N: int
    BN: int
    C0: int
    C1: int
    order: str = 'halo'
    wsinv: Optional[torch.Tensor] = None  # order 'f16x3': 2^-sW[n]
    res_f16: bool = False  # f16x3: the residual segment packed as fp16 pieces (needs an A bound)


@functools.lru_cache(maxsize=None)
def x6_tile(N: int) -> Tuple[int, int]:
    """(TH, BN) of wc_conv3x3_x6 for N output channels (mirrors wc_conv3x3_x6_tile_n)."""
    bn = _native.load().wc_conv3x3_x6_tile_n(N)
    return (16 if bn == 64 else 8), bn


def split3_bits(x: torch.Tensor) -> torch.Tensor:
    """Exact 3-piece bf16 split by truncation (csrc/wc_conv6.hip split3): x == p0 + p1 + p2, each
    piece a bf16 bit pattern.  Returns int16 (3, *x.shape)."""
    _req(x.dtype == torch.float32, 'split3 takes fp32')
    mask = torch.tensor(-65536, dtype=torch.int32, device=x.device)  # 0xffff0000
    u0 = x.view(torch.int32)
    r1 = x - (u0 & mask).view(torch.float32)
    u1 = r1.view(torch.int32)
    r2 = r1 - (u1 & mask).view(torch.float32)
    u2 = r2.view(torch.int32)
    return (torch.stack([u0, u1, u2]) >> 16).to(torch.int16)


def _pack_dev(w: torch.Tensor, C0: int, C1: int, ntaps: int, order: str, mode: int, res_f16: bool):
    """One-launch device re-pack (wc_pack_split) of a [N][ntaps*C0 + C1] fp32 CUDA weight: (data, wsinv)
    in exactly the layout of the torch definitions below, evaluated with IEEE fp32 arithmetic and
    round-to-nearest-even conversions — bit for bit the definitions run on the CPU
    (tests/test_gpu_train.py).  (The same torch ops run on the GPU are not: their fp16 / power-of-two
    scaling ops differ in the last bit of some pieces, which the split tolerates.)"""
    N, K = w.shape
    _, BN = x6_tile(N)
    Np = -(-N // BN) * BN
    P0, P1 = (2, 2 if res_f16 else 3) if mode == 1 else (3, 3)
    row = (ntaps * C0 // 16 * P0 + C1 // 16 * P1) * 2 * BN * 8
    w = w.float().contiguous()
    data = torch.empty((Np // BN, row), dtype=torch.int16, device=w.device)
    wsinv = torch.empty(Np, dtype=torch.float32, device=w.device) if mode == 1 else None
    _timed('pack_split_kernel', 'wc_pack_split', 0.0, w.data_ptr(), K, N, C0, ntaps, C1,
           0 if order == 'halo' else 1, mode, int(res_f16), BN, data.data_ptr(), data.numel() * 2, _ptr(wsinv),
           _stream())
    return data, wsinv


def pack_device_enabled() -> bool:
    """Weight packs built by the one-launch device kernel for CUDA weights; WC_PACK_DEVICE=0 keeps the
    torch-op definitions (A/B, and the reference the kernel is tested against)."""
    return os.environ.get('WC_PACK_DEVICE', '1') != '0'


def pack_x6(w: torch.Tensor, C0: int, C1: int = 0, *, ntaps: int = 9, order: str = 'halo',
            device: Optional[bool] = None) -> X6Weight:
    """Re-pack a [N][ntaps*C0 + C1] conv weight (K = (tap, c) then the 1x1 residual columns, as
    engine.pack_conv) for the bf16x6 kernels.  order 'halo' (wc_conv3x3_x6, ntaps 9): steps are
    (16-channel chunk, tap) then the residual chunks; 'natural' (wc_conv_igemm_x6): K/16 in order.
    A CUDA weight is packed by the device kernel (device=None: unless WC_PACK_DEVICE=0)."""
    N, K = w.shape
    if (device if device is not None else pack_device_enabled()) and w.is_cuda:
        _req(K == ntaps * C0 + C1 and C0 % 16 == 0 and C1 % 16 == 0, 'x6 weight shape')
        _req(order == 'natural' or ntaps == 9, "order 'halo' is for 3x3 weights")
        data, _ = _pack_dev(w, C0, C1, ntaps, order, 0, False)
        BN = x6_tile(N)[1]
        S = (ntaps * C0 + C1) // 16
        return X6Weight(data.view(data.shape[0], S, 3, 2, BN, 8), N, BN, C0, C1, order)
    _req(K == ntaps * C0 + C1 and C0 % 16 == 0 and C1 % 16 == 0, 'x6 weight shape')
    _req(order == 'natural' or ntaps == 9, "order 'halo' is for 3x3 weights")
    _, BN = x6_tile(N)
    Np = -(-N // BN) * BN
    wp = torch.zeros((Np, K), dtype=torch.float32, device=w.device)
    wp[:N] = w.float()
    if order == 'halo':
        s0 = wp[:, :9 * C0].reshape(Np, 9, C0 // 16, 2, 8).permute(0, 2, 1, 3, 4).reshape(Np, 9 * (C0 // 16), 2, 8)
        s1 = wp[:, 9 * C0:].reshape(Np, C1 // 16, 2, 8)
        allw = torch.cat([s0, s1], 1)
    else:
        _req(order == 'natural', f'unknown x6 order {order!r}')
        allw = wp.reshape(Np, K // 16, 2, 8)
    S = allw.shape[1]
    pieces = split3_bits(allw)  # (3, Np, S, 2, 8)
    data = pieces.view(3, Np // BN, BN, S, 2, 8).permute(1, 3, 0, 4, 2, 5).contiguous()
    return X6Weight(data, N, BN, C0, C1, order)


def pack_f16x3(w: torch.Tensor, C0: int, C1: int = 0, *, ntaps: int = 9, order: str = 'halo',
               res_f16: bool = False, amax: Optional[torch.Tensor] = None, device: Optional[bool] = None) -> X6Weight:
    """Re-pack a [N][ntaps*C0 + C1] conv (+ 1x1 residual) weight for the f16x3 kernels: per output
    channel n a power-of-two scale 2^sW[n] with max_k |w[n, k]| * 2^sW[n] <= 2^14 over the fp16-packed
    columns (segment 0, and the residual with res_f16); segment 0
    as two round-to-nearest fp16 pieces, in (chunk, tap) step order for wc_conv3x3_f16x3 ('halo',
    ntaps 9) or natural K order for wc_conv_igemm_f16x3 ('natural'); the residual part as three
    bf16 pieces (same scale), or as two fp16 pieces with res_f16 (for a conv given a per-image A
    bound, wc_conv3x3_f16x3)."""
    N, K = w.shape
    _req(K == ntaps * C0 + C1 and C0 % 16 == 0 and C1 % 16 == 0, 'f16x3 weight shape')
    _req(order == 'natural' or ntaps in (9, 4), "order 'halo' is for 3x3 (or s2d 2x2) weights")
    if (device if device is not None else pack_device_enabled()) and w.is_cuda and amax is None:
        data, wsinv = _pack_dev(w, C0, C1, ntaps, order, 1, res_f16)
        order_tag = ('f16x3' if ntaps == 9 else 'f16x3s') if order == 'halo' else 'f16x3n'
        return X6Weight(data, N, x6_tile(N)[1], C0, C1, order_tag, wsinv, res_f16)
    _, BN = x6_tile(N)
    Np = -(-N // BN) * BN
    T = Np // BN
    wp = torch.zeros((Np, K), dtype=torch.float32, device=w.device)
    wp[:N] = w.float()
    K0 = ntaps * C0
    # the scale must keep every fp16-packed column <= 2^14: segment 0, plus the residual with res_f16
    if amax is None:  # (a caller packing several weights under one scale passes their common max)
        amax = (wp if res_f16 else wp[:, :K0]).abs().amax(1).double()
    else:
        amax = torch.cat([amax.double().to(w.device), torch.zeros(Np - N, dtype=torch.float64, device=w.device)])
    sw = torch.where(amax > 0, torch.floor(torch.log2(2.0**14 / amax.clamp_min(1e-300))), torch.zeros_like(amax))
    sw = sw.clamp(-60, 60).to(torch.int32)
    ws = wp * torch.ldexp(torch.ones_like(wp[:, :1]), sw[:, None].float())  # exact power-of-two scaling
    S0, S1 = K0 // 16, C1 // 16
    if order == 'halo':
        main = ws[:, :K0].reshape(Np, ntaps, C0 // 16, 2, 8).permute(0, 2, 1, 3, 4).reshape(Np, S0, 2, 8)
    else:
        _req(order == 'natural', f'unknown f16x3 order {order!r}')
        main = ws[:, :K0].reshape(Np, S0, 2, 8)
    h, lo = _split2(main)
    pm = torch.stack([h, lo]).view(torch.int16).view(2, T, BN, S0, 2, 8).permute(1, 3, 0, 4, 2, 5)
    parts = [pm.reshape(T, -1)]
    if C1:
        rw = ws[:, K0:].reshape(Np, S1, 2, 8)
        if res_f16:
            pr = torch.stack(_split2(rw)).view(torch.int16).view(2, T, BN, S1, 2, 8)
        else:
            pr = split3_bits(rw).view(3, T, BN, S1, 2, 8)
        parts.append(pr.permute(1, 3, 0, 4, 2, 5).reshape(T, -1))
    data = torch.cat(parts, 1).contiguous()
    wsinv = torch.ldexp(torch.ones(Np, dtype=torch.float32, device=w.device), (-sw).float()).contiguous()
    order_tag = ('f16x3' if ntaps == 9 else 'f16x3s') if order == 'halo' else 'f16x3n'
    return X6Weight(data, N, BN, C0, C1, order_tag, wsinv, res_f16)


def f16x3_a_exp(gamma_absmax: float, beta_absmax: float, n_group: int) -> int:
    """sA for wc_conv3x3_f16x3: (sqrt(n - 1) max|gamma| + max|beta|) * 2^sA <= 2^14 (Samuelson's
    bound on a GroupNorm output, times a 4x margin under the fp16 maximum 65504)."""
    import math
    bound = math.sqrt(max(n_group - 1, 1)) * gamma_absmax + beta_absmax
    if not math.isfinite(bound):
        raise RuntimeError('weatherconverter_amd: non-finite GroupNorm affine in an f16x3 conv')
    if bound <= 0:
        return 0
    return max(-60, min(60, math.floor(math.log2(2.0**14 / bound))))


def conv3x3_f16x3(segs: Sequence[Seg], w3: X6Weight, bias: Optional[torch.Tensor], out: View, *, Hm: int, Wm: int,
                  a_exp: int, a_bound: Optional[torch.Tensor] = None, temb: Optional[torch.Tensor] = None,
                  temb_ld: int = 0, res: Optional[View] = None, act: int = 0,
                  absmax: Optional[torch.Tensor] = None, gn: Optional[GnPart] = None):
    """3x3 stride-1 conv with a GN(+SiLU) prologue on f16x3 (see wc_conv3x3_f16x3); a_exp from
    f16x3_a_exp of that GroupNorm; a_bound = per-image bound of the residual segment's input
    (gn_affine(..., bound=True)), required iff w3 packs the residual in fp16.  absmax: optional
    caller-zeroed float32[B], raised to each image's max |out|."""
    _req(w3.data.is_cuda and w3.data.is_contiguous() and w3.order == 'f16x3', 'f16x3 weight')
    _req((a_bound is not None) == (w3.res_f16 and w3.C1 > 0) or w3.C1 == 0 and not w3.res_f16,
         'a residual packed in fp16 needs an A bound (and only then)')
    if a_bound is not None:
        _req(a_bound.is_cuda and a_bound.dtype == torch.float32 and a_bound.numel() == segs[0].view.B, 'A bound')
    _req(w3.C0 == segs[0].view.C and w3.C1 == (segs[1].view.C if len(segs) == 2 else 0), 'f16x3 weight segments')
    _req(segs[0].scale is not None or (a_bound is not None and len(segs) == 1),
         'f16x3 needs the GroupNorm prologue or (one raw segment) a per-image A bound')
    a = _conv_args(segs, w3.N, bias, out, Hm, Wm, temb, temb_ld, res, (1, 1, 0, 0), None, act, absmax, gn=gn)
    TH, BN = x6_tile(w3.N)
    pro = 2 if segs[0].silu else 1
    res_seg = 'true' if len(segs) == 2 else 'false'
    r16 = 'true' if a_bound is not None and len(segs) == 2 else 'false'
    _timed(f'conv3x3_x6_kernel<{TH}, {BN}, {pro}, {res_seg}, true, {r16}>', 'wc_conv3x3_f16x3',
           _flops(segs, Hm, Wm, w3.N) if _measuring() else 0.0, ctypes.byref(a),
           w3.data.data_ptr(), w3.data.numel() * 2, int(a_exp), w3.wsinv.data_ptr(), _ptr(a_bound), _stream(),
           nbytes=_abytes(segs, w3.N, Hm * Wm, res))


@functools.lru_cache(maxsize=None)
def wino_tile(N: int) -> Tuple[int, int]:
    """(TH, BN) of wc_conv3x3_wino_f16x3 for N output channels."""
    bn = _native.load().wc_conv3x3_wino_tile_n(N)
    return (16 if bn == 64 else 8), bn


def wino_enabled() -> bool:
    """ResBlock 3x3 convs through the Winograd F(2,3)-along-x kernel (WC_WINO=0: the direct halo
    kernel, kept for A/B and as the reference the Winograd kernel is tested against)."""
    return os.environ.get('WC_WINO', '1') != '0'


def wino_filter(w: torch.Tensor, C0: int) -> torch.Tensor:
    """The F(2,3) filter transform of the 3x3 part of a [N][9*C0 (+ C1)] weight (K = (ky*3 + kx, c)),
    in float64: U[n][ky][p][c] = (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2) of row ky."""
    g = w[:, :9 * C0].double().reshape(w.shape[0], 3, 3, C0)
    g0, g1, g2 = g[:, :, 0], g[:, :, 1], g[:, :, 2]
    return torch.stack([g0, (g0 + g1 + g2) * 0.5, (g0 - g1 + g2) * 0.5, g2], 2)


def pack_wino_raw(w4: torch.Tensor, wres: Optional[torch.Tensor] = None, transposed: bool = False) -> X6Weight:
    """pack_wino straight from a conv module's [Co][Ci][3][3] weight on the device (wc_pack_wino_raw): the
    conv itself (+ the residual 1x1 weight wres [Co][C1]), or with transposed=True its data gradient's
    flipped, transposed filter (N = Ci, C0 = Co) -- bit-identical to pack_wino(pack_conv(...)) of the host
    re-layouts, without them."""
    _req(w4.is_cuda and w4.dtype == torch.float32 and w4.is_contiguous() and w4.dim() == 4 and w4.shape[2:] == (3, 3),
         'pack_wino_raw: contiguous fp32 [Co][Ci][3][3] device weight')
    Co, Ci = w4.shape[:2]
    N, C0 = (Ci, Co) if transposed else (Co, Ci)
    C1 = 0
    if wres is not None:
        _req(not transposed and wres.is_cuda and wres.dtype == torch.float32 and wres.is_contiguous()
             and wres.shape[0] == Co, 'pack_wino_raw residual: contiguous fp32 [Co][C1]')
        C1 = wres.shape[1]
    _req(C0 % 16 == 0 and C1 % 16 == 0, 'wino weight shape')
    _, BN = wino_tile(N)
    Np = -(-N // BN) * BN
    T = Np // BN
    data = torch.empty((T, (12 * C0 + C1) // 16 * 2 * 2 * BN * 8), dtype=torch.int16, device=w4.device)
    wsinv = torch.empty(Np, dtype=torch.float32, device=w4.device)
    _timed('pack_wino_raw_kernel', 'wc_pack_wino_raw', 0.0, w4.data_ptr(), _ptr(wres), N, C0, C1, int(transposed),
           data.data_ptr(), data.numel() * 2, wsinv.data_ptr(), _stream())
    return X6Weight(data, N, BN, C0, C1, 'wino', wsinv, bool(C1))


def pack_wino_raw_batch(reqs: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor], bool]]) -> List[X6Weight]:
    """pack_wino_raw of every (w4, wres, transposed) in reqs in ONE launch (wc_pack_wino_batch): the same
    pieces and scales, bit for bit, as one wc_pack_wino_raw each."""
    if not reqs:
        return []
    outs, rows, wg, max_c0 = [], [], 0, 0
    dev = reqs[0][0].device
    for w4, wres, transposed in reqs:
        _req(w4.is_cuda and w4.dtype == torch.float32 and w4.is_contiguous() and w4.dim() == 4
             and w4.shape[2:] == (3, 3), 'pack_wino_raw: contiguous fp32 [Co][Ci][3][3] device weight')
        Co, Ci = w4.shape[:2]
        N, C0 = (Ci, Co) if transposed else (Co, Ci)
        C1 = 0
        if wres is not None:
            _req(not transposed and wres.is_cuda and wres.dtype == torch.float32 and wres.is_contiguous()
                 and wres.shape[0] == Co, 'pack_wino_raw residual: contiguous fp32 [Co][C1]')
            C1 = wres.shape[1]
        _req(C0 % 16 == 0 and C1 % 16 == 0 and 9 * (C0 + 4) * 4 <= 64 * 1024, "wino weight shape")
        _, BN = wino_tile(N)
        Np = -(-N // BN) * BN
        data = torch.empty((Np // BN, (12 * C0 + C1) // 16 * 2 * 2 * BN * 8), dtype=torch.int16, device=dev)
        wsinv = torch.empty(Np, dtype=torch.float32, device=dev)
        outs.append(X6Weight(data, N, BN, C0, C1, 'wino', wsinv, bool(C1)))
        rows.append([w4.data_ptr(), _ptr(wres) or 0, data.data_ptr(), wsinv.data_ptr(),
                     N | (C0 << 32), C1 | (int(transposed) << 32), BN | (wg << 32), 0])
        wg += Np
        max_c0 = max(max_c0, C0)
    _req(wg < 2**31, 'pack batch too large')
    tab = torch.empty((len(rows), 8), dtype=torch.int64, pin_memory=True)
    tab.copy_(torch.tensor(rows, dtype=torch.int64))
    dtab = tab.to(dev, non_blocking=True)
    _timed('pack_wino_batch_kernel', 'wc_pack_wino_batch', 0.0, dtab.data_ptr(), len(rows), wg, max_c0, _stream())
    return outs


def pack_wino(w: torch.Tensor, C0: int, C1: int = 0, *, device: Optional[bool] = None) -> X6Weight:
    """Pack a [N][9*C0 + C1] ResBlock conv weight (3x3 taps then the 1x1 residual columns, as
    engine.pack_conv) for wc_conv3x3_wino_f16x3: the F(2,3) filter transform in float64, a per-channel
    power-of-two scale 2^sW[n] with max |U|, |w_res| * 2^sW <= 2^14, each value rounded once to fp32 and
    split into two round-to-nearest fp16 pieces; layout [N tile][C0/16][ky 3][p 4][piece][k-half][BN][8]
    then [N tile][C1/16][piece][k-half][BN][8].  A CUDA weight is packed by the device kernel (device=None:
    unless WC_PACK_DEVICE=0)."""
    N, K = w.shape
    _req(K == 9 * C0 + C1 and C0 % 16 == 0 and C1 % 16 == 0, 'wino weight shape')
    _, BN = wino_tile(N)
    Np = -(-N // BN) * BN
    T = Np // BN
    if (device if device is not None else pack_device_enabled()) and w.is_cuda:
        # one launch (wc_pack_wino), bit-identical to the definition below evaluated on the CPU
        data = torch.empty((T, (12 * C0 + C1) // 16 * 2 * 2 * BN * 8), dtype=torch.int16, device=w.device)
        wsinv = torch.empty(Np, dtype=torch.float32, device=w.device)
        wf = w.float().contiguous()
        _timed('pack_wino_kernel', 'wc_pack_wino', 0.0, wf.data_ptr(), N, C0, C1, data.data_ptr(), data.numel() * 2,
               wsinv.data_ptr(), _stream())
        return X6Weight(data, N, BN, C0, C1, 'wino', wsinv, bool(C1))
    wd = torch.zeros((Np, K), dtype=torch.float64, device=w.device)
    wd[:N] = w.double()
    U = wino_filter(wd, C0)  # [Np][3][4][C0]
    r = wd[:, 9 * C0:]
    amax = U.abs().reshape(Np, -1).amax(1)
    if C1:
        amax = torch.maximum(amax, r.abs().amax(1))
    # sW = floor(log2(2^14 / amax)) from the exponent (exact): amax = m 2^e, m in [0.5, 1)
    m, e = torch.frexp(amax)
    sw = torch.where(amax > 0, torch.where(m == 0.5, 15 - e, 14 - e).double(), torch.zeros_like(amax))
    sw = sw.clamp(-60, 60)
    scale = torch.ldexp(torch.ones_like(sw), sw)

    def pieces(v):  # exact power-of-two scaling, one rounding to fp32, two fp16 pieces
        v32 = (v * scale.reshape((-1, ) + (1, ) * (v.dim() - 1))).float()
        return torch.stack(_split2(v32)).view(torch.int16)

    nc0 = C0 // 16
    p0 = pieces(U).view(2, T, BN, 3, 4, nc0, 2, 8).permute(1, 5, 3, 4, 0, 6, 2, 7).reshape(T, -1)
    parts = [p0]
    if C1:
        p1 = pieces(r).view(2, T, BN, C1 // 16, 2, 8).permute(1, 3, 0, 4, 2, 5).reshape(T, -1)
        parts.append(p1)
    data = torch.cat(parts, 1).contiguous()
    wsinv = torch.ldexp(torch.ones(Np, dtype=torch.float32, device=w.device), (-sw).float()).contiguous()
    return X6Weight(data, N, BN, C0, C1, 'wino', wsinv, bool(C1))


def wino_eligible(segs: Sequence[Seg], N: int, Hm: int, Wm: int) -> bool:
    """True when wc_conv3x3_wino_f16x3 accepts this conv (mirrors its host checks): segment 0 with the
    GN+SiLU prologue (+ an optional 1x1 residual segment), or one raw segment (given a per-image bound)."""
    s0 = segs[0]
    TH, _ = wino_tile(N)
    if len(s0.taps) != 9 or s0.view.C % 16 or Hm % TH or Wm % 16 or s0.stride != 1:
        return False
    if list(s0.taps) != [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]:
        return False
    if s0.view.H != Hm or s0.view.W != Wm:
        return False
    if s0.scale is None:
        return len(segs) == 1
    # (the 64-channel form with a residual segment runs its residual chunks as a tail phase, one barrier
    # each: measured slower than the direct halo kernel, 1.14 vs 0.87 ms/step; it stays direct)
    return s0.silu and (len(segs) == 1 or (segs[1].view.C % 16 == 0 and TH == 8))


@dataclass
class GnbSums:
    """The GroupNorm(+SiLU) backward's per-channel sums of a data gradient dz, formed by the epilogue of
    the Winograd conv that writes dz (conv3x3_wino(..., gnb=)) instead of a wc_gn_bwd_reduce pass over
    it: part [B][splits][C][2] = (sum dy, sum dy*xhat), part3 [B][splits][C] = sum xhat (dx_sums), one
    split per (image, conv tile, wave row).  gn_backward(..., pre=) takes them."""
    x: 'View'
    sc0: torch.Tensor
    sh0: torch.Tensor
    gamma: Optional[torch.Tensor]
    beta: Optional[torch.Tensor]
    silu: bool
    part: torch.Tensor
    part3: Optional[torch.Tensor]
    splits: int

    @staticmethod
    def make(x: 'View', sc0: torch.Tensor, sh0: torch.Tensor, gamma: Optional[torch.Tensor],
             beta: Optional[torch.Tensor], silu: bool, dx_sums: bool = False) -> Optional['GnbSums']:
        """Buffers for the sums of a dz shaped like x (None where the Winograd tiling does not cover x)."""
        sp = _native.load().wc_conv3x3_wino_gnb_splits(x.C, x.H, x.W)
        if sp <= 0:
            return None
        dev = x.t.device
        return GnbSums(x, sc0, sh0, gamma, beta, silu,
                       torch.empty(x.B * sp * x.C * 2, dtype=torch.float32, device=dev),
                       torch.empty(x.B * sp * x.C, dtype=torch.float32, device=dev) if dx_sums else None, sp)

    def epi(self) -> '_native.GnbEpi':
        x = self.x
        return _native.GnbEpi(x.ptr, x.ldc, int(self.silu), self.sc0.data_ptr(), self.sh0.data_ptr(), _ptr(self.gamma),
                              _ptr(self.beta), self.part.data_ptr(), _ptr(self.part3), self.splits, 0)


def gnb_epilogue_enabled() -> bool:
    """The training backward forms the GroupNorm-backward sums in the data-gradient conv's epilogue
    (WC_TRAIN_GNB_EPI=0: a wc_gn_bwd_reduce pass over dz, A/B)."""
    return os.environ.get('WC_TRAIN_GNB_EPI', '1') != '0'


def conv3x3_wino(segs: Sequence[Seg], w: X6Weight, bias: Optional[torch.Tensor], out: View, *, Hm: int, Wm: int,
                 a_exp: int, a_bound: Optional[torch.Tensor] = None, temb: Optional[torch.Tensor] = None,
                 temb_ld: int = 0, res: Optional[View] = None, absmax: Optional[torch.Tensor] = None,
                 gn: Optional[GnPart] = None, gnb: Optional[GnbSums] = None):
    """The ResBlock 3x3 conv through the Winograd F(2,3)-along-x kernel (wc_conv3x3_wino_f16x3): segment 0
    with the GN+SiLU prologue (a_exp = f16x3_a_exp of that GroupNorm) and an optional fused 1x1
    residual under the per-image bound a_bound, or one raw segment under a_bound (a_exp = 60: the
    training data gradients)."""
    _req(w.data.is_cuda and w.data.is_contiguous() and w.order == 'wino', 'wino weight')
    _req(w.C0 == segs[0].view.C and w.C1 == (segs[1].view.C if len(segs) == 2 else 0), 'wino weight segments')
    raw = segs[0].scale is None
    _req((len(segs) == 1 and not raw) or a_bound is not None, 'a raw or residual wino segment needs a per-image A bound')
    if a_bound is not None:
        _req(a_bound.is_cuda and a_bound.dtype == torch.float32 and a_bound.numel() == segs[0].view.B, 'A bound')
    a = _conv_args(segs, w.N, bias, out, Hm, Wm, temb, temb_ld, res, (1, 1, 0, 0), None, 0, absmax, gn=gn)
    TH, BN = wino_tile(w.N)
    prof = _measuring()
    ab = _ptr(a_bound) if (len(segs) == 2 or raw) else None
    wbytes = float(w.data.numel() * w.data.element_size())  # the packed filter: read at least once as well
    if gnb is not None:
        # the data gradient dz of a GroupNorm(+SiLU): its backward sums formed in the epilogue
        xv = gnb.x
        _req(raw and len(segs) == 1 and xv.B == segs[0].view.B and xv.H == Hm and xv.W == Wm and xv.C == w.N
             and gnb.sc0.numel() == xv.B * w.N, 'GN-backward sums: the raw data-gradient conv of x')
        e = gnb.epi()
        _timed(f'conv3x3_wino_kernel<{TH}, {BN}, 0, false>', 'wc_conv3x3_wino_f16x3_gnb',
               _flops(segs, Hm, Wm, w.N) if prof else 0.0, ctypes.byref(a), w.data.data_ptr(), w.data.numel() * 2,
               int(a_exp), w.wsinv.data_ptr(), ab, ctypes.byref(e), _stream(),
               nbytes=(_abytes(segs, w.N, Hm * Wm, res) + 4.0 * xv.B * Hm * Wm * w.N + wbytes) if prof else 0.0,
               mfma=wino_mfma_flops(segs, Hm, Wm, w.N))
        return
    if not raw and wino_vsplit_wanted(segs, w.N, Hm, Wm):
        # segment 0 GN+SiLU'd, transformed and split once (not once per output-channel tile), then the
        # conv copies its halo planes by LDS-DMA (wc_wino_vsplit_f16x3 + wc_conv3x3_wino_f16x3_vp)
        v = segs[0].view
        nb = ctypes.c_int64()
        _native.call('wc_wino_vsplit_bytes', v.B, v.C, Hm, Wm, ctypes.byref(nb))
        vbuf = torch.empty(nb.value, dtype=torch.uint8, device=v.t.device)
        _timed('wino_vsplit_kernel', 'wc_wino_vsplit_f16x3', 0.0, ctypes.byref(a), int(a_exp), ab,
               vbuf.data_ptr(), nb.value, _stream(), nbytes=4.0 * v.B * Hm * Wm * v.C + nb.value)
        wide = _WINO_VP_WIDE and BN == 128 and w.N % 256 == 0
        _timed(f'conv3x3_wino_kernel<{TH}, {256 if wide else BN}, 3, {"true" if len(segs) == 2 else "false"}>',
               'wc_conv3x3_wino_f16x3_vp8' if wide else 'wc_conv3x3_wino_f16x3_vp', _flops(segs, Hm, Wm, w.N) if prof else 0.0,
               ctypes.byref(a), w.data.data_ptr(), w.data.numel() * 2, int(a_exp), w.wsinv.data_ptr(), ab,
               vbuf.data_ptr(), nb.value, _stream(),
               nbytes=(nb.value + _abytes(segs[1:], w.N, Hm * Wm, res, B=v.B) + wbytes) if prof else 0.0,
               mfma=wino_mfma_flops(segs, Hm, Wm, w.N))
        return
    _timed(f'conv3x3_wino_kernel<{TH}, {BN}, {0 if raw else 2}, {"true" if len(segs) == 2 else "false"}>',
           'wc_conv3x3_wino_f16x3', _flops(segs, Hm, Wm, w.N) if prof else 0.0,
           ctypes.byref(a), w.data.data_ptr(), w.data.numel() * 2, int(a_exp), w.wsinv.data_ptr(),
           ab, _stream(), nbytes=(_abytes(segs, w.N, Hm * Wm, res) + wbytes) if prof else 0.0,
           mfma=wino_mfma_flops(segs, Hm, Wm, w.N))


# Pre-split Winograd segment 0 (wc_wino_vsplit_f16x3) for convs with at least this many 128-channel
# output tiles (the redundancy the in-conv prologue pays: every output tile re-transforms the halo);
# 0 = never.  WC_WINO_VP sets it (A/B runs); set_wino_vsplit at run time.
_WINO_VP_MIN_TILES = int(os.environ.get('WC_WINO_VP', '4'))


# The pre-split convs with N % 256 == 0 on 8-wave 256-channel workgroups (wc_conv3x3_wino_f16x3_vp8):
# set while a forward is captured beside another concurrent one (the two-group sampling graph), where
# that form measured faster; alone the 4-wave form is (profiles/r06_wino_vp8_ab.txt).
_WINO_VP_WIDE = False


@contextlib.contextmanager
def wino_vp_wide(on: bool = True):
    """Inside the block the pre-split Winograd convs with N % 256 == 0 take the 8-wave form
    (WC_WINO_VP8=0: never, A/B runs)."""
    global _WINO_VP_WIDE
    prev, _WINO_VP_WIDE = _WINO_VP_WIDE, bool(on) and os.environ.get('WC_WINO_VP8', '1') != '0'
    try:
        yield
    finally:
        _WINO_VP_WIDE = prev


def set_wino_vsplit(min_tiles: int) -> int:
    """Use the pre-split Winograd form for GN+SiLU convs with >= min_tiles output-channel tiles of 128
    (0 = never); returns the previous setting."""
    global _WINO_VP_MIN_TILES
    prev, _WINO_VP_MIN_TILES = _WINO_VP_MIN_TILES, int(min_tiles)
    return prev


def wino_vsplit_wanted(segs: Sequence[Seg], N: int, Hm: int, Wm: int) -> bool:
    """Whether the conv takes the pre-split form: the tile threshold, and every constraint
    wc_wino_vsplit_f16x3 checks (otherwise the in-conv prologue form runs, which accepts more shapes)."""
    s0 = segs[0]
    v = s0.view
    return (_WINO_VP_MIN_TILES > 0 and N > 64 and -(-N // 128) >= _WINO_VP_MIN_TILES and s0.silu
            and s0.scale is not None and Wm % 16 == 0 and Wm <= 256 and v.W == Wm and v.H == Hm
            and v.C % 16 == 0 and v.ldc % 4 == 0 and v.ptr % 16 == 0)


def wino_mfma_flops(segs: Sequence[Seg], Hm: int, Wm: int, N: int, pieces: int = 3) -> float:
    """Dense f16 MFMA FLOPs one wc_conv3x3_wino_f16x3 launch issues: per output pair and 16 input channels
    12 K-steps on the 3x3 segment (the direct form's 18) and 2 on the 1x1 residual (its 2), each K-step
    `pieces` MFMAs (f16x3: h*h + h*l + l*h); N counted padded to the kernel's channel tile."""
    TH, BN = wino_tile(N)
    Np = -(-N // BN) * BN
    c0 = segs[0].view.C
    c1 = segs[1].view.C if len(segs) == 2 else 0
    return pieces * 2.0 * segs[0].view.B * Hm * Wm * Np * (6 * c0 + c1)


def conv_igemm_f16x3(segs: Sequence[Seg], w3: X6Weight, bias: Optional[torch.Tensor], out: Optional[View], *,
                     Hm: int, Wm: int, a_exp: int, a_bound: Optional[torch.Tensor] = None,
                     temb: Optional[torch.Tensor] = None, temb_ld: int = 0, res: Optional[View] = None,
                     out_map=(1, 1, 0, 0), out_nchw: Optional[torch.Tensor] = None,
                     absmax: Optional[torch.Tensor] = None, gn: Optional[GnPart] = None, gn_p64: int = 0):
    """conv_igemm's contract with segment 0 on f16x3; the caller guarantees |a| * 2^a_exp <= 2^14 for
    every segment-0 value after the prologue (a GroupNorm bound, f16x3_a_exp, or a bound the
    producer implies, e.g. an attention output by its V bound), or passes a_bound, a per-image
    float32[B] bound of those values (e.g. the producer's absmax), which lowers the exponent per
    image (tiles must not straddle images).  absmax: optional caller-zeroed float32[B] output."""
    _req(w3.data.is_cuda and w3.data.is_contiguous() and w3.order == 'f16x3n', 'f16x3 weight (natural order)')
    _req(w3.C0 == segs[0].view.C and w3.C1 == (segs[1].view.C if len(segs) == 2 else 0), 'f16x3 weight segments')
    a = _conv_args(segs, w3.N, bias, out, Hm, Wm, temb, temb_ld, res, out_map, out_nchw, 0, absmax, gn=gn,
                   gn_p64=gn_p64)
    bm, bn = (256, 64) if w3.N <= 64 else (128, 128)
    s0 = segs[0]
    pro = 0 if s0.scale is None else (2 if s0.silu else 1)
    unib = 'true' if (Hm * Wm) % bm == 0 else 'false'
    if a_bound is not None:
        _req(a_bound.is_cuda and a_bound.dtype == torch.float32 and a_bound.numel() == s0.view.B, 'A bound')
        _req(unib == 'true', 'a per-image A bound needs (Hm*Wm) % BM == 0')
    _timed(f'conv_igemm_x6_kernel<{bm}, {bn}, {pro}, {unib}, 0, true>', 'wc_conv_igemm_f16x3',
           _flops(segs, Hm, Wm, w3.N) if _measuring() else 0.0, ctypes.byref(a), w3.data.data_ptr(),
           w3.data.numel() * 2, int(a_exp), w3.wsinv.data_ptr(), _ptr(a_bound), _stream())


def pack_f16x3_s2d(w: torch.Tensor, C: int) -> X6Weight:
    """f16x3 pack of a 4x4 stride-2 conv weight for wc_conv4x4s2_f16x3.  w is [N][(ky*4 + kx)*C + c]
    (engine.pack_conv); the kernel's view is a 2x2 conv over the space-to-depth input, tap (a, b),
    channel (2py + px)*C + c <- w[n][c][2a + py][2b + px]."""
    N = w.shape[0]
    _req(w.shape[1] == 16 * C and C % 16 == 0, '4x4 conv weight shape')
    w2 = w.reshape(N, 2, 2, 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, 16 * C)  # (a, py, b, px) -> (a, b, py, px)
    return pack_f16x3(w2, 4 * C, ntaps=4, order='halo')


def pack_f16x3_convT(wt: torch.Tensor) -> X6Weight:
    """f16x3 pack of a ConvTranspose2d(Ci, N, 4, 2, 1) weight [Ci][N][4][4] for wc_convtr4x4s2_f16x3:
    per N tile the four parities (py, px) in order, each the 2x2-tap halo pack of
    engine.pack_convT(wt, py, px), under one per-channel scale."""
    from .diffusion_model.models.engine import pack_convT
    Ci, N = wt.shape[0], wt.shape[1]
    _req(Ci % 16 == 0, 'ConvT input channels % 16')
    parts = [pack_convT(wt, py, px)[1].to(wt.device) for py in (0, 1) for px in (0, 1)]
    if pack_device_enabled() and wt.is_cuda and os.environ.get('WC_PACK_DEVICE_CONVT', '1') != '0':
        # one device pack of the four parities side by side, columns ordered (parity, chunk, tap, c%16):
        # its natural step order is then the stacked per-parity halo order below, and its per-row scale
        # the common one (the row max over all four parities) -- one launch instead of ~60 torch ops
        wcat = torch.stack(parts, 1).view(N, 4, 4, Ci // 16, 16).permute(0, 1, 3, 2, 4).reshape(N, 16 * Ci)
        data, wsinv = _pack_dev(wcat, 16 * Ci, 0, 1, 'natural', 1, False)
        return X6Weight(data, N, x6_tile(N)[1], Ci, 0, 'f16x3t', wsinv)
    amax = torch.stack([p.abs().amax(1) for p in parts]).amax(0)
    packs = [pack_f16x3(p, Ci, ntaps=4, order='halo', amax=amax) for p in parts]
    T = packs[0].data.shape[0]
    data = torch.stack([pk.data for pk in packs], 1).reshape(T, -1).contiguous()
    return X6Weight(data, N, packs[0].BN, Ci, 0, 'f16x3t', packs[0].wsinv)


def convT4x4s2_f16x3_ok(seg: Seg, N: int) -> bool:
    """Shapes wc_convtr4x4s2_f16x3 takes (else the four implicit-GEMM parities)."""
    v = seg.view
    TH = x6_tile(N)[0]
    return v.H % TH == 0 and v.W % 16 == 0 and v.C % 16 == 0 and seg.scale is None and seg.stride == 1


def convT4x4s2_f16x3(seg: Seg, w3: X6Weight, bias: Optional[torch.Tensor], out: View, *, a_bound: torch.Tensor,
                     gn: Optional[GnPart] = None, res: Optional[View] = None, absmax: Optional[torch.Tensor] = None):
    """Up-sampling 4x4 / stride-2 / pad-1 transposed conv of a raw input on f16x3 in one launch
    (wc_convtr4x4s2_f16x3); out is the 2H x 2W view (+ res, same grid); a_bound = per-image max |x|;
    absmax: optional float32[B] raised to the max |out| written per image."""
    _req(w3.data.is_cuda and w3.data.is_contiguous() and w3.order == 'f16x3t', 'f16x3 ConvT weight')
    v = seg.view
    _req(w3.C0 == v.C and out.H == 2 * v.H and out.W == 2 * v.W, 'ConvT shapes')
    _req(a_bound.is_cuda and a_bound.dtype == torch.float32 and a_bound.numel() == v.B, 'A bound')
    a = _conv_args([seg], w3.N, bias, out, v.H, v.W, None, 0, res, (2, 2, 0, 0), None, 0, absmax, gn=gn)
    TH, BN = x6_tile(w3.N)
    _timed(f'conv3x3_x6_kernel<{TH}, {BN}, 0, false, true, false, false, 2> (ConvT 4x4/s2)', 'wc_convtr4x4s2_f16x3',
           2.0 * v.B * v.H * v.W * w3.N * 16 * v.C if _measuring() else 0.0, ctypes.byref(a),
           w3.data.data_ptr(), w3.data.numel() * 2, w3.wsinv.data_ptr(), _ptr(a_bound), _stream(),
           nbytes=_abytes([seg], w3.N, 4 * v.H * v.W))


def conv4x4s2_f16x3_ok(seg: Seg, N: int, Hm: int, Wm: int) -> bool:
    """Shapes wc_conv4x4s2_f16x3 takes (else use conv_igemm_f16x3)."""
    v = seg.view
    return (x6_tile(N)[1] == 128 and Hm % 8 == 0 and Wm % 16 == 0 and v.H == 2 * Hm and v.W == 2 * Wm
            and v.C % 16 == 0 and seg.scale is None and seg.stride == 2)


def conv4x4s2_f16x3(seg: Seg, w3: X6Weight, bias: Optional[torch.Tensor], out: View, *, Hm: int, Wm: int,
                    a_bound: torch.Tensor, absmax: Optional[torch.Tensor] = None, gn: Optional[GnPart] = None,
                    res: Optional[View] = None):
    """Down-sampling 4x4 / stride-2 / pad-1 conv of a raw input on f16x3 (wc_conv4x4s2_f16x3): the
    halo-tiled kernel over the space-to-depth view; a_bound = per-image max |x| (the producer's absmax);
    res: optional view added in the epilogue."""
    _req(w3.data.is_cuda and w3.data.is_contiguous() and w3.order == 'f16x3s', 'f16x3 s2d weight')
    _req(w3.C0 == 4 * seg.view.C and w3.C1 == 0, 'f16x3 s2d weight channels')
    _req(a_bound.is_cuda and a_bound.dtype == torch.float32 and a_bound.numel() == seg.view.B, 'A bound')
    a = _conv_args([seg], w3.N, bias, out, Hm, Wm, None, 0, res, (1, 1, 0, 0), None, 0, absmax, gn=gn)
    _timed('conv3x3_x6_kernel<8, 128, 0, false, true, false, false, true> (s2d 4x4/s2)', 'wc_conv4x4s2_f16x3',
           _flops([seg], Hm, Wm, w3.N) if _measuring() else 0.0, ctypes.byref(a), w3.data.data_ptr(),
           w3.data.numel() * 2, w3.wsinv.data_ptr(), _ptr(a_bound), _stream(), nbytes=_abytes([seg], w3.N, Hm * Wm))


def qkv_presplit_ok(B: int, N: int, C: int, heads: int) -> bool:
    """True when the attention of (B, N tokens, C, heads) can run on the pre-split projection
    (wc_conv_igemm_f16x3_qkv + wc_attention_fwd_f16x3_presplit)."""
    return C % heads == 0 and (C // heads) % 32 == 0 and N % 128 == 0 and 3 * C > 64


def conv_igemm_f16x3_qkv(seg: Seg, w3: X6Weight, bias: Optional[torch.Tensor], qkv3: torch.Tensor, *, Hm: int,
                         Wm: int, a_exp: int, C: int, heads: int, exps: Tuple[int, int, int]):
    """The attention in-projection (1x1 conv, GN prologue) on f16x3 writing the pre-split form
    (wc_conv_igemm_f16x3_qkv): qkv3 is an int16 tensor of B * 6 * C * Hm * Wm elements."""
    _req(w3.data.is_cuda and w3.data.is_contiguous() and w3.order == 'f16x3n' and w3.N == 3 * C, 'f16x3 qkv weight')
    B = seg.view.B
    _req(qkv3.is_cuda and qkv3.dtype == torch.int16 and qkv3.is_contiguous() and qkv3.numel() == B * 6 * C * Hm * Wm,
         'pre-split qkv buffer: int16, B * 6 * C * HW elements')
    a = _conv_args([seg], w3.N, bias, None, Hm, Wm, None, 0, None, (1, 1, 0, 0), None, 0, out_dummy=True)
    ex = (ctypes.c_int * 3)(*[int(e) for e in exps])  # host array, read during the call
    pro = 0 if seg.scale is None else (2 if seg.silu else 1)
    _timed(f'conv_igemm_x6_kernel<128, 128, {pro}, true, 0, true> (qkv pre-split)', 'wc_conv_igemm_f16x3_qkv',
           _flops([seg], Hm, Wm, w3.N) if _measuring() else 0.0, ctypes.byref(a), w3.data.data_ptr(),
           w3.data.numel() * 2, int(a_exp), w3.wsinv.data_ptr(), qkv3.data_ptr(), C, heads,
           ctypes.cast(ex, ctypes.c_void_p), _stream())


def proj_pa_enabled() -> bool:
    """Attention projections on a pre-split A operand (wc_split_f16x3_tiled + wc_proj_f16x3[_qkv]);
    WC_PROJ_PA=0 keeps the register-staged implicit GEMM (for A/B measurement)."""
    return os.environ.get('WC_PROJ_PA', '1') != '0'


def proj_pa_ok(v: View, N: int) -> bool:
    """Shapes the pre-split projection takes: HW % 128 == 0, C % 32 == 0, N % 128 == 0, aligned view."""
    return (v.H * v.W) % 128 == 0 and v.C % 32 == 0 and N % 128 == 0 and v.ptr % 16 == 0 and v.ldc % 4 == 0


def split_f16x3_tiled(v: View, a_exp: int, scale: Optional[torch.Tensor] = None,
                      shift: Optional[torch.Tensor] = None, silu: bool = False) -> torch.Tensor:
    """The rows of v (optionally GN-affine, + SiLU) x 2^a_exp as two fp16 pieces in the projection
    GEMM's LDS stage order (wc_split_f16x3_tiled); an int16 tensor of 2 * B*H*W*C elements."""
    v.check()
    _req(proj_pa_ok(v, 128), 'pre-split rows: HW % 128 == 0, C % 32 == 0, 16-byte aligned view')
    if scale is not None:
        _req(scale.shape == (v.B, v.C) and shift.shape == (v.B, v.C) and scale.is_contiguous()
             and shift.is_contiguous() and scale.dtype == torch.float32, 'GN affine [B][C]')
    a3 = torch.empty(2 * v.B * v.H * v.W * v.C, dtype=torch.int16, device=v.t.device)
    _timed('split_tiled_kernel', 'wc_split_f16x3_tiled', 8.0 * v.B * v.H * v.W * v.C if _measuring() else 0.0,
           v.ptr, v.ldc, v.B, v.H * v.W, v.C, _ptr(scale), _ptr(shift), int(silu), int(a_exp), a3.data_ptr(),
           a3.numel() * 2, _stream())
    return a3


def set_proj_tile(rows: int) -> int:
    """wc_proj_set_tile: form of the pre-split projection GEMMs (0 the measured default, 256 or 128 rows);
    returns the previous setting."""
    prev = _native.set_selector('wc_proj_set_tile', int(rows), lambda v: v in (0, 128, 256))
    return prev


def proj_f16x3(v: View, a3: torch.Tensor, w3: 'X6Weight', bias: Optional[torch.Tensor], out: View, *, a_exp: int,
               res: Optional[View] = None, absmax: Optional[torch.Tensor] = None, gn: Optional[GnPart] = None):
    """out = (a3 . W^T) x 2^-(a_exp + sW) + bias (+ res): the 1x1 projection of the view v that a3 was
    split from (wc_proj_f16x3)."""
    _req(w3.data.is_cuda and w3.data.is_contiguous() and w3.order == 'f16x3n' and w3.C0 == v.C and w3.C1 == 0,
         'f16x3 projection weight (natural order)')
    seg = Seg(v, [(0, 0)])
    a = _conv_args([seg], w3.N, bias, out, v.H, v.W, None, 0, res, (1, 1, 0, 0), None, 0, absmax, gn=gn)
    _timed('conv_igemm_x6_kernel<128, 128, 0, true, 0, true> (pre-split A)', 'wc_proj_f16x3',
           _flops([seg], v.H, v.W, w3.N) if _measuring() else 0.0, ctypes.byref(a), a3.data_ptr(),
           a3.numel() * 2, w3.data.data_ptr(), w3.data.numel() * 2, int(a_exp), w3.wsinv.data_ptr(), _stream())


def proj_f16x3_qkv(v: View, a3: torch.Tensor, w3: 'X6Weight', bias: Optional[torch.Tensor], qkv3: torch.Tensor, *,
                   a_exp: int, C: int, heads: int, exps: Tuple[int, int, int]):
    """conv_igemm_f16x3_qkv on the pre-split (GN already applied) A operand a3 (wc_proj_f16x3_qkv)."""
    _req(w3.data.is_cuda and w3.data.is_contiguous() and w3.order == 'f16x3n' and w3.N == 3 * C, 'f16x3 qkv weight')
    B = v.B
    _req(qkv3.is_cuda and qkv3.dtype == torch.int16 and qkv3.is_contiguous()
         and qkv3.numel() == B * 6 * C * v.H * v.W, 'pre-split qkv buffer: int16, B * 6 * C * HW elements')
    seg = Seg(v, [(0, 0)])
    a = _conv_args([seg], w3.N, bias, None, v.H, v.W, None, 0, None, (1, 1, 0, 0), None, 0, out_dummy=True)
    ex = (ctypes.c_int * 3)(*[int(e) for e in exps])  # host array, read during the call
    _timed('conv_igemm_x6_kernel<128, 128, 0, true, 0, true> (qkv pre-split, pre-split A)', 'wc_proj_f16x3_qkv',
           _flops([seg], v.H, v.W, w3.N) if _measuring() else 0.0, ctypes.byref(a), a3.data_ptr(),
           a3.numel() * 2, w3.data.data_ptr(), w3.data.numel() * 2, int(a_exp), w3.wsinv.data_ptr(),
           qkv3.data_ptr(), C, heads, ctypes.cast(ex, ctypes.c_void_p), _stream())


def attention_presplit(qkv3: torch.Tensor, out: torch.Tensor, B: int, N: int, C: int, heads: int,
                       exps: Tuple[int, int, int]):
    """f16x3 attention on the pre-split projection of conv_igemm_f16x3_qkv (same exps)."""
    _req(qkv3.is_cuda and qkv3.dtype == torch.int16 and qkv3.numel() == B * 6 * C * N, 'pre-split qkv buffer')
    _req(out.shape == (B * N, C) and out.is_contiguous(), 'attention output shape')
    d = C // heads
    _timed(f'attention_x6_kernel<{d}, true> (pre-split)', 'wc_attention_fwd_f16x3_presplit', 4.0 * B * N * N * C,
           qkv3.data_ptr(), out.data_ptr(), C, B, N, C, heads, float(d)**-0.5, *[int(e) for e in exps], _stream())


def attention_presplit_a3(qkv3: torch.Tensor, B: int, N: int, C: int, heads: int,
                          exps: Tuple[int, int, int]) -> torch.Tensor:
    """attention_presplit writing the out-projection's pre-split A operand (O x 2^exps[2] in the
    split_f16x3_tiled layout, wc_attention_fwd_f16x3_presplit_a3): an int16 tensor of 2*B*N*C."""
    _req(qkv3.is_cuda and qkv3.dtype == torch.int16 and qkv3.numel() == B * 6 * C * N, 'pre-split qkv buffer')
    _req(N % 128 == 0 and C % 32 == 0, 'pre-split attention output: N % 128 == 0, C % 32 == 0')
    a3 = torch.empty(2 * B * N * C, dtype=torch.int16, device=qkv3.device)
    d = C // heads
    _timed(f'attention_x6_kernel<{d}, true> (pre-split)', 'wc_attention_fwd_f16x3_presplit_a3', 4.0 * B * N * N * C,
           qkv3.data_ptr(), a3.data_ptr(), a3.numel() * 2, B, N, C, heads, float(d)**-0.5, *[int(e) for e in exps],
           _stream())
    return a3


def x6_eligible(segs: Sequence[Seg], N: int, Hm: int, Wm: int) -> bool:
    """True when wc_conv3x3_x6 accepts this conv (mirrors its host checks; output must be a plain
    NHWC view on the same grid)."""
    TH, _ = x6_tile(N)
    s0 = segs[0]
    v = s0.view
    ok = (list(s0.taps) == TAPS3 and s0.stride == 1 and v.C % 16 == 0 and v.H == Hm and v.W == Wm
          and Hm % TH == 0 and Wm % 16 == 0 and v.B * v.H * v.W * v.ldc * 4 < 2**31)
    if len(segs) == 2:
        s1 = segs[1]
        ok = ok and (list(s1.taps) == [(0, 0)] and s1.stride == 1 and s1.scale is None and s1.view.C % 16 == 0
                     and s1.view.H == Hm and s1.view.W == Wm and s1.view.B * Hm * Wm * s1.view.ldc * 4 < 2**31)
    return ok


def conv3x3_x6(segs: Sequence[Seg], w6: X6Weight, bias: Optional[torch.Tensor], out: View, *, Hm: int, Wm: int,
               temb: Optional[torch.Tensor] = None, temb_ld: int = 0, res: Optional[View] = None, act: int = 0,
               absmax: Optional[torch.Tensor] = None, gn: Optional[GnPart] = None):
    """3x3 stride-1 conv (+ fused 1x1 residual segment) on bf16x6 split-precision MFMA."""
    _req(w6.data.is_cuda and w6.data.is_contiguous() and w6.order == 'halo', 'x6 weight (halo order)')
    _req(w6.C0 == segs[0].view.C and w6.C1 == (segs[1].view.C if len(segs) == 2 else 0), 'x6 weight segments')
    a = _conv_args(segs, w6.N, bias, out, Hm, Wm, temb, temb_ld, res, (1, 1, 0, 0), None, act, absmax, gn=gn)
    TH, BN = x6_tile(w6.N)
    s0 = segs[0]
    pro = 0 if s0.scale is None else (2 if s0.silu else 1)
    res_seg = 'true' if len(segs) == 2 else 'false'
    _timed(f'conv3x3_x6_kernel<{TH}, {BN}, {pro}, {res_seg}, false, false>', 'wc_conv3x3_x6',
           _flops(segs, Hm, Wm, w6.N) if _measuring() else 0.0, ctypes.byref(a), w6.data.data_ptr(),
           w6.data.numel() * 2, _stream())


def conv_igemm_x6(segs: Sequence[Seg], w6: X6Weight, bias: Optional[torch.Tensor], out: Optional[View], *, Hm: int,
                  Wm: int, temb: Optional[torch.Tensor] = None, temb_ld: int = 0, res: Optional[View] = None,
                  out_map=(1, 1, 0, 0), out_nchw: Optional[torch.Tensor] = None, act: int = 0,
                  absmax: Optional[torch.Tensor] = None, gn: Optional[GnPart] = None, gn_p64: int = 0):
    """conv_igemm's contract (any taps, strides, output map) on bf16x6 split-precision MFMA."""
    _req(w6.data.is_cuda and w6.data.is_contiguous() and w6.order == 'natural', 'x6 weight (natural order)')
    _req(w6.C0 == segs[0].view.C and w6.C1 == (segs[1].view.C if len(segs) == 2 else 0), 'x6 weight segments')
    a = _conv_args(segs, w6.N, bias, out, Hm, Wm, temb, temb_ld, res, out_map, out_nchw, act, absmax, gn=gn,
                   gn_p64=gn_p64)
    bm, bn = (256, 64) if w6.N <= 64 else (128, 128)
    s0 = segs[0]
    pro = 0 if s0.scale is None else (2 if s0.silu else 1)
    unib = 'true' if (Hm * Wm) % bm == 0 else 'false'
    _timed(f'conv_igemm_x6_kernel<{bm}, {bn}, {pro}, {unib}, {act}, false>', 'wc_conv_igemm_x6',
           _flops(segs, Hm, Wm, w6.N) if _measuring() else 0.0, ctypes.byref(a), w6.data.data_ptr(),
           w6.data.numel() * 2, _stream())


def gn_partials(v: View, gp: GnPart):
    """Fill the tile partials of view v (channels [v.c0, v.c0 + v.C) of gp's tensor) from memory."""
    v.check()
    _req(gp.covers(v), 'GN partials: view of the partials tensor, 32-channel aligned')
    _timed('gn_partials_kernel', 'wc_gn_partials', 4.0 * v.B * v.H * v.W * v.C, v.ptr, v.ldc, v.B, v.H * v.W, v.C,
           gp.part.data_ptr(), gp.ncb, gp.sw, v.c0, _stream())


def gn_conv_ok(out: Optional[View], gn: Optional[GnPart], N: int, Hm: int, Wm: int, bm: Optional[int] = None) -> bool:
    """True when a split-precision conv writing `out` can emit gn's tile partials from its epilogue
    (mirrors the host checks of wc_conv3x3_x6 / wc_conv_igemm_x6; bm = the implicit GEMM's M tile)."""
    return (gn is not None and out is not None and gn.covers(out) and N == out.C and N % 32 == 0
            and (Hm * Wm) % 64 == 0 and (bm is None or (Hm * Wm) % bm == 0))


def gn_affine(v: View, gamma: Optional[torch.Tensor], beta: Optional[torch.Tensor], eps: float = 1e-5,
              groups: int = 8, bound: bool = False, part: Optional[GnPart] = None):
    """GroupNorm statistics of a view -> per-(b, c) (scale, shift) so that GN(x) = x*scale + shift;
    with bound=True also the per-image bound of |x| (wc_gn_finalize_bound) as a third result.
    With `part` (tile partials of v's tensor, already written by v's producers) no pass over v."""
    v.check()
    B, HW, C = v.B, v.H * v.W, v.C
    if part is not None:
        _req(part.covers(v) and (C // groups) % part.sw == 0, 'GN partials do not tile these groups')
        scale = torch.empty((B, C), dtype=torch.float32, device=v.t.device)
        shift = torch.empty_like(scale)
        bnd = torch.empty((B, ), dtype=torch.float32, device=v.t.device) if bound else None
        _native.call('wc_gn_finalize_part', part.part.data_ptr(), B, HW, part.ncb, part.sw, v.c0, C, groups,
                     _ptr(gamma), _ptr(beta), eps, scale.data_ptr(), shift.data_ptr(), _ptr(bnd), _stream())
        return (scale, shift, bnd) if bound else (scale, shift)
    lib = _native.load()
    splits = lib.wc_gn_num_splits(B, HW, C)
    part = torch.empty((B, splits, groups, 2), dtype=torch.float32, device=v.t.device)
    scale = torch.empty((B, C), dtype=torch.float32, device=v.t.device)
    shift = torch.empty_like(scale)
    s = _stream()
    # HBM-bound: the algorithmic bytes are one read of the view (partials are negligible)
    _timed('gn_stats_rows_kernel' if C // 4 <= 256 else 'gn_stats_kernel', 'wc_gn_stats', 4.0 * B * HW * C,
           v.ptr, B, HW, C, v.ldc, groups, part.data_ptr(), s)
    if bound:
        bnd = torch.empty((B, ), dtype=torch.float32, device=v.t.device)
        _native.call('wc_gn_finalize_bound', part.data_ptr(), B, HW, C, groups, _ptr(gamma), _ptr(beta), eps,
                     scale.data_ptr(), shift.data_ptr(), bnd.data_ptr(), s)
        return scale, shift, bnd
    _native.call('wc_gn_finalize', part.data_ptr(), B, HW, C, groups, _ptr(gamma), _ptr(beta), eps,
                 scale.data_ptr(), shift.data_ptr(), s)
    return scale, shift


def attention(qkv: torch.Tensor, out: torch.Tensor, B: int, N: int, C: int, heads: int, precision: str = 'fp32',
              exps: Optional[Tuple[int, int, int]] = None):
    """softmax(Q K^T / sqrt(d)) V per (batch, head) over qkv rows [q | k | v].  'bf16x6' / 'f16x3'
    run the split-precision kernel when the head dim is a multiple of 32 (else the fp32-MFMA
    kernel); 'f16x3' needs exps = (q, k, v) power-of-two exponents from attention_f16x3_exps."""
    _req(qkv.shape == (B * N, 3 * C) and qkv.is_contiguous(), 'qkv shape')
    _req(out.shape == (B * N, C) and out.is_contiguous(), 'attention output shape')
    _req(precision in CONV_PRECISIONS, f'attention precision {precision!r}')
    d = C // heads
    split = precision != 'fp32' and d % 32 == 0
    flops = 4.0 * B * N * N * C
    args = (qkv.data_ptr(), 3 * C, out.data_ptr(), C, B, N, C, heads, float(d)**-0.5)
    if split and precision == 'f16x3':
        _req(exps is not None, 'f16x3 attention needs (q, k, v) exponents')
        _timed(f'attention_x6_kernel<{d}, true>', 'wc_attention_fwd_f16x3', flops, *args, *[int(e) for e in exps],
               _stream())
    elif split:
        _timed(f'attention_x6_kernel<{d}, false>', 'wc_attention_fwd_x6', flops, *args, _stream())
    else:
        _timed(f'attention_kernel<{d}>', 'wc_attention_fwd', flops, *args, _stream())


def attention_f16x3_exps(w_in: torch.Tensor, b_in: torch.Tensor, gamma_absmax: float, beta_absmax: float,
                         n_group: int) -> Tuple[int, int, int]:
    """Exponents (q, k, v) for wc_attention_fwd_f16x3 when qkv = GN(Y) W_in^T + b_in (see
    attention_exps_from_norms)."""
    l1 = w_in.detach().double().abs().sum(1).cpu()
    babs = b_in.detach().double().abs().cpu()
    return attention_exps_from_norms(l1, babs, gamma_absmax, beta_absmax, n_group)


def attention_exps_from_norms(l1: torch.Tensor, babs: torch.Tensor, gamma_absmax: float, beta_absmax: float,
                              n_group: int) -> Tuple[int, int, int]:
    """The GroupNorm output is bounded by sqrt(n - 1) max|gamma| + max|beta| (Samuelson), so row i of
    the projection by l1[i] times that plus babs[i] (l1 = row L1 norms of W_in, babs = |b_in|, host
    tensors); each exponent puts the max bound of its q / k / v block at <= 2^14."""
    import math
    C = l1.shape[0] // 3
    bound_y = math.sqrt(max(n_group - 1, 1)) * gamma_absmax + beta_absmax
    exps = []
    for part in range(3):
        sl = slice(part * C, (part + 1) * C)
        bound = float((l1[sl] * bound_y + babs[sl]).max())
        if not math.isfinite(bound):
            raise RuntimeError('weatherconverter_amd: non-finite attention projection bound')
        exps.append(0 if bound <= 0 else max(-60, min(60, math.floor(math.log2(2.0**14 / bound)))))
    return tuple(exps)


def temb(t: torch.Tensor, w1, b1, w2, b2, proj_w, proj_b) -> torch.Tensor:
    _req(t.dtype == torch.int64 and t.is_cuda and t.dim() == 1, 'timesteps must be a 1-D int64 device tensor')
    nt = t.shape[0]
    D = w1.shape[0]
    P = proj_w.shape[0]
    out = torch.empty((nt, P), dtype=torch.float32, device=t.device)
    _native.call('wc_temb', t.data_ptr(), nt, D, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                 proj_w.data_ptr(), proj_b.data_ptr(), P, out.data_ptr(), _stream())
    return out


def conv_in(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: View, gn: Optional[GnPart] = None):
    """The stem conv (wc_conv_in); with gn (the output's tile partials, a 3 -> 64 stem) the same launch
    writes the output's GroupNorm partials (wc_conv_in_gn).  Returns True when it did."""
    _req(x.is_contiguous() and x.dtype == torch.float32 and x.dim() == 4, 'conv_in input must be NCHW fp32')
    B, Cin, H, W = x.shape
    out.check()
    _req(out.H == H and out.W == W and out.B == B, 'conv_in output view shape')
    if gn is not None and gn.covers(out) and Cin == 3 and out.C == 64 and (H * W) % 64 == 0:
        # the weight transposed to [Cin*9][Cout], cached on the weight tensor (rebuilt if it changes in place)
        wt = getattr(w, '_wc_t', None)
        if wt is None or w._wc_t_version != w._version:
            wt = w.reshape(out.C, Cin * 9).t().contiguous()
            w._wc_t, w._wc_t_version = wt, w._version
        _native.call('wc_conv_in_gn', x.data_ptr(), B, Cin, H, W, wt.data_ptr(), b.data_ptr(), out.C, out.ptr,
                     out.ldc, gn.part.data_ptr(), gn.ncb, gn.sw, out.c0, _stream())
        return True
    _native.call('wc_conv_in', x.data_ptr(), B, Cin, H, W, w.data_ptr(), b.data_ptr(), out.C, out.ptr, out.ldc,
                 _stream())
    return False


def pack_head(w: torch.Tensor) -> torch.Tensor:
    """conv_out weight (NO, C, 3, 3) -> wc_head_conv layout [C/16][9][16][4] (outputs zero-padded)."""
    NO, C = w.shape[0], w.shape[1]
    _req(NO <= 4 and C % 16 == 0 and tuple(w.shape[2:]) == (3, 3), 'head conv: <= 4 outputs, C % 16 == 0, 3x3')
    wp = torch.zeros((C // 16, 9, 16, 4), dtype=torch.float32, device=w.device)
    wt = w.detach().float().reshape(NO, C // 16, 16, 9)  # [n][chunk][c][tap]
    wp[..., :NO] = wt.permute(1, 3, 2, 0)
    return wp.contiguous()


def head_conv(x: View, scale: torch.Tensor, shift: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor,
              out: torch.Tensor):
    """GN-affine + SiLU + 3x3 conv to <= 4 channels, NCHW output (wc_head_conv)."""
    x.check()
    B, NO = out.shape[0], out.shape[1]
    _req(out.is_contiguous() and out.shape == (x.B, NO, x.H, x.W) and bias.numel() >= NO, 'head output shape')
    _req(w_packed.shape == (x.C // 16, 9, 16, 4), 'head weight layout')
    _timed('head_conv_kernel', 'wc_head_conv', 2.0 * x.B * x.H * x.W * NO * 9 * x.C if _measuring() else 0.0,
           x.ptr, x.ldc, scale.data_ptr(), shift.data_ptr(), x.B, x.H, x.W, x.C, w_packed.data_ptr(),
           bias.data_ptr(), NO, out.data_ptr(), _stream())


def smallconv_enabled() -> bool:
    """Training's 3-channel convs (the head's forward / weight / data gradient, the stem's weight
    gradient) on their fp32 VALU kernels (WC_TRAIN_SMALLCONV=0: the generic implicit GEMMs, for A/B)."""
    return os.environ.get('WC_TRAIN_SMALLCONV', '1') != '0'


def head_dgrad(g: torch.Tensor, w: torch.Tensor, dz: View):
    """Data gradient of conv_out (unet_base.py:485) from the NCHW loss gradient g (B, NO, H, W): the
    transposed 3x3 conv into the NHWC view dz (C = conv_out.in_channels), fp32 (wc_head_dgrad)."""
    dz.check()
    B, NO, H, W = g.shape
    _req(g.is_cuda and g.dtype == torch.float32 and g.is_contiguous(), 'head_dgrad: contiguous fp32 NCHW gradient')
    _req(tuple(w.shape) == (NO, dz.C, 3, 3) and dz.B == B and dz.H == H and dz.W == W, 'head_dgrad shapes')
    wp = w.detach().float().permute(0, 2, 3, 1).contiguous()  # [NO][ky][kx][C]
    _timed(f'head_dgrad_kernel<{NO}>', 'wc_head_dgrad', 2.0 * B * H * W * NO * 9 * dz.C, g.data_ptr(), B, NO, H, W,
           wp.data_ptr(), dz.C, dz.ptr, dz.ldc, _stream(), nbytes=4.0 * B * H * W * (NO + dz.C))


def _small_work(B: int, H: int, W: int, L: int, dev) -> torch.Tensor:
    n = _native.load().wc_small_wgrad_workspace(B, H, W, L)
    _req(n > 0, 'small wgrad workspace')
    return torch.empty(n, dtype=torch.float32, device=dev)


def head_wgrad(x: View, scale: torch.Tensor, shift: torch.Tensor, g: torch.Tensor, dw: torch.Tensor,
               accumulate: bool = False):
    """Weight gradient of conv_out: dw [NO][C][3][3] (+)= sum over pixels of g (NCHW) times the forward's
    SiLU(x*scale + shift) at each tap, fp32, fixed-order reduction (wc_head_wgrad)."""
    x.check()
    B, NO, H, W = g.shape
    _req(g.is_cuda and g.dtype == torch.float32 and g.is_contiguous(), 'head_wgrad: contiguous fp32 NCHW gradient')
    _req(x.B == B and x.H == H and x.W == W and tuple(dw.shape) == (NO, x.C, 3, 3) and dw.is_contiguous()
         and dw.dtype == torch.float32, 'head_wgrad shapes')
    work = _small_work(B, H, W, dw.numel(), dw.device)
    _timed('head_wgrad_kernel', 'wc_head_wgrad', 2.0 * B * H * W * NO * 9 * x.C, x.ptr, x.ldc, scale.data_ptr(),
           shift.data_ptr(), g.data_ptr(), B, NO, H, W, x.C, work.data_ptr(), work.numel(), dw.data_ptr(),
           int(accumulate), _stream(), nbytes=4.0 * B * H * W * (NO + x.C))


def stem_wgrad(x: torch.Tensor, g: View, dw: torch.Tensor, accumulate: bool = False):
    """Weight gradient of conv_in (unet_base.py:400): dw [N][3][3][3] (+)= sum over pixels of g (NHWC
    view, N channels) times the NCHW input x at each tap, fp32, fixed-order reduction (wc_stem_wgrad)."""
    g.check()
    B, CI, H, W = x.shape
    _req(x.is_cuda and x.dtype == torch.float32 and x.is_contiguous(), 'stem_wgrad: contiguous fp32 NCHW input')
    _req(g.B == B and g.H == H and g.W == W and tuple(dw.shape) == (g.C, CI, 3, 3) and dw.is_contiguous()
         and dw.dtype == torch.float32, 'stem_wgrad shapes')
    work = _small_work(B, H, W, dw.numel(), dw.device)
    _timed('stem_wgrad_kernel', 'wc_stem_wgrad', 2.0 * B * H * W * CI * 9 * g.C, x.data_ptr(), CI, g.ptr, g.ldc, B, H,
           W, g.C, work.data_ptr(), work.numel(), dw.data_ptr(), int(accumulate), _stream(),
           nbytes=4.0 * B * H * W * (CI + g.C))


def ddpm_step(x: torch.Tensor, eps: torch.Tensor, out: torch.Tensor, beta: float, s1m: float, sqrt_alpha: float,
              sigma: float, *, z: Optional[torch.Tensor] = None, mode: int = _native.NOISE_NONE, seed: int = 0,
              sample0: int = 0, step: int = 0, sz_out: Optional[torch.Tensor] = None):
    def dev_f32(v, what):  # the kernel reads / writes float4 vectors of device memory
        _req(v.is_cuda and v.dtype == torch.float32 and v.is_contiguous() and v.data_ptr() % 16 == 0,
             f'ddpm_step {what}: contiguous 16-byte-aligned fp32 device tensor')

    _req(x.shape == eps.shape == out.shape, 'ddpm_step shapes')
    for v, what in ((x, 'x'), (eps, 'eps'), (out, 'out')):
        dev_f32(v, what)
    if mode == _native.NOISE_TENSOR:
        _req(z is not None and z.shape == x.shape, 'noise tensor shape')
        dev_f32(z, 'z')
    B = x.shape[0]
    per = x.numel() // B
    if sz_out is not None:
        _req(sz_out.shape == x.shape, 'sz_out shape')
        dev_f32(sz_out, 'sz_out')
    _native.call('wc_ddpm_step', x.data_ptr(), eps.data_ptr(), _ptr(z), out.data_ptr(), _ptr(sz_out), B, per, beta, s1m,
                 sqrt_alpha, sigma, mode, seed & ((1 << 64) - 1), sample0, step, _stream())


def add_noise(x0: torch.Tensor, noise: torch.Tensor, coef_a: torch.Tensor, coef_b: torch.Tensor) -> torch.Tensor:
    _req(x0.shape == noise.shape and x0.is_contiguous() and noise.is_contiguous(), 'add_noise shapes')
    _req(x0.is_cuda and noise.is_cuda and x0.dtype == torch.float32 and noise.dtype == torch.float32
         and x0.data_ptr() % 16 == 0 and noise.data_ptr() % 16 == 0, 'add_noise: 16-byte-aligned fp32 device tensors')
    _req(coef_a.is_cuda and coef_b.is_cuda and coef_a.dtype == torch.float32 and coef_b.dtype == torch.float32,
         'add_noise coefficients: fp32 device tensors')
    B = x0.shape[0]
    _req(coef_a.numel() == B and coef_b.numel() == B, 'add_noise coefficient count')
    out = torch.empty_like(x0)
    _native.call('wc_add_noise', x0.data_ptr(), noise.data_ptr(), coef_a.contiguous().data_ptr(),
                 coef_b.contiguous().data_ptr(), out.data_ptr(), B, x0.numel() // B, _stream())
    return out


def mse_loss(pred: torch.Tensor, target: torch.Tensor, grad: bool = False):
    """torch.nn.MSELoss() (mean) on the device (wc_mse_loss); returns the 0-dim loss, and with
    grad=True also d loss / d pred = 2 (pred - target) / n from the same pass."""
    _req(pred.shape == target.shape and pred.is_cuda and target.is_cuda and pred.dtype == torch.float32
         and target.dtype == torch.float32, 'mse_loss operands: equal-shape fp32 device tensors')
    pred, target = pred.contiguous(), target.contiguous()
    n = pred.numel()
    lib = _native.load()
    ws = torch.empty(lib.wc_mse_workspace_doubles(), dtype=torch.float64, device=pred.device)
    loss = torch.empty((), dtype=torch.float32, device=pred.device)
    g = torch.empty_like(pred) if grad else None
    _native.call('wc_mse_loss', pred.data_ptr(), target.data_ptr(), n, _ptr(g), 2.0 / n, ws.data_ptr(),
                 loss.data_ptr(), _stream())
    return (loss, g) if grad else loss


def philox_normal(shape, device, seed: int, sample0: int = 0, step: int = 0) -> torch.Tensor:
    out = torch.empty(shape, dtype=torch.float32, device=device)
    B = shape[0]
    _native.call('wc_philox_normal', out.data_ptr(), B, out.numel() // B, seed & ((1 << 64) - 1), sample0, step,
                 _stream())
    return out


def sgg_update(grad: torch.Tensor, mu: torch.Tensor, sigma: torch.Tensor, lam: float,
               std=(0.229, 0.224, 0.225), batch_axis_sum: bool = False):
    """Returns (xt, magnitude) — see include/wc_kernels.h wc_sgg_update."""
    nb, c3, S, S2 = mu.shape
    _req(c3 == 3 and S == S2 and sigma.shape == mu.shape, 'mu/sigma must be (nb, 3, S, S)')
    _req(grad.shape == (nb, 3, 4 * S, 4 * S), 'grad must be (nb, 3, 4S, 4S)')
    grad, mu, sigma = grad.contiguous(), mu.contiguous(), sigma.contiguous()
    xt = torch.empty_like(mu)
    mag = torch.empty((3 if batch_axis_sum else nb, S, S), dtype=torch.float32, device=mu.device)
    # algorithmic bytes: the (nb, 3, 4S, 4S) gradient, mu, sigma and xt (nb, 3, S, S), the magnitude (S, S) per plane
    nbytes = 4.0 * nb * S * S * (48 + 9) + 4.0 * mag.numel()
    _timed('sgg_kernel', 'wc_sgg_update', 0.0, grad.data_ptr(), mu.data_ptr(), sigma.data_ptr(), xt.data_ptr(),
           mag.data_ptr(), nb, S, float(lam), float(std[0]), float(std[1]), float(std[2]), int(batch_axis_sum),
           _stream(), nbytes=nbytes)
    return xt, mag


def dwconv(x: View, w: torch.Tensor, bias: Optional[torch.Tensor], out: View, K: int):
    """Depthwise KxK conv, padding K//2 (wc_dwconv); w: (C, 1, K, K) or (C, K*K) fp32, C = x.C."""
    x.check()
    out.check()
    _req(out.B == x.B and out.H == x.H and out.W == x.W and out.C == x.C, 'dwconv shapes')
    w = w.reshape(x.C, K * K).contiguous()
    px = x.B * x.H * x.W
    _timed(f'dwconv_kernel<{K}>', 'wc_dwconv', 2.0 * px * x.C * K * K, x.ptr, x.ldc, out.ptr, out.ldc, w.data_ptr(),
           _ptr(bias), x.B, x.H, x.W, x.C, K, _stream(), nbytes=8.0 * px * x.C)


def avgpool2x2(x: View, out: View):
    x.check()
    out.check()
    _req(out.H * 2 == x.H and out.W * 2 == x.W and out.C == x.C and out.B == x.B, 'avgpool2x2 shapes')
    _native.call('wc_avgpool2x2', x.ptr, x.ldc, out.ptr, out.ldc, x.B, x.H, x.W, x.C, _stream())


def upsample2x_bilinear(x: View, out: View):
    x.check()
    out.check()
    _req(out.H == 2 * x.H and out.W == 2 * x.W and out.C == x.C and out.B == x.B, 'upsample2x shapes')
    _native.call('wc_upsample2x_bilinear', x.ptr, x.ldc, out.ptr, out.ldc, x.B, x.H, x.W, x.C, _stream())


def layernorm_channels(x: View, gamma: torch.Tensor, beta: torch.Tensor, out: View, eps: float = 1e-5):
    x.check()
    out.check()
    _req(out.C == x.C and out.B * out.H * out.W == x.B * x.H * x.W, 'layernorm shapes')
    _req(x.ldc == x.C or x.H * x.W > 0, 'layernorm view')
    _native.call('wc_layernorm_channels', x.ptr, x.ldc, gamma.data_ptr(), beta.data_ptr(), eps, out.ptr, out.ldc,
                 x.B * x.H * x.W, x.C, _stream())


def noise_embed(noise: torch.Tensor, ang: torch.Tensor, out: View):
    out.check()
    K = ang.numel()
    _req(out.C == 2 * K and noise.numel() == out.B and noise.is_contiguous() and ang.is_contiguous(),
         'noise_embed shapes')
    _native.call('wc_noise_embed', noise.data_ptr(), ang.data_ptr(), K, out.ptr, out.ldc, out.B, out.H * out.W,
                 _stream())


# ---- UNet backward (csrc/wc_backward.hip, csrc/wc_attention_bwd.hip) ----

def _fill_seg(cs, s: Seg, B: int):
    v = s.view
    v.check()
    _req(v.B == B, 'segment batch mismatch')
    _req(len(s.taps) <= _native.MAX_TAPS, 'too many taps')
    cs.src, cs.C, cs.ldc, cs.H, cs.W = v.ptr, v.C, v.ldc, v.H, v.W
    cs.sy = cs.sx = s.stride
    cs.ntaps = len(s.taps)
    for j, (dy, dx) in enumerate(s.taps):
        cs.dy[j], cs.dx[j] = dy, dx
    if s.scale is not None:
        _req(s.scale.shape == (B, v.C) and s.shift.shape == (B, v.C), 'GN affine shape')
        cs.scale, cs.shift = s.scale.data_ptr(), s.shift.data_ptr()
    cs.silu = int(s.silu)
    cs.kbase = s.kbase


def absmax_images(v: View) -> torch.Tensor:
    """float32[B]: max |x| over each image of the view (wc_absmax_images)."""
    v.check()
    _req(v.C % 4 == 0 and v.ldc % 4 == 0 and v.ptr % 16 == 0, 'absmax view: C % 4, 16-byte aligned')
    out = torch.zeros((v.B, ), dtype=torch.float32, device=v.t.device)
    _timed('absmax_images_kernel', 'wc_absmax_images', 0.0, v.ptr, v.ldc, v.B, v.H * v.W, v.C, out.data_ptr(), _stream())
    return out


def dgrad_f16x3_enabled() -> bool:
    """Training data gradients on f16x3 under per-image absmax bounds; WC_DGRAD_F16X3=0 keeps bf16x6."""
    return os.environ.get('WC_DGRAD_F16X3', '1') != '0'


def wgrad3_enabled() -> bool:
    """The halo-tiled 3x3 weight gradient (wc_conv_wgrad3); WC_WGRAD3=0 keeps the generic GEMM (A/B)."""
    return os.environ.get('WC_WGRAD3', '1') != '0'


def wgrad3_ok(g: View, s0: Seg) -> bool:
    """Shapes wc_conv_wgrad3 takes: segment 0 a 3x3 stride-1 grid at the gradient's own grid, M % 64,
    C0 % 32 (% 64 when M % 128 != 0), W % 16, H % 8 (H % 2 for the 64-channel tiles)."""
    v = s0.view
    if list(s0.taps) != TAPS3 or s0.stride != 1 or v.H != g.H or v.W != g.W or g.C % 64 or g.W % 16:
        return False
    wide = g.C % 128 == 0
    return v.C % (32 if wide else 64) == 0 and g.H % (8 if wide else 2) == 0 and v.ldc % 4 == 0 and g.ldc % 4 == 0 \
        and v.ptr % 16 == 0 and g.ptr % 16 == 0


class F3Bounds(NamedTuple):
    """Range bounds for an f16x3 weight gradient: g = per-image max |gradient| (device float32 [B]);
    segment 0 at the static exponent x_exp0 (a GroupNorm-bounded operand: |x| 2^x_exp0 <= 2^14) or,
    raw, under x0 = its per-image max |x|; segment 1 (raw) under x1."""
    g: torch.Tensor
    x_exp0: int = 60
    x0: Optional[torch.Tensor] = None
    x1: Optional[torch.Tensor] = None


def _bound_ok(t: torch.Tensor, B: int) -> bool:
    return t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() >= B


def wgrad_f16x3_enabled() -> bool:
    """The generic weight gradient on f16x3 when the caller supplies bounds (WC_WGRAD_F16X3=0: bf16x6)."""
    return os.environ.get('WC_WGRAD_F16X3', '1') != '0'


def wgrad3_f16x3_enabled() -> bool:
    """The halo 3x3 weight gradient on f16x3 when the caller supplies the bounds (WC_WGRAD3_F16X3=0:
    bf16x6, for A/B)."""
    return os.environ.get('WC_WGRAD3_F16X3', '1') != '0'


def conv_wgrad(g: View, segs: Sequence[Seg], dw0: torch.Tensor, s0: Tuple[int, int, int], *, Cw: Optional[int] = None,
               dw1: Optional[torch.Tensor] = None, s1: int = 0, accumulate: bool = False, x6: bool = False,
               f3: Optional[F3Bounds] = None):
    """Weight gradient of a conv whose input segments are `segs` (as the forward read them, prologue
    included) and whose output gradient is the view g (pixel grid = g's H x W): GEMM over the pixels
    on fp32 MFMA (or bf16x6 with x6), split and reduced in a fixed order.  Column (tap t, channel c < Cw) of segment 0 is
    written to dw0.flat[m*s0[0] + c*s0[1] + t*s0[2]], segment 1's columns to dw1.flat[m*s1 + c].
    f3: the f16x3 range bounds (F3Bounds); with x6, the 3x3 halo kernel (segment 0 GroupNorm-bounded)
    and the generic GEMM then run f16x3."""
    g.check()
    _req(1 <= len(segs) <= 2, 'wgrad takes 1 or 2 segments')
    _req(dw0.is_cuda and dw0.dtype == torch.float32 and dw0.is_contiguous(), 'dw0: contiguous fp32 device tensor')
    a = _native.WgradArgs()
    B = g.B
    for i, s in enumerate(segs):
        _fill_seg(a.seg[i], s, B)
    a.nseg = len(segs)
    a.g, a.M, a.ldg = g.ptr, g.C, g.ldc
    a.B, a.Hm, a.Wm = B, g.H, g.W
    C0, T = segs[0].view.C, len(segs[0].taps)
    K0 = T * C0
    C1 = segs[1].view.C if len(segs) == 2 else 0
    Kc = K0 + C1
    Cw = C0 if Cw is None else Cw
    # the reduce kernel's writes must stay inside the destination tensors
    _req((g.C - 1) * s0[0] + (Cw - 1) * s0[1] + (T - 1) * s0[2] < dw0.numel(), 'dw0 too small for its strides')
    if C1:
        _req(dw1 is not None and dw1.is_cuda and dw1.is_contiguous() and (g.C - 1) * s1 + C1 <= dw1.numel(),
             'dw1: the residual segment gradient')
    lib = _native.load()
    if x6 and wgrad3_ok(g, segs[0]) and wgrad3_enabled():
        # 3x3 segment on the halo-tiled kernel; the residual 1x1 segment (if any) as its own GEMM
        P = B * g.H * g.W
        splits = lib.wc_conv_wgrad3_splits(g.C, C0, B, g.H, g.W, 512)
        a.nseg = 1
        part = torch.empty(splits * g.C * K0, dtype=torch.float32, device=g.t.device)
        s = _stream()
        if f3 is not None and segs[0].scale is not None and f3.x0 is None and wgrad3_f16x3_enabled():
            _req(_bound_ok(f3.g, B), 'f3 bound: float32 [B] on the device')
            _timed('conv_wgrad3_kernel', 'wc_conv_wgrad3_f16x3', 2.0 * P * g.C * K0, ctypes.byref(a), part.data_ptr(),
                   splits, int(f3.x_exp0), f3.g.data_ptr(), s)
        else:
            _timed('conv_wgrad3_kernel', 'wc_conv_wgrad3', 2.0 * P * g.C * K0, ctypes.byref(a), part.data_ptr(), splits,
                   s)
        _native.call('wc_wgrad_reduce', part.data_ptr(), splits, g.C, K0, K0, C0, Cw, dw0.data_ptr(), s0[0], s0[1],
                     s0[2], None, 0, int(accumulate), s)
        if C1:
            r = segs[1]
            f31 = F3Bounds(f3.g, 60, f3.x1) if f3 is not None and f3.x1 is not None else None
            conv_wgrad(g, [Seg(r.view, r.taps, r.stride)], dw1, (s1, 1, 0), accumulate=accumulate, x6=x6, f3=f31)
        return
    P = B * g.H * g.W
    splits = lib.wc_conv_wgrad_splits(g.C, Kc, P, 2048)
    part = torch.empty(splits * g.C * Kc, dtype=torch.float32, device=g.t.device)
    s = _stream()
    if (x6 and f3 is not None and wgrad_f16x3_enabled() and (C1 == 0 or f3.x1 is not None)
            and (f3.x0 is not None or f3.x_exp0 < 60)):
        for t_ in (f3.g, f3.x0, f3.x1):
            _req(t_ is None or _bound_ok(t_, B), 'f3 bounds: float32 [B] on the device')
        _timed('conv_wgrad_kernel', 'wc_conv_wgrad_f16x3', 2.0 * P * g.C * Kc, ctypes.byref(a), part.data_ptr(), splits,
               f3.g.data_ptr(), int(f3.x_exp0), _ptr(f3.x0), _ptr(f3.x1), s)
    else:
        _timed('conv_wgrad_kernel' + ('<x6>' if x6 else ''), 'wc_conv_wgrad_x6' if x6 else 'wc_conv_wgrad',
               2.0 * P * g.C * Kc, ctypes.byref(a), part.data_ptr(), splits, s)
    _native.call('wc_wgrad_reduce', part.data_ptr(), splits, g.C, Kc, K0, C0, Cw, dw0.data_ptr(), s0[0], s0[1], s0[2],
                 _ptr(dw1), s1, int(accumulate), s)


def gn_stats_pair(v: View, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5, groups: int = 8,
                  bound: bool = False, part: Optional[GnPart] = None):
    """GroupNorm statistics of v once, finalized twice: (scale, shift) of the affine GN and
    (sc0, sh0) = (rstd, -mean*rstd) of the plain normalisation (what the backward needs); with
    bound=True a fifth result, the per-image bound of |v| (wc_gn_finalize_bound).  With `part` (tile
    partials of v's tensor written by v's producer's epilogue) no pass over v: two wc_gn_finalize_part."""
    v.check()
    B, HW, C = v.B, v.H * v.W, v.C
    if part is not None:
        aff = gn_affine(v, gamma, beta, eps, groups, bound=bound, part=part)
        plain = gn_affine(v, None, None, eps, groups, part=part)
        return (aff[0], aff[1], plain[0], plain[1]) + ((aff[2], ) if bound else ())
    lib = _native.load()
    splits = lib.wc_gn_num_splits(B, HW, C)
    part = torch.empty((B, splits, groups, 2), dtype=torch.float32, device=v.t.device)
    s = _stream()
    _native.call('wc_gn_stats', v.ptr, B, HW, C, v.ldc, groups, part.data_ptr(), s)
    out = [torch.empty((B, C), dtype=torch.float32, device=v.t.device) for _ in range(4)]
    if bound:
        bnd = torch.empty((B, ), dtype=torch.float32, device=v.t.device)
        _native.call('wc_gn_finalize_bound', part.data_ptr(), B, HW, C, groups, _ptr(gamma), _ptr(beta), eps,
                     out[0].data_ptr(), out[1].data_ptr(), bnd.data_ptr(), s)
    else:
        _native.call('wc_gn_finalize', part.data_ptr(), B, HW, C, groups, _ptr(gamma), _ptr(beta), eps,
                     out[0].data_ptr(), out[1].data_ptr(), s)
    _native.call('wc_gn_finalize', part.data_ptr(), B, HW, C, groups, None, None, eps, out[2].data_ptr(),
                 out[3].data_ptr(), s)
    return tuple(out) + ((bnd, ) if bound else ())


def channel_sums(g: View) -> torch.Tensor:
    """Per-(b, c) sums over pixels of view g -> float32 [B][C][2] (second entry 0), fixed order."""
    g.check()
    B, HW, C = g.B, g.H * g.W, g.C
    lib = _native.load()
    splits = lib.wc_gn_bwd_splits(B, HW)
    part = torch.empty(B * splits * C * 2, dtype=torch.float32, device=g.t.device)
    sums = torch.empty((B, C, 2), dtype=torch.float32, device=g.t.device)
    s = _stream()
    _native.call('wc_gn_bwd_reduce', g.ptr, g.ldc, None, 0, None, None, None, None, 0, B, HW, C, splits,
                 part.data_ptr(), None, s)
    _native.call('wc_gn_bwd_finalize', part.data_ptr(), B, splits, C, 0, HW, None, None, sums.data_ptr(), None, None,
                 None, s)
    return sums


# WC_ATTN_BWD192_FP32=1 (read once): the d = 192 dK / dV on the fp32-MFMA kernel; the C side follows the
# dqkv_absmax argument alone (NULL selects the fp32 kernel), so the two sides cannot disagree
_ATTN_BWD192_FP32 = os.environ.get('WC_ATTN_BWD192_FP32', '0') == '1'

# The bsum deferral queue is per thread: autograd runs each device's backward on its own worker thread
# (as _native's library selector), so two engines' backwards never share one queue.
_BSUM = threading.local()


def bsum(sums: torch.Tensor, idx: int, out: torch.Tensor, accumulate: bool = False, now: bool = False):
    """out[c] (+)= sum_b sums[b][c][idx] (fixed order).  Between bsum_defer() and bsum_flush() the sum is
    queued and all queued sums go out in one launch (wc_bsum_batch) at the flush, each output's in
    queue order (the same values as one launch each); now=True launches at once regardless (an output
    the caller reads before the flush)."""
    B, C, _ = sums.shape
    _req(out.is_cuda and out.is_contiguous() and out.numel() == C, 'bsum output')
    queue = getattr(_BSUM, 'queue', None)
    if queue is not None and not now:
        _req(not queue or queue[0][0].shape[0] == B, 'deferred bsums of one batch size')
        queue.append((sums, idx, out, accumulate))
        return
    _native.call('wc_bsum', sums.data_ptr(), B, C, idx, out.data_ptr(), int(accumulate), _stream())


def bsum_defer():
    """Queue every bsum until bsum_flush() (the training backward: ~200 small sums -> one launch)."""
    _req(getattr(_BSUM, 'queue', None) is None, 'bsum_defer: already deferring (this thread)')
    _BSUM.queue = []


def bsum_flush():
    """Launch the queued bsums (wc_bsum_batch): an output's k-th queued sum goes in launch k, so every
    output accumulates in queue order; ends the deferral."""
    q, _BSUM.queue = getattr(_BSUM, 'queue', None), None
    if not q:
        return
    launches: List[list] = []
    seen: Dict[int, int] = {}
    for sums, idx, out, acc in q:
        k = seen.get(out.data_ptr(), -1) + 1
        seen[out.data_ptr()] = k
        if k == len(launches):
            launches.append([])
        launches[k].append((sums, idx, out, acc))
    B = q[0][0].shape[0]
    s = _stream()
    for jobs in launches:
        tab = torch.empty((len(jobs), 4), dtype=torch.int64, pin_memory=True)
        rows = [[sm.data_ptr(), o.data_ptr(), sm.shape[1] | (idx << 32), int(acc)] for sm, idx, o, acc in jobs]
        tab.copy_(torch.tensor(rows, dtype=torch.int64))
        dtab = tab.to(q[0][2].device, non_blocking=True)
        _native.call('wc_bsum_batch', dtab.data_ptr(), len(jobs), B, max(sm.shape[1] for sm, _, _, _ in jobs), s)


def gn_backward(dz: View, x: View, sc0: torch.Tensor, sh0: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                silu: bool, dx: View, *, dgamma: Optional[torch.Tensor] = None, dbeta: Optional[torch.Tensor] = None,
                accumulate: bool = True, groups: int = 8, absmax: Optional[torch.Tensor] = None,
                dx_sums: bool = False, pre: Optional[GnbSums] = None) -> Optional[torch.Tensor]:
    """Backward of SiLU(GroupNorm(x)) (silu) or GroupNorm(x): dx (+)= d/dx given dz = d/d output;
    dgamma / dbeta (+)= their gradients.  absmax: optional float32[B] raised to the max |dx| written
    per image.  dx_sums (accumulate off): also return float32 [B][C][2] whose [..., 0] is each image's
    per-channel sum of dx (channel_sums(dx)'s layout, from the reduce's sums in closed form instead of
    a pass over dx).  pre: the sums of dz already formed by the epilogue of the conv that wrote it
    (GnbSums for this x, sc0, sh0, gamma, beta, silu; part3 present when dx_sums): no reduce pass."""
    for v in (dz, x, dx):
        v.check()
    B, HW, C = x.B, x.H * x.W, x.C
    _req(dz.C == C and dx.C == C and dz.B == B and dx.B == B, 'GN backward view shapes')
    _req(not (dx_sums and accumulate), 'dx_sums needs accumulate=False (the sums are of the written values)')
    lib = _native.load()
    dev = x.t.device
    dsum = torch.empty((B, C, 2), dtype=torch.float32, device=dev) if dx_sums else None
    sums = torch.empty((B, C, 2), dtype=torch.float32, device=dev)
    coef = torch.empty((B, C, 4), dtype=torch.float32, device=dev)
    s = _stream()
    if pre is not None:
        _req(pre.x.ptr == x.ptr and pre.x.C == C and pre.silu == bool(silu) and pre.sc0 is sc0 and pre.sh0 is sh0
             and (pre.part3 is not None or not dx_sums), 'GN backward: sums formed for another GroupNorm')
        splits, part, part3 = pre.splits, pre.part, (pre.part3 if dx_sums else None)
    else:
        splits = lib.wc_gn_bwd_splits(B, HW)
        part = torch.empty(B * splits * C * 2, dtype=torch.float32, device=dev)
        part3 = torch.empty(B * splits * C, dtype=torch.float32, device=dev) if dx_sums else None
        _timed('gnb_reduce_kernel', 'wc_gn_bwd_reduce', 8.0 * B * HW * C, dz.ptr, dz.ldc, x.ptr, x.ldc,
               sc0.data_ptr(), sh0.data_ptr(), _ptr(gamma), _ptr(beta), int(silu), B, HW, C, splits, part.data_ptr(),
               _ptr(part3), s)
    _native.call('wc_gn_bwd_finalize', part.data_ptr(), B, splits, C, groups, HW, sc0.data_ptr(), _ptr(gamma),
                 sums.data_ptr(), coef.data_ptr(), _ptr(part3), _ptr(dsum), s)
    if dbeta is not None:
        bsum(sums, 0, dbeta, accumulate=True)
    if dgamma is not None:
        bsum(sums, 1, dgamma, accumulate=True)
    _timed('gnb_apply_kernel', 'wc_gn_bwd_apply', 16.0 * B * HW * C, dz.ptr, dz.ldc, x.ptr, x.ldc, sc0.data_ptr(),
           sh0.data_ptr(), _ptr(gamma), _ptr(beta), int(silu), coef.data_ptr(), B, HW, C, dx.ptr, dx.ldc,
           int(accumulate), _ptr(absmax), s)
    return dsum


def attention_fwd_lse(qkv: torch.Tensor, out: torch.Tensor, lse: torch.Tensor, B: int, N: int, C: int, heads: int,
                      precision: str = 'fp32', exps: Optional[Tuple[int, int, int]] = None):
    """Attention that also writes lse[b][h][q] (log2 domain) for the backward: fp32 MFMA
    (wc_attention_fwd_lse), or, for head dims % 32 == 0, the sampler's split-precision kernel
    ('f16x3' with the (q, k, v) exponents of attention_exps_from_norms: wc_attention_fwd_f16x3_lse;
    'bf16x6': wc_attention_fwd_x6_lse)."""
    _req(qkv.shape == (B * N, 3 * C) and qkv.is_contiguous() and out.shape == (B * N, C) and out.is_contiguous(),
         'attention shapes')
    _req(lse.is_contiguous() and lse.dtype == torch.float32 and lse.numel() == B * heads * N, 'lse: B*heads*N floats')
    _req(precision in CONV_PRECISIONS, f'attention precision {precision!r}')
    d = C // heads
    flops = 4.0 * B * N * N * C
    if precision != 'fp32' and d % 32 == 0:
        args = (qkv.data_ptr(), 3 * C, out.data_ptr(), C, lse.data_ptr(), B, N, C, heads, float(d)**-0.5)
        if precision == 'f16x3':
            _req(exps is not None, 'f16x3 attention needs (q, k, v) exponents')
            _timed(f'attention_x6_kernel<{d}, true, false, false>', 'wc_attention_fwd_f16x3_lse', flops, *args,
                   *[int(e) for e in exps], _stream())
        else:
            _timed(f'attention_x6_kernel<{d}, false, false, false>', 'wc_attention_fwd_x6_lse', flops, *args, _stream())
        return
    _timed(f'attention_kernel<{d}> (lse)', 'wc_attention_fwd_lse', flops, qkv.data_ptr(), 3 * C,
           out.data_ptr(), C, lse.data_ptr(), B, N, C, heads, float(d**-0.5), _stream())


def attention_bwd6_enabled() -> bool:
    """The bf16x6 attention backward (wc_attention_bwd6); WC_ATTN_BWD6=0 keeps fp32 MFMA (A/B)."""
    return os.environ.get('WC_ATTN_BWD6', '1') != '0'


def attention_bwd_f16x3_enabled() -> bool:
    """The f16x3 attention backward when the caller supplies the bounds (WC_ATTN_BWD_F16X3=0: bf16x6, A/B)."""
    return os.environ.get('WC_ATTN_BWD_F16X3', '1') != '0'


def attention_bwd(qkv: torch.Tensor, out: torch.Tensor, dout: torch.Tensor, lse: torch.Tensor, dqkv: torch.Tensor,
                  B: int, N: int, C: int, heads: int, precision: str = 'fp32', exps: Optional[Tuple[int, int, int]] = None,
                  dout_bound: Optional[torch.Tensor] = None, dqkv_absmax: Optional[torch.Tensor] = None) -> bool:
    """d qkv (same [q | k | v] rows as qkv) of softmax(Q K^T / sqrt(d)) V from the forward's output and lse:
    fp32 MFMA (wc_attention_bwd), or with precision 'bf16x6' / 'f16x3' and a head dim in {32, 64, 128}
    (f16x3 also 192) the split-precision kernels: f16x3 (wc_attention_bwd_f16x3) when the Q / K / V exponents of the
    forward (exps) and the per-image max |dout| (dout_bound, device float32 [B]) are given, else
    bf16x6 (wc_attention_bwd6).  dqkv_absmax: float32 [B] raised to the max |dqkv| written per image
    by the f16x3 kernels; returns whether it was (else the caller measures the bound itself)."""
    for t_, w in ((qkv, 3 * C), (out, C), (dout, C), (dqkv, 3 * C)):
        _req(t_.is_cuda and t_.dtype == torch.float32 and t_.is_contiguous() and t_.numel() == B * N * w,
             'attention backward operands')
    d = C // heads
    dv = torch.empty(B * heads * N, dtype=torch.float32, device=qkv.device)
    args = (qkv.data_ptr(), 3 * C, out.data_ptr(), C, dout.data_ptr(), C, lse.data_ptr(), dv.data_ptr(),
            dqkv.data_ptr(), 3 * C, B, N, C, heads, float(d**-0.5))
    f3ok = precision == 'f16x3' and exps is not None and dout_bound is not None and attention_bwd_f16x3_enabled()
    if d == 192 and f3ok and attention_bwd6_enabled():
        # dQ on f16x3 with the output dims in three parts; dK / dV on f16x3 with the V rows in LDS (or, with
        # WC_ATTN_BWD192_FP32=1, on fp32 MFMA, which raises no bound)
        _req(_bound_ok(dout_bound, B), 'dout_bound: float32 [B] on the device')
        amx = dqkv_absmax if not _ATTN_BWD192_FP32 else None
        if amx is not None:
            _req(_bound_ok(amx, B), 'dqkv_absmax: float32 [B] on the device')
        _timed(f'attention_bwd<{d}>', 'wc_attention_bwd_f16x3', 10.0 * B * N * N * C, *args, int(exps[0]),
               int(exps[1]), int(exps[2]), dout_bound.data_ptr(), _ptr(amx), _stream())
        return amx is not None
    if precision != 'fp32' and d in (32, 64, 128) and attention_bwd6_enabled():
        if f3ok:
            _req(dout_bound.is_cuda and dout_bound.dtype == torch.float32 and dout_bound.numel() >= B,
                 'dout_bound: float32 [B] on the device')
            if dqkv_absmax is not None:
                _req(_bound_ok(dqkv_absmax, B), 'dqkv_absmax: float32 [B] on the device')
            _timed(f'attention_bwd<{d}>', 'wc_attention_bwd_f16x3', 10.0 * B * N * N * C, *args, int(exps[0]),
                   int(exps[1]), int(exps[2]), dout_bound.data_ptr(), _ptr(dqkv_absmax), _stream())
            return dqkv_absmax is not None
        _timed(f'attention_bwd<{d}>', 'wc_attention_bwd6', 10.0 * B * N * N * C, *args, _stream())
        return False
    _timed(f'attention_bwd<{d}>', 'wc_attention_bwd', 10.0 * B * N * N * C, *args, _stream())
    return False


def gemm_small(M: int, N: int, K: int, A: torch.Tensor, sa: Tuple[int, int], Bm: torch.Tensor, sb: Tuple[int, int],
               Cm: torch.Tensor, ldc: int, alpha: float = 1.0, beta: float = 0.0, offs: Tuple[int, int, int] = (0, 0, 0)):
    """C[m][n] = alpha*sum_k A[m*sa0 + k*sa1] B[k*sb0 + n*sb1] + beta*C (small matrices; element offsets offs)."""
    for t_ in (A, Bm, Cm):
        _req(t_.is_cuda and t_.dtype == torch.float32 and t_.is_contiguous(), 'gemm_small operands')
    _native.call('wc_gemm_small', M, N, K, A.data_ptr() + 4 * offs[0], sa[0], sa[1], Bm.data_ptr() + 4 * offs[1], sb[0],
                 sb[1], Cm.data_ptr() + 4 * offs[2], ldc, alpha, beta, _stream())


def silu_map(y: torch.Tensor, dz: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(y), or dz * silu'(y) when dz is given."""
    _req(y.is_cuda and y.dtype == torch.float32 and y.is_contiguous(), 'silu operand')
    out = torch.empty_like(y)
    if dz is not None:
        _req(dz.shape == y.shape and dz.is_contiguous(), 'silu gradient operand')
    _native.call('wc_silu', y.data_ptr(), _ptr(dz), out.data_ptr(), y.numel(), 0 if dz is None else 1, _stream())
    return out


def colsum(X: torch.Tensor, out: torch.Tensor, accumulate: bool = False, col0: int = 0, ncol: Optional[int] = None):
    """out[n] (+)= sum_r X[r][col0 + n] over a 2-D contiguous X."""
    R, Ntot = X.shape
    n = Ntot - col0 if ncol is None else ncol
    _req(out.is_contiguous() and out.numel() == n, 'colsum output')
    _native.call('wc_colsum', X.data_ptr() + 4 * col0, R, n, Ntot, out.data_ptr(), int(accumulate), _stream())


def time_embedding(t: torch.Tensor, D: int) -> torch.Tensor:
    tt = t.reshape(-1).to(torch.int64).contiguous()
    out = torch.empty((tt.numel(), D), dtype=torch.float32, device=tt.device)
    _native.call('wc_time_embedding', tt.data_ptr(), tt.numel(), D, out.data_ptr(), _stream())
    return out


def nchw_to_nhwc(x: torch.Tensor, ldc: int) -> torch.Tensor:
    """(B, C, H, W) -> (B, H, W, ldc) with zero channels C..ldc-1."""
    _req(x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 4, 'NCHW fp32 device tensor')
    B, C, H, W = x.shape
    out = torch.empty((B, H, W, ldc), dtype=torch.float32, device=x.device)
    _native.call('wc_nchw_to_nhwc', x.data_ptr(), B, C, H, W, out.data_ptr(), ldc, _stream())
    return out
