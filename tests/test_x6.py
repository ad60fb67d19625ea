"""bf16x6 split-precision kernels: the 3x3 halo conv (csrc/wc_conv6.hip), the implicit-GEMM conv
(csrc/wc_igemm6.hip) and flash attention (csrc/wc_attention6.hip).

CPU: the 3-piece bf16 split is exact, and the weight re-pack has the layout the kernel reads.
GPU: the conv against a float64 PyTorch reference of the same op.  Stated tolerance: relative L2
<= 1e-5 (the fp32 tolerance of SURVEY.md §8c) and, tighter, within 4x (+1e-7) of the error of the
fp32-MFMA conv on the same inputs, i.e. fp32-class accuracy.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]


def _bits_to_f32(p16: torch.Tensor) -> torch.Tensor:
    return (p16.to(torch.int32) << 16).view(torch.float32)


def test_split3_exact():
    from weatherconverter_amd.kernels import split3_bits
    g = torch.Generator().manual_seed(0)
    x = torch.cat([torch.randn(100000, generator=g) * 10.0**e for e in range(-6, 7)])
    x = torch.cat([x, torch.tensor([0.0, -0.0, 1.0, -1.0, 3.0e38, -1.17549435e-38, 1 / 3])])
    p = split3_bits(x)
    f = _bits_to_f32(p)
    # exact: sum of the pieces in float64 reproduces x, and each piece is a bf16 value
    assert torch.equal(f.double().sum(0), x.double())
    assert torch.equal(f, _bits_to_f32((f.view(torch.int32) >> 16).to(torch.int16)))
    # pieces shrink by >= 2^8: |p1| < 2^-7 |x|, |p2| < 2^-15 |x|
    ax = x.abs().double()
    assert bool((f[1].abs().double() <= ax * 2.0**-7).all()) and bool((f[2].abs().double() <= ax * 2.0**-15).all())


@pytest.mark.parametrize('N,C0,C1', [(128, 64, 32), (64, 32, 0), (96, 48, 16), (256, 16, 64)])
def test_pack_x6_layout(N, C0, C1):
    """Unpack [tile][step][piece][half][BN][8] back to [N][9*C0 + C1] and compare exactly."""
    from weatherconverter_amd.kernels import pack_x6
    g = torch.Generator().manual_seed(1)
    w = torch.randn((N, 9 * C0 + C1), generator=g)
    x6 = pack_x6(w, C0, C1)
    BN = x6.BN
    assert BN == (64 if N <= 64 else 128)
    T, S = x6.data.shape[0], x6.data.shape[1]
    assert x6.data.shape == (T, S, 3, 2, BN, 8) and S == 9 * (C0 // 16) + C1 // 16
    v = _bits_to_f32(x6.data).double().sum(2)  # (T, S, 2, BN, 8): sum of the pieces
    v = v.permute(0, 3, 1, 2, 4).reshape(T * BN, S, 16)[:N]  # (n, step, k16)
    s0 = v[:, :9 * (C0 // 16)].reshape(N, C0 // 16, 9, 16).permute(0, 2, 1, 3).reshape(N, 9 * C0)
    s1 = v[:, 9 * (C0 // 16):].reshape(N, C1)
    assert torch.equal(torch.cat([s0, s1], 1), w.double())
    if N % BN:
        assert not _bits_to_f32(x6.data).view(T, S, 3, 2, BN, 8)[-1, :, :, :, N % BN:].any()


# ---------------------------------------------------------------------------------------------- GPU


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def _pack(w):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


CASES = [
    # B, H, W, Ci, Co, Cr (1x1 residual channels), prologue, act
    (2, 16, 32, 64, 128, 32, 'silu', 0),
    (1, 32, 32, 128, 64, 0, 'silu', 0),
    (2, 8, 16, 96, 256, 64, 'affine', 0),
    (1, 16, 16, 32, 96, 0, 'raw', 0),
    (1, 16, 48, 64, 80, 0, 'raw', 1),  # activations: raw segment 0 (as wc_conv_igemm requires)
    (2, 32, 16, 256, 128, 128, 'silu', 0),
]


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Ci,Co,Cr,pro,act', CASES)
def test_conv3x3_x6_vs_float64(B, H, W, Ci, Co, Cr, pro, act):
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(7)
    h = torch.randn((B, Ci, H, W), generator=g) * 1.5 + 0.3
    x2 = torch.randn((B, max(Cr, 16), H, W), generator=g)
    w = torch.randn((Co, Ci, 3, 3), generator=g) / (Ci * 9)**0.5
    wr = torch.randn((Co, max(Cr, 16), 1, 1), generator=g) / max(Cr, 16)**0.5
    b = torch.randn(Co, generator=g) * 0.1
    temb = torch.randn((B, Co), generator=g)
    sc = 1 + 0.2 * torch.randn((B, Ci), generator=g)
    sh = 0.2 * torch.randn((B, Ci), generator=g)
    resv = torch.randn((B, H, W, Co), generator=g)

    a = h.double()
    if pro != 'raw':
        a = a * sc.double()[:, :, None, None] + sh.double()[:, :, None, None]
    if pro == 'silu':
        a = F.silu(a)
    ref = F.conv2d(a, w.double(), b.double(), padding=1) + temb.double()[:, :, None, None]
    if Cr:
        ref = ref + F.conv2d(x2.double(), wr.double())
    if act == 1:
        ref = F.gelu(ref)
    ref = ref + _nchw(resv).double()

    segs = [K.Seg(K.View.full(_nhwc(h).cuda()), TAPS3, scale=None if pro == 'raw' else sc.cuda(),
                  shift=None if pro == 'raw' else sh.cuda(), silu=pro == 'silu')]
    wp = _pack(w)
    if Cr:
        segs.append(K.Seg(K.View.full(_nhwc(x2).cuda()), [(0, 0)], kbase=9 * Ci))
        wp = torch.cat([wp, wr.reshape(Co, Cr)], 1)
    wp = wp.contiguous().cuda()
    assert K.x6_eligible(segs, Co, H, W)
    # output into a channel slice of a wider buffer (the skip-concat layout)
    outs = {}
    for mode in ('x6', 'fp32'):
        buf = torch.full((B, H, W, Co + 32), 7.0, device='cuda')
        out = K.View(buf, 16, Co)
        kw = dict(Hm=H, Wm=W, temb=temb.cuda(), temb_ld=Co, res=K.View.full(resv.cuda()), act=act)
        if mode == 'x6':
            K.conv3x3_x6(segs, K.pack_x6(wp, Ci, Cr), b.cuda(), out, **kw)
        else:
            K.conv_igemm(segs, wp, b.cuda(), out, **kw)
        torch.cuda.synchronize()
        bc = buf.cpu()
        assert bool((bc[..., :16] == 7.0).all()) and bool((bc[..., 16 + Co:] == 7.0).all())
        outs[mode] = _nchw(bc[..., 16:16 + Co])
    e6 = rel_l2(outs['x6'].double(), ref)
    e32 = rel_l2(outs['fp32'].double(), ref)
    assert e6 < 1e-5
    assert e6 <= 4 * e32 + 1e-7, (e6, e32)


@pytest.mark.gpu
def test_conv3x3_x6_rejects_untiled_shape():
    from weatherconverter_amd import kernels as K
    h = torch.randn((1, 12, 16, 32), device='cuda')
    segs = [K.Seg(K.View.full(h), TAPS3)]
    assert not K.x6_eligible(segs, 128, 12, 16)  # H % 8 != 0
    w6 = K.pack_x6(torch.randn((128, 9 * 32), device='cuda'), 32)
    out = torch.empty((1, 12, 16, 128), device='cuda')
    with pytest.raises(RuntimeError):
        K.conv3x3_x6(segs, w6, None, K.View.full(out), Hm=12, Wm=16)


# ---------------------------------------------------------------- general implicit GEMM (wc_conv_igemm_x6)

TAPS4S2 = [(ky - 1, kx - 1) for ky in range(4) for kx in range(4)]


def _run_both(K, segs, wp, C0, C1, ntaps, bias, out_fn, **kw):
    """Run wc_conv_igemm (fp32) and wc_conv_igemm_x6 on identical args; return both outputs (CPU)."""
    outs = {}
    for mode in ('x6', 'fp32'):
        out_view, out_nchw, read = out_fn()
        if mode == 'x6':
            K.conv_igemm_x6(segs, K.pack_x6(wp, C0, C1, ntaps=ntaps, order='natural'), bias, out_view,
                            out_nchw=out_nchw, **kw)
        else:
            K.conv_igemm(segs, wp, bias, out_view, out_nchw=out_nchw, **kw)
        torch.cuda.synchronize()
        outs[mode] = read()
    return outs


def _check(outs, ref):
    e6 = rel_l2(outs['x6'].double(), ref)
    e32 = rel_l2(outs['fp32'].double(), ref)
    assert e6 < 1e-5 and e6 <= 4 * e32 + 1e-7, (e6, e32)


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,C,N', [(2, 16, 16, 128, 384), (1, 32, 32, 64, 64), (3, 8, 12, 96, 160)])
def test_igemm_x6_linear_gn_prologue_residual(B, H, W, C, N):
    """Attention in_proj / out_proj shapes: (GN-affine(x)) W^T + b (+ residual view)."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(11)
    x = torch.randn((B, H, W, C), generator=g) * 3 + 1
    sc = 1 + 0.3 * torch.randn((B, C), generator=g)
    sh = 0.3 * torch.randn((B, C), generator=g)
    w = torch.randn((N, C), generator=g) / C**0.5
    b = torch.randn(N, generator=g) * 0.1
    res = torch.randn((B, H, W, N), generator=g)
    a = x.double() * sc.double()[:, None, None, :] + sh.double()[:, None, None, :]
    ref = a @ w.double().t() + b.double() + res.double()
    segs = [K.Seg(K.View.full(x.cuda()), [(0, 0)], scale=sc.cuda(), shift=sh.cuda())]
    resv = K.View.full(res.cuda())

    def out_fn():
        o = torch.empty((B, H, W, N), device='cuda')
        return K.View.full(o), None, lambda: o.cpu()
    _check(_run_both(K, segs, w.cuda(), C, 0, 1, b.cuda(), out_fn, Hm=H, Wm=W, res=resv), ref)


@pytest.mark.gpu
def test_igemm_x6_down_conv_4x4_s2():
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(12)
    B, H, Ci, Co = 2, 16, 64, 128
    x = torch.randn((B, Ci, H, H), generator=g)
    w = torch.randn((Co, Ci, 4, 4), generator=g) / (16 * Ci)**0.5
    b = torch.randn(Co, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1)
    segs = [K.Seg(K.View.full(_nhwc(x).cuda()), TAPS4S2, stride=2)]

    def out_fn():
        o = torch.empty((B, H // 2, H // 2, Co), device='cuda')
        return K.View.full(o), None, lambda: _nchw(o.cpu())
    _check(_run_both(K, segs, _pack(w).cuda(), Ci, 0, 16, b.cuda(), out_fn, Hm=H // 2, Wm=H // 2), ref)


@pytest.mark.gpu
def test_igemm_x6_conv_transpose_into_concat_slice():
    from weatherconverter_amd import kernels as K
    from weatherconverter_amd.diffusion_model.models.engine import pack_convT
    g = torch.Generator().manual_seed(13)
    B, H, Ci, Co = 2, 8, 128, 64
    x = torch.randn((B, Ci, H, H), generator=g)
    wt = torch.randn((Ci, Co, 4, 4), generator=g) / (4 * Ci)**0.5
    b = torch.randn(Co, generator=g) * 0.1
    ref = F.conv_transpose2d(x.double(), wt.double(), b.double(), stride=2, padding=1)
    xv = K.View.full(_nhwc(x).cuda())
    outs = {'x6': None, 'fp32': None}
    for mode in outs:
        buf = torch.full((B, 2 * H, 2 * H, 2 * Co), 5.0, device='cuda')
        dst = K.View(buf, 0, Co)
        for py in (0, 1):
            for px in (0, 1):
                taps, w = pack_convT(wt, py, px)
                if mode == 'x6':
                    K.conv_igemm_x6([K.Seg(xv, taps)], K.pack_x6(w.cuda(), Ci, 0, ntaps=4, order='natural'),
                                    b.cuda(), dst, Hm=H, Wm=H, out_map=(2, 2, py, px))
                else:
                    K.conv_igemm([K.Seg(xv, taps)], w.cuda(), b.cuda(), dst, Hm=H, Wm=H, out_map=(2, 2, py, px))
        torch.cuda.synchronize()
        bc = buf.cpu()
        assert bool((bc[..., Co:] == 5.0).all())
        outs[mode] = _nchw(bc[..., :Co])
    _check(outs, ref)


@pytest.mark.gpu
def test_igemm_x6_nchw_head_and_gelu():
    """The N=3 head (GN+SiLU prologue, NCHW store) and a raw 1x1 with GELU epilogue."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(14)
    B, H, C = 2, 12, 64
    h = torch.randn((B, C, H, H), generator=g)
    sc = 1 + 0.2 * torch.randn((B, C), generator=g)
    sh = 0.2 * torch.randn((B, C), generator=g)
    w = torch.randn((3, C, 3, 3), generator=g) / (9 * C)**0.5
    b = torch.randn(3, generator=g) * 0.1
    a = F.silu(h.double() * sc.double()[:, :, None, None] + sh.double()[:, :, None, None])
    ref = F.conv2d(a, w.double(), b.double(), padding=1)
    segs = [K.Seg(K.View.full(_nhwc(h).cuda()), TAPS3, scale=sc.cuda(), shift=sh.cuda(), silu=True)]

    def out_fn():
        o = torch.empty((B, 3, H, H), device='cuda')
        return None, o, lambda: o.cpu()
    _check(_run_both(K, segs, _pack(w).cuda(), C, 0, 9, b.cuda(), out_fn, Hm=H, Wm=H), ref)

    x = torch.randn((B, H, H, C), generator=g)
    w2 = torch.randn((96, C), generator=g) / C**0.5
    ref2 = F.gelu(x.double() @ w2.double().t())

    def out_fn2():
        o = torch.empty((B, H, H, 96), device='cuda')
        return K.View.full(o), None, lambda: o.cpu()
    _check(_run_both(K, [K.Seg(K.View.full(x.cuda()), [(0, 0)])], w2.cuda(), C, 0, 1, None, out_fn2, Hm=H, Wm=H,
                     act=1), ref2)


@pytest.mark.gpu
def test_igemm_x6_3x3_with_residual_segment_odd_grid():
    """ResBlock conv2 on a grid the halo kernel does not tile (9 x 20): the implicit-GEMM fallback."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(15)
    B, H, W, Ci, Co, Cr = 2, 9, 20, 64, 128, 32
    h = torch.randn((B, Ci, H, W), generator=g)
    x2 = torch.randn((B, Cr, H, W), generator=g)
    w = torch.randn((Co, Ci, 3, 3), generator=g) / (9 * Ci)**0.5
    wr = torch.randn((Co, Cr, 1, 1), generator=g) / Cr**0.5
    b = torch.randn(Co, generator=g) * 0.1
    temb = torch.randn((B, Co), generator=g)
    sc = 1 + 0.2 * torch.randn((B, Ci), generator=g)
    sh = 0.2 * torch.randn((B, Ci), generator=g)
    a = F.silu(h.double() * sc.double()[:, :, None, None] + sh.double()[:, :, None, None])
    ref = F.conv2d(a, w.double(), b.double(), padding=1) + temb.double()[:, :, None, None] + F.conv2d(
        x2.double(), wr.double())
    segs = [K.Seg(K.View.full(_nhwc(h).cuda()), TAPS3, scale=sc.cuda(), shift=sh.cuda(), silu=True),
            K.Seg(K.View.full(_nhwc(x2).cuda()), [(0, 0)], kbase=9 * Ci)]
    wp = torch.cat([_pack(w), wr.reshape(Co, Cr)], 1).contiguous().cuda()

    def out_fn():
        o = torch.empty((B, H, W, Co), device='cuda')
        return K.View.full(o), None, lambda: _nchw(o.cpu())
    _check(_run_both(K, segs, wp, Ci, Cr, 9, b.cuda(), out_fn, Hm=H, Wm=W, temb=temb.cuda(), temb_ld=Co), ref)


# ---------------------------------------------------------------- attention (wc_attention_fwd_x6)


def _attn_ref(qkv, B, N, C, heads):
    d = C // heads
    q, k, v = qkv.double().split(C, -1)
    q = q.reshape(B, N, heads, d).transpose(1, 2)
    k = k.reshape(B, N, heads, d).transpose(1, 2)
    v = v.reshape(B, N, heads, d).transpose(1, 2)
    return (torch.softmax((q * d**-0.5) @ k.transpose(-1, -2), -1) @ v).transpose(1, 2).reshape(B, N, C)


@pytest.mark.gpu
@pytest.mark.parametrize('B,N,C,heads', [(2, 100, 128, 4), (1, 1024, 256, 4), (2, 300, 512, 4), (1, 257, 768, 4),
                                         (1, 64, 384, 4), (1, 96, 640, 4)])
def test_attention_x6_vs_float64(B, N, C, heads):
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(21)
    qkv = torch.randn((B, N, 3 * C), generator=g) * 1.5
    ref = _attn_ref(qkv, B, N, C, heads)
    errs = {}
    for prec in ('bf16x6', 'fp32'):
        out = torch.full((B * N, C), 9.0, device='cuda')
        K.attention(qkv.reshape(B * N, 3 * C).cuda(), out, B, N, C, heads, prec)
        errs[prec] = rel_l2(out.cpu().double().reshape(B, N, C), ref)
    assert errs['bf16x6'] < 1e-5 and errs['bf16x6'] <= 4 * errs['fp32'] + 1e-7, errs


@pytest.mark.gpu
def test_attention_x6_spiky_scores():
    """A dominant key forces the running max to jump mid-sequence (online-softmax rescale path)."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(22)
    B, N, C, heads = 1, 512, 256, 4
    qkv = torch.randn((B, N, 3 * C), generator=g)
    qkv[0, 400, C:2 * C] *= 25.0
    ref = _attn_ref(qkv, B, N, C, heads)
    out = torch.empty((B * N, C), device='cuda')
    K.attention(qkv.reshape(B * N, 3 * C).cuda(), out, B, N, C, heads, 'bf16x6')
    assert rel_l2(out.cpu().double().reshape(B, N, C), ref) < 1e-5


# ---------------------------------------------------------------- f16x3 (wc_conv3x3_f16x3)


@pytest.mark.parametrize('N,C0,C1', [(128, 64, 32), (64, 32, 0), (96, 48, 16)])
def test_pack_f16x3_layout_and_scale(N, C0, C1):
    """Unpack the f16x3 weight: fp16 pieces (h + l) * 2^-sW reproduce the 3x3 part to 2^-22 relative,
    the bf16 residual pieces exactly; every scaled 3x3 weight is <= 2^14."""
    from weatherconverter_amd.kernels import pack_f16x3
    g = torch.Generator().manual_seed(3)
    w = torch.randn((N, 9 * C0 + C1), generator=g) * 0.05
    w3 = pack_f16x3(w, C0, C1)
    BN, T = w3.BN, w3.data.shape[0]
    S0, S1 = 9 * (C0 // 16), C1 // 16
    raw = w3.data.view(T, -1)
    main = raw[:, :S0 * 2 * 2 * BN * 8].reshape(T, S0, 2, 2, BN, 8)
    hl = main.view(torch.float16).double()
    assert hl[:, :, 0].abs().max() <= 2.0**14
    v = hl.sum(2).permute(0, 3, 1, 2, 4).reshape(T * BN, S0, 16)[:N]
    inv = w3.wsinv[:N].double()[:, None]
    s0 = v.reshape(N, C0 // 16, 9, 16).permute(0, 2, 1, 3).reshape(N, 9 * C0) * inv
    ref = w[:, :9 * C0].double()
    assert ((s0 - ref).abs() <= ref.abs() * 2.0**-21 + 2.0**-40).all()
    if C1:
        res = raw[:, S0 * 2 * 2 * BN * 8:].reshape(T, S1, 3, 2, BN, 8)
        r = _bits_to_f32(res).double().sum(2).permute(0, 3, 1, 2, 4).reshape(T * BN, S1 * 16)[:N] * inv
        assert torch.equal(r, w[:, 9 * C0:].double())


def test_f16x3_a_exp_bound():
    from weatherconverter_amd.kernels import f16x3_a_exp
    for gmax, bmax, n in [(1.0, 0.0, 524288), (3.7, 1.2, 4096), (1e-3, 0.0, 64), (200.0, 5.0, 1 << 20)]:
        e = f16x3_a_exp(gmax, bmax, n)
        bound = (n - 1)**0.5 * gmax + bmax
        assert bound * 2.0**e <= 2.0**14 < bound * 2.0**(e + 1) or e in (-60, 60)


def _gn_affine(x, gamma, beta, G=8, eps=1e-5):
    """Per-(b, c) scale/shift of GroupNorm(G) on NCHW x (float64)."""
    B, C = x.shape[:2]
    xg = x.double().reshape(B, G, -1)
    rstd = 1.0 / torch.sqrt(xg.var(-1, unbiased=False) + eps)
    mean = xg.mean(-1)
    sc = rstd.repeat_interleave(C // G, 1) * gamma.double()
    sh = beta.double() - mean.repeat_interleave(C // G, 1) * sc
    return sc, sh


F3_CASES = [
    # B, H, W, Ci, Co, Cr, silu, gamma scale, outlier
    (2, 16, 32, 64, 128, 32, True, 1.0, False),
    (1, 32, 32, 128, 64, 0, True, 1.0, False),
    (2, 8, 16, 96, 256, 64, False, 1.0, False),
    (1, 16, 16, 64, 128, 64, True, 20.0, True),  # Samuelson-extreme outlier + large gamma
]


@pytest.mark.gpu
def test_gn_finalize_bound_covers_every_element():
    """wc_gn_finalize_bound: bound[b] >= max |x[b]| (Samuelson), also for a group with one extreme outlier."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(61)
    x = torch.randn((3, 16, 16, 64), generator=g) * 4 + 2
    x[1] = 0.5
    x[1, 3, 5, ::8] = 3e3  # one huge value per group of image 1
    x[2] *= 1e-3
    _, _, bnd = K.gn_affine(K.View.full(x.cuda()), None, None, bound=True)
    bnd = bnd.cpu()
    amax = x.abs().amax((1, 2, 3))
    assert bool((bnd >= amax).all()), (bnd, amax)
    assert bool((bnd <= amax * (16 * 16 * 8)**0.5 * 1.01).all())


@pytest.mark.gpu
@pytest.mark.parametrize('bounded', [False, True])
@pytest.mark.parametrize('B,H,W,Ci,Co,Cr,silu,gs,outlier', F3_CASES)
def test_conv3x3_f16x3_vs_float64(B, H, W, Ci, Co, Cr, silu, gs, outlier, bounded):
    if bounded and not Cr:
        pytest.skip('the per-image bound only matters with a residual segment')
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(31)
    h = torch.randn((B, Ci, H, W), generator=g) * 3 + 0.7
    if outlier:  # one huge value per group: its normalized value approaches sqrt(n - 1)
        h.zero_()
        h[:, ::Ci // 8, 0, 0] = 1e4
    gamma = gs * (1 + 0.3 * torch.randn(Ci, generator=g))
    beta = 0.5 * torch.randn(Ci, generator=g)
    sc, sh = _gn_affine(h, gamma, beta)
    x2 = torch.randn((B, max(Cr, 16), H, W), generator=g) * 5
    w = torch.randn((Co, Ci, 3, 3), generator=g) / (Ci * 9)**0.5
    wr = torch.randn((Co, max(Cr, 16), 1, 1), generator=g) / max(Cr, 16)**0.5
    b = torch.randn(Co, generator=g) * 0.1
    a = h.double() * sc[:, :, None, None] + sh[:, :, None, None]
    if silu:
        a = F.silu(a)
    ref = F.conv2d(a, w.double(), b.double(), padding=1)
    if Cr:
        ref = ref + F.conv2d(x2.double(), wr.double())
    segs = [K.Seg(K.View.full(_nhwc(h).cuda()), TAPS3, scale=sc.float().cuda(), shift=sh.float().cuda(), silu=silu)]
    wp = _pack(w)
    if Cr:
        segs.append(K.Seg(K.View.full(_nhwc(x2).cuda()), [(0, 0)], kbase=9 * Ci))
        wp = torch.cat([wp, wr.reshape(Co, Cr)], 1)
    wp = wp.contiguous().cuda()
    e = K.f16x3_a_exp(float(gamma.abs().max()), float(beta.abs().max()), H * W * Ci // 8)
    xb = None
    if bounded:  # the residual input's per-image bound from its own GroupNorm statistics
        if outlier:
            x2v = segs[1].view.t
            x2v[:, 0, 0, :] = 5e3  # a large raw residual value lowers the image's scale
            x2[:, :, 0, 0] = 5e3
            ref = F.conv2d(a if not silu else F.silu(h.double() * sc[:, :, None, None] + sh[:, :, None, None]),
                           w.double(), b.double(), padding=1) + F.conv2d(x2.double(), wr.double())
        _, _, xb = K.gn_affine(segs[1].view, None, None, bound=True)
    outs = {}
    for mode in ('f16x3', 'fp32'):
        out = torch.empty((B, H, W, Co), device='cuda')
        if mode == 'f16x3':
            K.conv3x3_f16x3(segs, K.pack_f16x3(wp, Ci, Cr, res_f16=bounded), b.cuda(), K.View.full(out), Hm=H, Wm=W,
                            a_exp=e, a_bound=xb)
        else:
            K.conv_igemm(segs, wp, b.cuda(), K.View.full(out), Hm=H, Wm=W)
        torch.cuda.synchronize()
        outs[mode] = _nchw(out.cpu()).double()
    assert torch.isfinite(outs['f16x3']).all()
    e3, e32 = rel_l2(outs['f16x3'], ref), rel_l2(outs['fp32'], ref)
    assert e3 < 1e-5 and e3 <= 4 * e32 + 2e-7, (e3, e32)


@pytest.mark.gpu
@pytest.mark.parametrize('B,N,C,heads,gs', [(2, 300, 128, 4, 1.0), (1, 1024, 256, 4, 1.0), (2, 257, 512, 4, 3.0),
                                            (1, 200, 768, 4, 1.0), (1, 96, 384, 4, 1.0), (1, 64, 640, 4, 0.5)])
def test_attention_f16x3_vs_float64(B, N, C, heads, gs):
    """qkv = GN(Y) W_in^T + b_in as in the UNet, exponents from the static bound; vs float64."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(41)
    y = torch.randn((B, C, N), generator=g) * 2 + 1
    gamma = gs * (1 + 0.3 * torch.randn(C, generator=g))
    beta = 0.3 * torch.randn(C, generator=g)
    yn = F.group_norm(y.double(), 8, gamma.double(), beta.double(), 1e-5).transpose(1, 2)  # (B, N, C)
    w_in = torch.randn((3 * C, C), generator=g) / C**0.5
    b_in = 0.1 * torch.randn(3 * C, generator=g)
    qkv = (yn @ w_in.double().t() + b_in.double()).float()
    ref = _attn_ref(qkv, B, N, C, heads)
    exps = K.attention_f16x3_exps(w_in, b_in, float(gamma.abs().max()), float(beta.abs().max()), N * C // 8)
    errs = {}
    for prec in ('f16x3', 'fp32'):
        out = torch.full((B * N, C), 9.0, device='cuda')
        K.attention(qkv.reshape(B * N, 3 * C).cuda(), out, B, N, C, heads, prec, exps)
        errs[prec] = rel_l2(out.cpu().double().reshape(B, N, C), ref)
    assert errs['f16x3'] < 1e-5 and errs['f16x3'] <= 4 * errs['fp32'] + 2e-7, (errs, exps)


def test_pack_f16x3_natural_order():
    from weatherconverter_amd.kernels import pack_f16x3
    g = torch.Generator().manual_seed(4)
    N, C0, nt = 96, 32, 16
    w = torch.randn((N, nt * C0), generator=g) * 0.05
    w3 = pack_f16x3(w, C0, ntaps=nt, order='natural')
    T, BN = w3.data.shape[0], w3.BN
    S0 = nt * C0 // 16
    hl = w3.data.view(T, S0, 2, 2, BN, 8).view(torch.float16).double().sum(2)
    v = hl.permute(0, 3, 1, 2, 4).reshape(T * BN, S0 * 16)[:N] * w3.wsinv[:N].double()[:, None]
    assert ((v - w.double()).abs() <= w.double().abs() * 2.0**-21 + 2.0**-40).all()


@pytest.mark.gpu
def test_igemm_f16x3_projections_and_head():
    """in_proj (GN-affine prologue, Samuelson bound), out_proj-style raw input with an explicit bound
    and residual, and the N=3 head (GN+SiLU, NCHW store) vs float64."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(51)
    B, H, C, N = 2, 16, 128, 384
    x = torch.randn((B, C, H, H), generator=g) * 2 + 1
    gamma = 1 + 0.3 * torch.randn(C, generator=g)
    beta = 0.3 * torch.randn(C, generator=g)
    sc, sh = _gn_affine(x, gamma, beta)
    w = torch.randn((N, C), generator=g) / C**0.5
    b = 0.1 * torch.randn(N, generator=g)
    a = x.double() * sc[:, :, None, None] + sh[:, :, None, None]
    ref = torch.einsum('bchw,nc->bhwn', a, w.double()) + b.double()
    e = K.f16x3_a_exp(float(gamma.abs().max()), float(beta.abs().max()), H * H * C // 8)
    out = torch.empty((B, H, H, N), device='cuda')
    seg = [K.Seg(K.View.full(_nhwc(x).cuda()), [(0, 0)], scale=sc.float().cuda(), shift=sh.float().cuda())]
    K.conv_igemm_f16x3(seg, K.pack_f16x3(w.cuda(), C, ntaps=1, order='natural'), b.cuda(), K.View.full(out),
                       Hm=H, Wm=H, a_exp=e)
    assert rel_l2(out.cpu().double(), ref) < 2e-6

    # raw input bounded by 7 (as |O| <= max|V|) + residual view
    o = (torch.rand((B, H, H, C), generator=g) * 14 - 7)
    res = torch.randn((B, H, H, C), generator=g)
    w2 = torch.randn((C, C), generator=g) / C**0.5
    ref2 = o.double() @ w2.double().t() + res.double()
    out2 = torch.empty((B, H, H, C), device='cuda')
    K.conv_igemm_f16x3([K.Seg(K.View.full(o.cuda()), [(0, 0)])], K.pack_f16x3(w2.cuda(), C, ntaps=1, order='natural'),
                       None, K.View.full(out2), Hm=H, Wm=H, a_exp=K.f16x3_a_exp(0.0, 7.0, 2),
                       res=K.View.full(res.cuda()))
    assert rel_l2(out2.cpu().double(), ref2) < 2e-6

    # head: GN + SiLU, 3 outputs, NCHW
    wh = torch.randn((3, C, 3, 3), generator=g) / (9 * C)**0.5
    bh = 0.1 * torch.randn(3, generator=g)
    ref3 = F.conv2d(F.silu(a), wh.double(), bh.double(), padding=1)
    out3 = torch.empty((B, 3, H, H), device='cuda')
    seg3 = [K.Seg(K.View.full(_nhwc(x).cuda()), TAPS3, scale=sc.float().cuda(), shift=sh.float().cuda(), silu=True)]
    K.conv_igemm_f16x3(seg3, K.pack_f16x3(_pack(wh).cuda(), C, order='natural'), bh.cuda(), None, Hm=H, Wm=H,
                       a_exp=e, out_nchw=out3)
    assert rel_l2(out3.cpu().double(), ref3) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize('pa', [False, True])
@pytest.mark.parametrize('sw', [4, 8, 16, 32])
def test_igemm_f16x3_pointwise_vector_epilogue(sw, pa):
    """The attention out-projection form of the pointwise f16x3 GEMM (transposed accumulators,
    16-byte residual loads and stores): in-place residual Y += O W^T + b into a channel slice,
    exact per-image absmax, and GroupNorm tile partials equal to a stats pass, for every sub-slot
    width; vs float64."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(53)
    B, H, C, N = 3, 16, 256, 8 * sw if 8 * sw >= 128 else 128
    o = (torch.rand((B, H, H, C), generator=g) * 14 - 7) * torch.tensor([1.0, 0.01, 1.0])[:, None, None, None]
    w = torch.randn((N, C), generator=g) / C**0.5
    b = 0.1 * torch.randn(N, generator=g)
    big = torch.randn((B, H, H, N + 64), generator=g) * 3
    ref = o.double() @ w.double().t() + b.double() + big[..., 32:32 + N].double()
    y = big.cuda()
    yv = K.View(y, 32, N)
    gp = K.GnPart.attach(y, sw) if (N + 64) % 32 == 0 and N % (8 * sw) == 0 else None
    am = torch.zeros(B, device='cuda')
    e = K.f16x3_a_exp(0.0, 7.0, 2)
    w3 = K.pack_f16x3(w.cuda(), C, ntaps=1, order='natural')
    ov = K.View.full(o.cuda())
    if pa:  # pre-split A operand (wc_split_f16x3_tiled + wc_proj_f16x3)
        K.proj_f16x3(ov, K.split_f16x3_tiled(ov, e), w3, b.cuda(), yv, a_exp=e, res=yv, absmax=am, gn=gp)
    else:
        K.conv_igemm_f16x3([K.Seg(ov, [(0, 0)])], w3, b.cuda(), yv, Hm=H, Wm=H, a_exp=e, res=yv, absmax=am, gn=gp)
    torch.cuda.synchronize()
    got = y.cpu()
    assert rel_l2(got[..., 32:32 + N].double(), ref) < 2e-6
    assert torch.equal(got[..., :32], big[..., :32]) and torch.equal(got[..., 32 + N:], big[..., 32 + N:])
    assert torch.equal(am.cpu(), got[..., 32:32 + N].reshape(B, -1).abs().amax(1))
    if gp is not None:
        gamma, beta = (1 + torch.randn(N, generator=g)).cuda(), torch.randn(N, generator=g).cuda()
        a1 = K.gn_affine(yv, gamma, beta, bound=True, part=gp)
        a0 = K.gn_affine(yv, gamma, beta, bound=True)
        for u, v in zip(a1, a0):
            assert torch.allclose(u, v, rtol=2e-6, atol=1e-7), (u - v).abs().max()


@pytest.mark.gpu
def test_projections_presplit_bit_identical_to_register_staged(monkeypatch):
    """The attention projections on a pre-split A operand (GN applied and split once by
    wc_split_f16x3_tiled, both operands copied by LDS-DMA) compute the same split values in the
    same MFMA order as the register-staged implicit GEMM: the UNet forward (256-cfg at 64 px, B=2,
    per-sample t) is bit-identical with WC_PROJ_PA=1 and 0; and the pre-split q/k/v equal too."""
    from weatherconverter_amd import kernels as K
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.synthetic import init_synthetic_
    mc = model_config(256)
    mc.im_size = 64
    net = Unet(mc)
    init_synthetic_(net, seed=0)
    net = net.cuda().eval()
    x = torch.randn((2, 3, 64, 64), generator=torch.Generator().manual_seed(9)).cuda()
    outs = []
    for pa in ('1', '0'):
        monkeypatch.setenv('WC_PROJ_PA', pa)
        with torch.no_grad():
            outs.append(net(x, torch.tensor([700, 3]).cuda()).cpu())
    assert torch.equal(outs[0], outs[1])
    # the qkv projection alone: GN prologue in the kernel vs GN in the split pass
    g = torch.Generator().manual_seed(57)
    B, H, C, heads = 2, 16, 256, 4
    y = torch.randn((B, C, H, H), generator=g) * 2 + 1
    gamma, beta = 1 + 0.3 * torch.randn(C, generator=g), 0.3 * torch.randn(C, generator=g)
    sc, sh = _gn_affine(y, gamma, beta)
    w = torch.randn((3 * C, C), generator=g) / C**0.5
    bias = 0.1 * torch.randn(3 * C, generator=g)
    w3 = K.pack_f16x3(w.cuda(), C, ntaps=1, order='natural')
    yv = K.View.full(_nhwc(y).cuda())
    e = K.f16x3_a_exp(float(gamma.abs().max()), float(beta.abs().max()), H * H * C // 8)
    exps = K.attention_exps_from_norms(w.double().abs().sum(1), bias.double().abs(), float(gamma.abs().max()),
                                       float(beta.abs().max()), H * H * C // 8)
    q0 = torch.zeros(B * 6 * C * H * H, dtype=torch.int16, device='cuda')
    q1 = torch.ones_like(q0)
    K.conv_igemm_f16x3_qkv(K.Seg(yv, [(0, 0)], scale=sc.float().cuda(), shift=sh.float().cuda()), w3, bias.cuda(), q0,
                           Hm=H, Wm=H, a_exp=e, C=C, heads=heads, exps=exps)
    a3 = K.split_f16x3_tiled(yv, e, sc.float().cuda().contiguous(), sh.float().cuda().contiguous())
    K.proj_f16x3_qkv(yv, a3, w3, bias.cuda(), q1, a_exp=e, C=C, heads=heads, exps=exps)
    torch.cuda.synchronize()
    assert torch.equal(q0, q1)
    # the attention writing its output pre-split == the split pass over its fp32 output
    N = H * H
    o = torch.empty((B * N, C), device='cuda')
    K.attention_presplit(q0, o, B, N, C, heads, exps)
    a3o = K.attention_presplit_a3(q0, B, N, C, heads, exps)
    a3s = K.split_f16x3_tiled(K.View(o.view(B, H, H, C), 0, C), exps[2])
    torch.cuda.synchronize()
    assert torch.equal(a3o, a3s)


# ---------------------------------------------------------------- producer absmax -> per-image f16x3 scale

def _img_amax(o_bhwc):
    return o_bhwc.reshape(o_bhwc.shape[0], -1).abs().amax(1)


@pytest.mark.gpu
def test_absmax_output_of_split_precision_kernels():
    """absmax_out = exact per-image max |out| of the written values (halo x6 / f16x3, igemm with
    tiles inside one image, straddling tiles, and a transposed-conv parity into a concat slice)."""
    from weatherconverter_amd import kernels as K
    from weatherconverter_amd.diffusion_model.models.engine import pack_convT
    g = torch.Generator().manual_seed(61)
    B, H, C, N = 3, 16, 64, 128
    x = torch.randn((B, C, H, H), generator=g) * torch.tensor([1.0, 30.0, 0.01])[:, None, None, None]
    sc = (1 + 0.3 * torch.randn((B, C), generator=g)).cuda()
    sh = (0.3 * torch.randn((B, C), generator=g)).cuda()
    w = (torch.randn((N, 9 * C), generator=g) / (9 * C)**0.5).cuda()
    xv = K.View.full(_nhwc(x).cuda())
    seg = [K.Seg(xv, TAPS3, scale=sc, shift=sh, silu=True)]
    for mode in ('x6', 'f3'):
        out = torch.empty((B, H, H, N), device='cuda')
        am = torch.zeros(B, device='cuda')
        if mode == 'x6':
            K.conv3x3_x6(seg, K.pack_x6(w, C), None, K.View.full(out), Hm=H, Wm=H, absmax=am)
        else:
            K.conv3x3_f16x3(seg, K.pack_f16x3(w, C), None, K.View.full(out), Hm=H, Wm=H, a_exp=6, absmax=am)
        torch.cuda.synchronize()
        assert torch.equal(am.cpu(), _img_amax(out.cpu())), mode
    # igemm x6: 8x8 grids straddle images (BM = 128), 16x16 grids do not
    for Hm in (8, 16):
        xr = torch.randn((B, Hm, Hm, C), generator=g) * torch.tensor([2.0, 0.1, 50.0])[:, None, None, None]
        wr = (torch.randn((N, C), generator=g) / C**0.5).cuda()
        out = torch.empty((B, Hm, Hm, N), device='cuda')
        am = torch.zeros(B, device='cuda')
        K.conv_igemm_x6([K.Seg(K.View.full(xr.cuda()), [(0, 0)])], K.pack_x6(wr, C, ntaps=1, order='natural'), None,
                        K.View.full(out), Hm=Hm, Wm=Hm, absmax=am)
        torch.cuda.synchronize()
        assert torch.equal(am.cpu(), _img_amax(out.cpu())), Hm
    # transposed conv parity into the first half of a concat buffer whose other half holds 1e6
    Ci, Co = 128, 64
    wt = torch.randn((Ci, Co, 4, 4), generator=g) / (4 * Ci)**0.5
    xt = K.View.full(torch.randn((B, 8, 8, Ci), generator=g).cuda())
    buf = torch.full((B, 16, 16, 2 * Co), 1e6, device='cuda')
    am = torch.zeros(B, device='cuda')
    for py in (0, 1):
        for px in (0, 1):
            taps, wp = pack_convT(wt, py, px)
            K.conv_igemm_x6([K.Seg(xt, taps)], K.pack_x6(wp.cuda(), Ci, 0, ntaps=4, order='natural'), None,
                            K.View(buf, 0, Co), Hm=8, Wm=8, out_map=(2, 2, py, px), absmax=am)
    torch.cuda.synchronize()
    assert torch.equal(am.cpu(), _img_amax(buf.cpu()[..., :Co]))


@pytest.mark.gpu
def test_fp32_conv_rejects_absmax():
    from weatherconverter_amd import kernels as K, _native
    x = torch.randn((1, 8, 8, 16), device='cuda')
    w = torch.randn((16, 16), device='cuda')
    out = torch.empty((1, 8, 8, 16), device='cuda')
    am = torch.zeros(1, device='cuda')
    a = K._conv_args([K.Seg(K.View.full(x), [(0, 0)])], 16, None, K.View.full(out), 8, 8, None, 0, None,
                     (1, 1, 0, 0), None, 0, am)
    a.w, a.ldw = w.data_ptr(), 16
    rc = _native.load().wc_conv_igemm(ctypes.byref(a), None)
    assert rc != 0


@pytest.mark.gpu
def test_igemm_f16x3_resampling_with_producer_bound():
    """Down-sampling 4x4/s2 conv and the transposed conv's four parities on f16x3, scaled per image
    by a bound: images of very different magnitude and one outlier, vs float64; the bound comes
    from the producer's absmax.  A straddling grid with a bound is rejected."""
    from weatherconverter_amd import kernels as K
    from weatherconverter_amd.diffusion_model.models.engine import pack_convT
    g = torch.Generator().manual_seed(62)
    B, H, Ci, Co = 3, 32, 64, 128
    x = torch.randn((B, Ci, H, H), generator=g) * torch.tensor([1.0, 1e3, 1e-3])[:, None, None, None]
    x[0, 5, 7, 9] = 4e4  # one outlier in image 0: far past the fp16 range unscaled
    # producer: an identity 1x1 conv on bf16x6 whose epilogue emits the absmax
    xin = _nhwc(x).cuda()
    xp = torch.empty_like(xin)
    am = torch.zeros(B, device='cuda')
    K.conv_igemm_x6([K.Seg(K.View.full(xin), [(0, 0)])], K.pack_x6(torch.eye(Ci).cuda(), Ci, ntaps=1,
                    order='natural'), None, K.View.full(xp), Hm=H, Wm=H, absmax=am)
    torch.cuda.synchronize()
    assert torch.equal(xp.cpu(), xin.cpu()) and torch.equal(am.cpu(), _img_amax(xin.cpu()))
    w = torch.randn((Co, Ci, 4, 4), generator=g) / (16 * Ci)**0.5
    b = torch.randn(Co, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1)
    seg = [K.Seg(K.View.full(xp), TAPS4S2, stride=2)]
    outs = {}
    for mode in ('f16x3', 's2d', 'fp32'):
        o = torch.empty((B, H // 2, H // 2, Co), device='cuda')
        if mode == 's2d':  # the halo kernel over the space-to-depth view (wc_conv4x4s2_f16x3)
            assert K.conv4x4s2_f16x3_ok(seg[0], Co, H // 2, H // 2)
            K.conv4x4s2_f16x3(seg[0], K.pack_f16x3_s2d(_pack(w).cuda(), Ci), b.cuda(), K.View.full(o),
                              Hm=H // 2, Wm=H // 2, a_bound=am)
        elif mode == 'f16x3':
            K.conv_igemm_f16x3(seg, K.pack_f16x3(_pack(w).cuda(), Ci, ntaps=16, order='natural'), b.cuda(),
                               K.View.full(o), Hm=H // 2, Wm=H // 2, a_exp=60, a_bound=am)
        else:
            K.conv_igemm(seg, _pack(w).cuda(), b.cuda(), K.View.full(o), Hm=H // 2, Wm=H // 2)
        torch.cuda.synchronize()
        outs[mode] = _nchw(o.cpu()).double()
    for i in range(B):  # per image: each one's own scale
        e32 = rel_l2(outs['fp32'][i], ref[i])
        for mode in ('f16x3', 's2d'):
            e3 = rel_l2(outs[mode][i], ref[i])
            assert e3 < 1e-5 and e3 <= 4 * e32 + 2e-7, (mode, i, e3, e32)

    # transposed conv (ConvTranspose2d(Ci, Co2, 4, 2, 1)) from the same producer output
    Co2 = 64
    wt = torch.randn((Ci, Co2, 4, 4), generator=g) / (4 * Ci)**0.5
    bt = torch.randn(Co2, generator=g) * 0.1
    reft = F.conv_transpose2d(x.double(), wt.double(), bt.double(), stride=2, padding=1)
    xv = K.View.full(xp)
    for mode in ('f16x3', 'fp32'):
        buf = torch.full((B, 2 * H, 2 * H, 2 * Co2), 5.0, device='cuda')
        dst = K.View(buf, 0, Co2)
        for py in (0, 1):
            for px in (0, 1):
                taps, wp = pack_convT(wt, py, px)
                if mode == 'f16x3':
                    K.conv_igemm_f16x3([K.Seg(xv, taps)], K.pack_f16x3(wp.cuda(), Ci, ntaps=4, order='natural'),
                                       bt.cuda(), dst, Hm=H, Wm=H, a_exp=60, a_bound=am, out_map=(2, 2, py, px))
                else:
                    K.conv_igemm([K.Seg(xv, taps)], wp.cuda(), bt.cuda(), dst, Hm=H, Wm=H, out_map=(2, 2, py, px))
        torch.cuda.synchronize()
        bc = buf.cpu()
        assert bool((bc[..., Co2:] == 5.0).all())
        outs[mode] = _nchw(bc[..., :Co2]).double()
    for i in range(B):
        e3, e32 = rel_l2(outs['f16x3'][i], reft[i]), rel_l2(outs['fp32'][i], reft[i])
        assert e3 < 1e-5 and e3 <= 4 * e32 + 2e-7, (i, e3, e32)

    with pytest.raises(RuntimeError):  # 12x12 grid: BM = 128 tiles straddle images
        xs = K.View.full(torch.randn((B, 12, 12, Ci), device='cuda'))
        K.conv_igemm_f16x3([K.Seg(xs, [(0, 0)])], K.pack_f16x3(torch.randn(Co, Ci).cuda(), Ci, ntaps=1,
                           order='natural'), None, K.View.full(torch.empty((B, 12, 12, Co), device='cuda')),
                           Hm=12, Wm=12, a_exp=60, a_bound=am)


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Ci,Co,ldc', [(2, 16, 32, 128, 128, 256), (1, 32, 32, 256, 256, 256),
                                             (2, 16, 64, 64, 192, 64)])
def test_conv4x4s2_s2d_vs_float64(B, H, W, Ci, Co, ldc):
    """wc_conv4x4s2_f16x3 (the down conv as a 2x2 conv over the space-to-depth input on the halo
    kernel) against float64 and the implicit-GEMM f16x3 path: strided input views, non-square
    grids, a ragged N tile (192 = 128 + 64), border blocks on every side, GN tile partials from the
    epilogue vs a stats pass; shapes outside its tiling are refused."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(7 + Ci)
    x = torch.randn((B, Ci, H, W), generator=g) * torch.tensor([3.0, 0.01][:B])[:, None, None, None]
    buf = torch.randn((B, H, W, ldc), generator=g).cuda()
    buf[..., :Ci] = _nhwc(x).cuda()
    xv = K.View(buf, 0, Ci)
    am = _img_amax(_nhwc(x)).cuda()
    w = torch.randn((Co, Ci, 4, 4), generator=g) / (16 * Ci)**0.5
    b = torch.randn(Co, generator=g) * 0.1
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1)
    seg = K.Seg(xv, TAPS4S2, stride=2)
    Hm, Wm = H // 2, W // 2
    assert K.conv4x4s2_f16x3_ok(seg, Co, Hm, Wm)
    o = torch.empty((B, Hm, Wm, Co), device='cuda')
    gp = K.GnPart.attach(o, 8) if Co % 32 == 0 else None
    K.conv4x4s2_f16x3(seg, K.pack_f16x3_s2d(_pack(w).cuda(), Ci), b.cuda(), K.View.full(o), Hm=Hm, Wm=Wm,
                      a_bound=am, gn=gp)
    oi = torch.empty_like(o)
    K.conv_igemm_f16x3([seg], K.pack_f16x3(_pack(w).cuda(), Ci, ntaps=16, order='natural'), b.cuda(),
                       K.View.full(oi), Hm=Hm, Wm=Wm, a_exp=60, a_bound=am)
    torch.cuda.synchronize()
    got, gi = _nchw(o.cpu()).double(), _nchw(oi.cpu()).double()
    for i in range(B):
        assert rel_l2(got[i], ref[i]) < 1e-5, (i, rel_l2(got[i], ref[i]))
        assert rel_l2(got[i], gi[i]) < 1e-5
    if gp is not None:  # epilogue partials give the stats pass's GroupNorm affine
        gam, bet = torch.randn(Co).cuda(), torch.randn(Co).cuda()
        s1, h1 = K.gn_affine(K.View.full(o), gam, bet, part=gp)
        s2, h2 = K.gn_affine(K.View.full(o), gam, bet)
        torch.cuda.synchronize()
        assert torch.allclose(s1, s2, rtol=1e-5, atol=0) and torch.allclose(h1, h2, rtol=1e-5, atol=1e-6)
    bad = K.Seg(K.View.full(torch.randn((B, 12, 32, Ci), device='cuda')), TAPS4S2, stride=2)
    assert not K.conv4x4s2_f16x3_ok(bad, Co, 6, 16)


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Ci,Co', [(2, 8, 16, 64, 128), (2, 16, 32, 128, 64), (1, 8, 32, 32, 192)])
def test_convT4x4s2_one_launch_vs_float64(B, H, W, Ci, Co):
    """wc_convtr4x4s2_f16x3 (all four output parities in one launch of the halo kernel) against
    float64 and the four implicit-GEMM parities, writing the first half of a wider (skip-concat)
    buffer whose other half stays untouched; both tile forms (N <= 64: TH 16), a ragged N tile;
    GN tile partials from the epilogue vs a stats pass."""
    from weatherconverter_amd import kernels as K
    from weatherconverter_amd.diffusion_model.models.engine import pack_convT
    g = torch.Generator().manual_seed(11 + Co)
    x = torch.randn((B, Ci, H, W), generator=g) * torch.tensor([2.0, 1e-2][:B])[:, None, None, None]
    xin = _nhwc(x).cuda()
    am = _img_amax(_nhwc(x)).cuda()
    wt = torch.randn((Ci, Co, 4, 4), generator=g) / (4 * Ci)**0.5
    bt = torch.randn(Co, generator=g) * 0.1
    ref = F.conv_transpose2d(x.double(), wt.double(), bt.double(), stride=2, padding=1)
    seg = K.Seg(K.View.full(xin), [(0, 0)])
    assert K.convT4x4s2_f16x3_ok(seg, Co)
    outs = {}
    for mode in ('one', 'parities'):
        buf = torch.full((B, 2 * H, 2 * W, 2 * Co), 5.0, device='cuda')
        dst = K.View(buf, 0, Co)
        gp = K.GnPart.attach(buf, 8) if mode == 'one' else None
        if mode == 'one':
            K.convT4x4s2_f16x3(seg, K.pack_f16x3_convT(wt.cuda()), bt.cuda(), dst, a_bound=am, gn=gp)
        else:
            for py in (0, 1):
                for px in (0, 1):
                    taps, wp = pack_convT(wt, py, px)
                    K.conv_igemm_f16x3([K.Seg(K.View.full(xin), taps)], K.pack_f16x3(wp.cuda(), Ci, ntaps=4,
                                       order='natural'), bt.cuda(), dst, Hm=H, Wm=W, a_exp=60, a_bound=am,
                                       out_map=(2, 2, py, px))
        torch.cuda.synchronize()
        bc = buf.cpu()
        assert bool((bc[..., Co:] == 5.0).all())
        outs[mode] = _nchw(bc[..., :Co]).double()
        if gp is not None:
            gam, bet = torch.randn(Co).cuda(), torch.randn(Co).cuda()
            s1, h1 = K.gn_affine(dst, gam, bet, part=gp)
            s2, h2 = K.gn_affine(dst, gam, bet)
            torch.cuda.synchronize()
            assert torch.allclose(s1, s2, rtol=1e-5, atol=0) and torch.allclose(h1, h2, rtol=1e-5, atol=1e-6)
    for i in range(B):
        assert rel_l2(outs['one'][i], ref[i]) < 1e-5, (i, rel_l2(outs['one'][i], ref[i]))
        assert rel_l2(outs['one'][i], outs['parities'][i]) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize('form', ['convT', 's2d'])
def test_halo_resample_residual_and_absmax(form):
    """The training data gradients of the down / up convs: the one-launch ConvT and the
    space-to-depth down conv with the epilogue residual (out = conv + res, the gradient accumulating)
    and the per-image absmax of the values written, against float64; into a wider buffer whose
    other channels stay untouched."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(21)
    B, Ci, Co = 2, 64, 128
    H, W = (8, 16) if form == 'convT' else (16, 32)
    x = torch.randn((B, Ci, H, W), generator=g) * torch.tensor([2.0, 1e-2])[:, None, None, None]
    xin = _nhwc(x).cuda()
    am = _img_amax(_nhwc(x)).cuda()
    if form == 'convT':
        wt = torch.randn((Ci, Co, 4, 4), generator=g) / (4 * Ci)**0.5
        ref = F.conv_transpose2d(x.double(), wt.double(), None, stride=2, padding=1)
        Ho, Wo = 2 * H, 2 * W
    else:
        w = torch.randn((Co, Ci, 4, 4), generator=g) / (16 * Ci)**0.5
        ref = F.conv2d(x.double(), w.double(), None, stride=2, padding=1)
        Ho, Wo = H // 2, W // 2
    r0 = torch.randn((B, Ho, Wo, 2 * Co), generator=g)
    buf = r0.clone().cuda()
    dst = K.View(buf, 0, Co)
    amx = torch.zeros(B, device='cuda')
    seg = K.Seg(K.View.full(xin), [(0, 0)]) if form == 'convT' else K.Seg(K.View.full(xin), TAPS4S2, stride=2)
    if form == 'convT':
        assert K.convT4x4s2_f16x3_ok(seg, Co)
        K.convT4x4s2_f16x3(seg, K.pack_f16x3_convT(wt.cuda()), None, dst, a_bound=am, res=dst, absmax=amx)
    else:
        assert K.conv4x4s2_f16x3_ok(seg, Co, Ho, Wo)
        K.conv4x4s2_f16x3(seg, K.pack_f16x3_s2d(_pack(w).cuda(), Ci), None, dst, Hm=Ho, Wm=Wo, a_bound=am, res=dst,
                          absmax=amx)
    torch.cuda.synchronize()
    bc = buf.cpu()
    assert torch.equal(bc[..., Co:], r0[..., Co:])
    want = ref + _nchw(r0[..., :Co]).double()
    got = _nchw(bc[..., :Co]).double()
    for i in range(B):
        assert rel_l2(got[i], want[i]) < 1e-5, (i, rel_l2(got[i], want[i]))
    assert torch.equal(amx.cpu(), bc[..., :Co].abs().amax((1, 2, 3)))


# ---------------------------------------------------------------- GroupNorm tile partials (epilogue-fused statistics)

@pytest.mark.gpu
@pytest.mark.parametrize('sw', [4, 8, 16, 32])
def test_gn_tile_partials_match_stats_pass(sw):
    """GroupNorm affine from tile partials emitted by (a) the halo conv's epilogue, (b) the implicit
    GEMM's epilogue for the four ConvT parities (pixel-block offsets) into half of a skip buffer and
    (c) wc_gn_partials for the other half == the stats-pass affine (wc_gn_stats) within fp32 rounding,
    for the half views and the whole buffer."""
    from weatherconverter_amd import kernels as K
    from weatherconverter_amd.diffusion_model.models.engine import pack_convT
    g = torch.Generator().manual_seed(71)
    B, H, C = 2, 16, 8 * sw
    # (a) 3x3 halo conv writing a (B, H, H, C) tensor with partials
    x = torch.randn((B, H, H, 64), generator=g).cuda() * 2 + 3
    sc = (1 + 0.2 * torch.randn((B, 64), generator=g)).cuda()
    sh = (0.2 * torch.randn((B, 64), generator=g)).cuda()
    w = (torch.randn((C, 9 * 64), generator=g) / 24).cuda()
    y = torch.empty((B, H, H, C), device='cuda')
    gp = K.GnPart.attach(y, sw)
    K.conv3x3_f16x3([K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True)], K.pack_f16x3(w, 64),
                    (torch.randn(C, generator=g) + 5).cuda(), K.View.full(y), Hm=H, Wm=H, a_exp=6, gn=gp)
    gamma, beta = (1 + torch.randn(C, generator=g)).cuda(), torch.randn(C, generator=g).cuda()
    a1 = K.gn_affine(K.View.full(y), gamma, beta, bound=True, part=gp)
    a0 = K.gn_affine(K.View.full(y), gamma, beta, bound=True)
    for u, v in zip(a1, a0):
        assert torch.allclose(u, v, rtol=2e-6, atol=1e-7), (u - v).abs().max()
    # (b)+(c) skip buffer (B, 2H, 2H, 2C): ConvT parities into [0, C), a raw tensor copied into [C, 2C)
    U = torch.full((B, 2 * H, 2 * H, 2 * C), float('nan'), device='cuda')
    gu = K.GnPart.attach(U, sw)
    xt = K.View.full(torch.randn((B, H, H, 64), generator=g).cuda())
    wt = torch.randn((64, C, 4, 4), generator=g) / 16
    for par, (py, px) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        taps, wp = pack_convT(wt, py, px)
        K.conv_igemm_x6([K.Seg(xt, taps)], K.pack_x6(wp.cuda(), 64, 0, ntaps=4, order='natural'), None,
                        K.View(U, 0, C), Hm=H, Wm=H, out_map=(2, 2, py, px), gn=gu, gn_p64=par * H * H // 64)
    U[..., C:] = torch.randn((B, 2 * H, 2 * H, C), generator=g).cuda() * 3 - 1
    K.gn_partials(K.View(U, C, C), gu)
    for v in (K.View(U, 0, C), K.View(U, C, C), K.View.full(U)):
        gm, bt = (1 + torch.randn(v.C, generator=g)).cuda(), torch.randn(v.C, generator=g).cuda()
        a1 = K.gn_affine(v, gm, bt, part=gu)
        a0 = K.gn_affine(v, gm, bt)
        for u_, v_ in zip(a1, a0):
            assert torch.isfinite(u_).all() and torch.allclose(u_, v_, rtol=2e-6, atol=1e-7), (u_ - v_).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize('precision', ['f16x3', 'bf16x6', 'fp32'])
def test_unet_gn_partials_equal_stats_pass(precision):
    """The whole UNet (256-cfg at 64 px, B=2) with epilogue GN partials vs one stats pass per GN."""
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.synthetic import init_synthetic_
    mc = model_config(256)
    mc.im_size = 64
    net = Unet(mc)
    init_synthetic_(net, seed=0)
    net.set_conv_precision(precision)
    net = net.cuda().eval()
    x = torch.randn((2, 3, 64, 64), generator=torch.Generator().manual_seed(3)).cuda()
    with torch.no_grad():
        y1 = net(x, torch.tensor([400]).cuda())
        net.engine().gn_partials = False
        y0 = net(x, torch.tensor([400]).cuda())
    assert rel_l2(y1, y0) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,C,heads', [(2, 16, 128, 4), (2, 16, 512, 4), (1, 16, 768, 4), (2, 32, 256, 4),
                                         (1, 16, 64, 2)])
def test_qkv_presplit_attention_bit_identical(B, H, C, heads):
    """The pre-split path (in_proj epilogue writes scaled fp16 pieces, attention copies K / V^T tiles
    by LDS-DMA) against the fp32-projection path: the same split values and MFMA order, so the
    attention output is bit-identical; and both within the fp32 tolerance of float64."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(77)
    N = H * H
    x = torch.randn((B, C, H, H), generator=g) * 2 + 1
    gamma = 1 + 0.3 * torch.randn(C, generator=g)
    beta = 0.3 * torch.randn(C, generator=g)
    sc, sh = _gn_affine(x, gamma, beta)
    w_in = torch.randn((3 * C, C), generator=g) / C**0.5
    b_in = 0.1 * torch.randn(3 * C, generator=g)
    ga, ba = float(gamma.abs().max()), float(beta.abs().max())
    a_exp = K.f16x3_a_exp(ga, ba, N * C // 8)
    exps = K.attention_f16x3_exps(w_in, b_in, ga, ba, N * C // 8)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda()
    seg = K.Seg(K.View.full(xd), [(0, 0)], scale=sc.float().cuda(), shift=sh.float().cuda())
    w3 = K.pack_f16x3(w_in.cuda(), C, ntaps=1, order='natural')
    bias = b_in.cuda()
    assert K.qkv_presplit_ok(B, N, C, heads)
    qkv = torch.empty((B, H, H, 3 * C), device='cuda')
    K.conv_igemm_f16x3([seg], w3, bias, K.View.full(qkv), Hm=H, Wm=H, a_exp=a_exp)
    ref_out = torch.empty((B * N, C), device='cuda')
    K.attention(qkv.view(B * N, 3 * C), ref_out, B, N, C, heads, 'f16x3', exps)
    qkv3 = torch.empty(B * 6 * C * N, dtype=torch.int16, device='cuda')
    K.conv_igemm_f16x3_qkv(seg, w3, bias, qkv3, Hm=H, Wm=H, a_exp=a_exp, C=C, heads=heads, exps=exps)
    out = torch.full((B * N, C), 7.0, device='cuda')
    K.attention_presplit(qkv3, out, B, N, C, heads, exps)
    torch.cuda.synchronize()
    assert torch.equal(out, ref_out)
    # the pre-split pieces are the scaled projection: q piece h + l == fp32 q * 2^eq (to 2^-22)
    D = C // heads
    q3 = qkv3.view(B, 6 * C * N)[:, :2 * D * N].view(B, 2, D // 8, N, 8)  # head 0, pieces of q
    qh = q3.view(torch.float16).float()
    q_rec = (qh[:, 0] + qh[:, 1]).permute(0, 2, 1, 3).reshape(B, N, D)
    q_ref = qkv.view(B, N, 3 * C)[:, :, :D] * 2.0**exps[0]
    assert rel_l2(q_rec.double().cpu(), q_ref.double().cpu()) < 1e-6
    a = (x.double() * sc[:, :, None, None] + sh[:, :, None, None]).permute(0, 2, 3, 1).reshape(B, N, C)
    ref64 = _attn_ref((a @ w_in.double().t() + b_in.double()).float(), B, N, C, heads)
    assert rel_l2(out.cpu().double().reshape(B, N, C), ref64) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,C,heads', [(2, 16, 16, 128, 4), (1, 32, 32, 512, 4), (2, 16, 32, 768, 4),
                                           (1, 64, 64, 256, 4), (3, 16, 24, 256, 2)])
def test_proj_pa256_bit_identical_to_128_rows(B, H, W, C, heads):
    """The pre-split projection GEMM on 256 x 128 tiles (proj_pa_kernel<QKV, 2, false>) against the
    128 x 128 LDS-DMA form: the out-projection form (in-place residual, bias, per-image absmax, GroupNorm tile
    partials) and the pre-split qkv form give bit-identical results; 16 x 24 images (HW % 256 != 0)
    fall back to 128 rows.  And the out-projection within the f16x3 tolerance of float64."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(91)
    HW = H * W
    o = torch.rand((B, H, W, C), generator=g) * 14 - 7
    e = K.f16x3_a_exp(0.0, 7.0, 2)
    ov = K.View.full(o.cuda())
    a3 = K.split_f16x3_tiled(ov, e)
    w = torch.randn((C, C), generator=g) / C**0.5
    b = 0.1 * torch.randn(C, generator=g)
    w3 = K.pack_f16x3(w.cuda(), C, ntaps=1, order='natural')
    y0 = torch.randn((B, H, W, C), generator=g)
    w_in = torch.randn((3 * C, C), generator=g) / C**0.5
    b_in = 0.1 * torch.randn(3 * C, generator=g)
    w3q = K.pack_f16x3(w_in.cuda(), C, ntaps=1, order='natural')
    res = {}
    prev = K.set_proj_tile(256)
    try:
        for rows in (256, 128):  # 256 x 128; the 128 x 128 LDS-DMA form
            K.set_proj_tile(rows)
            y = y0.cuda()
            yv = K.View.full(y)
            gp = K.GnPart.attach(y, 8)
            am = torch.zeros(B, device='cuda')
            K.proj_f16x3(ov, a3, w3, b.cuda(), yv, a_exp=e, res=yv, absmax=am, gn=gp)
            name = K._native.last_kernel_name()
            qkv3 = torch.zeros(B * 6 * C * HW, dtype=torch.int16, device='cuda')
            K.proj_f16x3_qkv(ov, a3, w3q, b_in.cuda(), qkv3, a_exp=e, C=C, heads=heads, exps=(9, 8, 7))
            torch.cuda.synchronize()
            res[rows] = (y.cpu(), am.cpu(), gp.part.cpu(), qkv3.cpu(), name)
    finally:
        K.set_proj_tile(prev)
    big = HW % 256 == 0
    assert res[256][4].startswith('proj_pa_kernel<false, 2' if big else 'conv_igemm_x6_kernel'), res[256][4]
    assert res[128][4].startswith('conv_igemm_x6_kernel'), res[128][4]
    for u, v in zip(res[256][:4], res[128][:4]):
        assert torch.equal(u, v)
    ref = o.double() @ w.double().t() + b.double() + y0.double()
    assert rel_l2(res[256][0].double(), ref) < 2e-6
    assert torch.equal(res[256][1], res[256][0].reshape(B, -1).abs().amax(1))


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,C,ld,gn', [(2, 16, 16, 64, 64, True), (1, 32, 32, 512, 512, False),
                                         (2, 8, 32, 96, 160, True), (3, 16, 8, 32, 32, False)])
def test_split_tiled_layout_vs_torch(B, H, W, C, ld, gn):
    """wc_split_f16x3_tiled: every value lands at its [mt][k-step][piece][k-half][row][8] slot of the GEMM's
    LDS stage order, the two fp16 pieces sum to (x sc + sh) 2^e within the split's 2^-22 relative, the
    high piece is the round-to-nearest fp16 of the value; strided channel views (ld > C)."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(3)
    t = torch.randn((B, H, W, ld), generator=g) * 3
    sc = (1 + 0.2 * torch.randn((B, C), generator=g)) if gn else None
    sh = (0.3 * torch.randn((B, C), generator=g)) if gn else None
    e = 5
    v = K.View(t.cuda(), 0, C)
    a3 = K.split_f16x3_tiled(v, e, sc.cuda() if gn else None, sh.cuda() if gn else None)
    torch.cuda.synchronize()
    M = B * H * W
    raw = a3.cpu().view(torch.float16).reshape(M // 128, C // 16, 2, 2, 128, 8)  # [mt][ks][piece][kh][row][8]
    pieces = raw.permute(2, 0, 4, 1, 3, 5).reshape(2, M, C).double()  # [piece][row][channel]
    x = t[..., :C].reshape(M, C).double()
    if gn:
        x = (x.reshape(B, H * W, C) * sc.double()[:, None] + sh.double()[:, None]).reshape(M, C)
    ref = x * 2.0**e
    assert torch.allclose(pieces[0] + pieces[1], ref, rtol=2e-6, atol=1e-6)
