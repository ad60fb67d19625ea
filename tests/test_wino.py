"""The Winograd F(2,3)-along-x ResBlock conv (csrc/wc_wino.hip, kernels.pack_wino / conv3x3_wino).

CPU: the transform algebra and the weight pack — the packed fp16 pieces, read back through the
layout the kernel uses, reconstruct the float64 filter transform, and the F(2,3) algorithm evaluated in
float64 on them reproduces the direct 3x3 conv (+ the 1x1 residual folded into positions 0 and 3).
GPU: the kernel against a float64 direct conv (reference ResBlock convs unet_base.py:87-109,
:146-150), within 4x (+2e-7) of the direct f16x3 kernel's own error and 1e-5, with bias, temb, residual
segment (chunk counts equal and unequal), the epilogue residual view, per-image absmax and GroupNorm
tile partials.
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]


def rel_l2(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def _pack(w):  # [Co][Ci][3][3] -> [Co][9 * Ci], K = (ky * 3 + kx, c) (engine.pack_conv)
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


def _unpack_wino(wp, N, C0, C1):
    """Invert pack_wino's layout: (U [N][3][4][C0] float64, residual [N][C1] float64) from the pieces."""
    BN, T = wp.BN, wp.data.shape[0]
    d = wp.data.cpu()
    n0 = 3 * 4 * C0 * 2 * BN
    seg0 = d[:, :n0].reshape(T, C0 // 16, 3, 4, 2, 2, BN, 8).view(torch.float16).double()
    u = (seg0[:, :, :, :, 0] + seg0[:, :, :, :, 1])  # [T][nc][3][4][kh][BN][8]
    u = u.permute(0, 5, 2, 3, 1, 4, 6).reshape(T * BN, 3, 4, C0)
    ws = wp.wsinv.cpu().double()
    U = u[:N] * ws[:N, None, None, None]
    R = None
    if C1:
        seg1 = d[:, n0:].reshape(T, C1 // 16, 2, 2, BN, 8).view(torch.float16).double()
        r = (seg1[:, :, 0] + seg1[:, :, 1]).permute(0, 3, 1, 2, 4).reshape(T * BN, C1)
        R = r[:N] * ws[:N, None]
    return U, R


def _wino_conv_f64(a, U, bias):
    """F(2,3) along x in float64: a [B][C][H][W] (prologue applied), U [N][3][4][C] -> [B][N][H][W]."""
    B, C, H, W = a.shape
    ap = F.pad(a, (1, 1, 1, 1))
    out = torch.zeros((B, U.shape[0], H, W), dtype=torch.float64)
    for ky in range(3):
        rows = ap[:, :, ky:ky + H, :]  # input rows oy + ky - 1
        d = [rows[:, :, :, k:k + W - 1:2] for k in range(4)]  # d_k of output pair t: column 2t - 1 + k
        V = [d[0] - d[2], d[1] + d[2], d[2] - d[1], d[1] - d[3]]
        M = [torch.einsum('bcht,nc->bnht', V[p], U[:, ky, p]) for p in range(4)]
        out[:, :, :, 0::2] += M[0] + M[1] + M[2]
        out[:, :, :, 1::2] += M[1] - M[2] - M[3]
    return out + bias[None, :, None, None]


@pytest.mark.parametrize('N,C0,C1', [(128, 32, 0), (64, 48, 32), (192, 16, 64)])
def test_pack_wino_reconstructs_the_filter_transform(N, C0, C1):
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(7)
    w = torch.randn((N, 9 * C0 + C1), generator=g) * torch.rand((N, 1), generator=g) * 3
    wp = K.pack_wino(w, C0, C1)
    assert wp.order == 'wino' and wp.res_f16 == bool(C1)
    assert wp.data.numel() * 2 == wp.data.shape[0] * (12 * C0 // 16 + C1 // 16) * wp.BN * 64
    U, R = _unpack_wino(wp, N, C0, C1)
    Uref = K.wino_filter(w, C0)
    assert rel_l2(U, Uref) < 3e-7
    # the per-channel scale puts every packed value under 2^14 and the largest at >= 2^13
    ws = wp.wsinv[:N].double()
    amax = Uref.abs().reshape(N, -1).amax(1)
    if C1:
        amax = torch.maximum(amax, w[:, 9 * C0:].double().abs().amax(1))
        assert rel_l2(R, w[:, 9 * C0:].double()) < 3e-7
    scaled = amax / ws
    assert bool((scaled <= 2**14).all()) and bool((scaled >= 2**13).all())


@pytest.mark.parametrize('B,H,W,Ci,Co,Cr', [(1, 4, 8, 16, 8, 0), (2, 6, 10, 8, 4, 5)])
def test_wino_algebra_equals_direct_conv(B, H, W, Ci, Co, Cr):
    """F(2,3) in float64 on the exact filter transform (+ the residual in positions 0 and 3) equals
    the direct conv to rounding."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(3)
    a = torch.randn((B, Ci, H, W), generator=g, dtype=torch.float64)
    w = torch.randn((Co, Ci, 3, 3), generator=g, dtype=torch.float64)
    b = torch.randn(Co, generator=g, dtype=torch.float64)
    U = K.wino_filter(_pack(w), Ci)
    got = _wino_conv_f64(a, U, b)
    ref = F.conv2d(a, w, b, padding=1)
    if Cr:
        xr = torch.randn((B, Cr, H, W), generator=g, dtype=torch.float64)
        wr = torch.randn((Co, Cr), generator=g, dtype=torch.float64)
        r = torch.einsum('bchw,nc->bnhw', xr, wr)
        ref = ref + r
        # the residual in the transform domain: M0 += x_even W_r, M3 += (-x_odd) W_r
        got = got + torch.stack([r[..., 0::2], r[..., 1::2]], -1).reshape(ref.shape)
    assert rel_l2(got, ref) < 1e-14


def _gn_affine(x, gamma, beta, G=8, eps=1e-5):
    B, C = x.shape[:2]
    xg = x.double().reshape(B, G, -1)
    rstd = 1.0 / torch.sqrt(xg.var(-1, unbiased=False) + eps)
    mean = xg.mean(-1)
    sc = rstd.repeat_interleave(C // G, 1) * gamma.double()
    sh = beta.double() - mean.repeat_interleave(C // G, 1) * sc
    return sc, sh


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2)


WINO_CASES = [
    # B, H, W, Ci, Co, Cr, gamma scale, outlier
    (2, 16, 32, 64, 128, 0, 1.0, False),    # odd chunk count 4 -> even; two N tiles
    (1, 8, 16, 48, 256, 48, 1.0, False),    # 3 chunks, residual chunks == 3x3 chunks
    (2, 16, 16, 32, 128, 96, 1.0, False),   # residual chunks > 3x3 chunks
    (1, 32, 16, 128, 64, 64, 1.0, False),   # the BN = 64 / TH = 16 form
    (1, 16, 16, 64, 128, 32, 20.0, True),   # Samuelson-extreme outlier + large gamma
    (1, 16, 16, 16, 64, 0, 1.0, False),     # one chunk, BN = 64
]


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Ci,Co,Cr,gs,outlier', WINO_CASES)
def test_conv3x3_wino_vs_float64(B, H, W, Ci, Co, Cr, gs, outlier):
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(41)
    h = torch.randn((B, Ci, H, W), generator=g) * 3 + 0.7
    if outlier:
        h.zero_()
        h[:, ::Ci // 8, 0, 0] = 1e4
    gamma = gs * (1 + 0.3 * torch.randn(Ci, generator=g))
    beta = 0.5 * torch.randn(Ci, generator=g)
    sc, sh = _gn_affine(h, gamma, beta)
    x2 = torch.randn((B, max(Cr, 16), H, W), generator=g) * 5
    w = torch.randn((Co, Ci, 3, 3), generator=g) / (Ci * 9)**0.5
    wr = torch.randn((Co, max(Cr, 16), 1, 1), generator=g) / max(Cr, 16)**0.5
    b = torch.randn(Co, generator=g) * 0.1
    temb = torch.randn((B, Co + 8), generator=g)
    a = F.silu(h.double() * sc[:, :, None, None] + sh[:, :, None, None])
    ref = F.conv2d(a, w.double(), b.double(), padding=1) + temb[:, :Co].double()[:, :, None, None]
    segs = [K.Seg(K.View.full(_nhwc(h).cuda()), TAPS3, scale=sc.float().cuda(), shift=sh.float().cuda(), silu=True)]
    wp = _pack(w)
    xb = None
    if Cr:
        ref = ref + F.conv2d(x2.double(), wr.double())
        segs.append(K.Seg(K.View.full(_nhwc(x2).cuda()), [(0, 0)], kbase=9 * Ci))
        wp = torch.cat([wp, wr.reshape(Co, Cr)], 1)
        # the residual input's per-image bound (the engine takes GN1's Samuelson bound; any bound >= max |x|)
        xb = x2.abs().reshape(B, -1).amax(1).cuda() * 1.5
    wp = wp.contiguous().cuda()
    e = K.f16x3_a_exp(float(gamma.abs().max()), float(beta.abs().max()), H * W * Ci // 8)
    tcu = temb.cuda()
    outs = {}
    for mode in ('wino', 'f16x3'):
        out = torch.empty((B, H, W, Co), device='cuda')
        kw = dict(Hm=H, Wm=W, a_exp=e, a_bound=xb, temb=tcu, temb_ld=Co + 8)
        if mode == 'wino':
            # (the 64-channel form with a residual is supported by the kernel but routed to the direct
            # one by the engine: wino_eligible says no)
            assert K.wino_eligible(segs, Co, H, W) == (not (Co <= 64 and Cr))
            K.conv3x3_wino(segs, K.pack_wino(wp, Ci, Cr), b.cuda(), K.View.full(out), **kw)
        else:
            K.conv3x3_f16x3(segs, K.pack_f16x3(wp, Ci, Cr, res_f16=bool(Cr)), b.cuda(), K.View.full(out), **kw)
        torch.cuda.synchronize()
        outs[mode] = _nchw(out.cpu()).double()
    assert torch.isfinite(outs['wino']).all()
    ew, ed = rel_l2(outs['wino'], ref), rel_l2(outs['f16x3'], ref)
    assert ew < 1e-5 and ew <= 4 * ed + 2e-7, (ew, ed)


@pytest.mark.gpu
@pytest.mark.parametrize('sw', [8, 32])
def test_conv3x3_wino_epilogue_res_absmax_gn_partials(sw):
    """Epilogue residual view (out = conv + res), per-image absmax and GroupNorm tile partials of the
    Winograd kernel against the values it stored (partials vs a stats pass over the output)."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(43)
    B, H, W, Ci, Co = 2, 16, 32, 64, 8 * sw if sw >= 16 else 128
    x = (torch.randn((B, H, W, Ci), generator=g) * 2 + 3).cuda()
    sc = (1 + 0.2 * torch.randn((B, Ci), generator=g)).cuda()
    sh = (0.2 * torch.randn((B, Ci), generator=g)).cuda()
    w = (torch.randn((Co, 9 * Ci), generator=g) / 24).cuda()
    bias = (torch.randn(Co, generator=g) + 5).cuda()
    r = torch.randn((B, H, W, Co), generator=g).cuda()
    seg = [K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True)]
    wp = K.pack_wino(w, Ci)
    y0 = torch.empty((B, H, W, Co), device='cuda')
    K.conv3x3_wino(seg, wp, bias, K.View.full(y0), Hm=H, Wm=W, a_exp=6)
    y = torch.empty((B, H, W, Co), device='cuda')
    gp = K.GnPart.attach(y, sw)
    amax = torch.zeros(B, device='cuda')
    K.conv3x3_wino(seg, wp, bias, K.View.full(y), Hm=H, Wm=W, a_exp=6, res=K.View.full(r), absmax=amax, gn=gp)
    torch.cuda.synchronize()
    assert torch.equal(y, y0 + r)
    assert torch.equal(amax, y.abs().amax((1, 2, 3)))
    gamma, beta = (1 + torch.randn(Co, generator=g)).cuda(), torch.randn(Co, generator=g).cuda()
    a1 = K.gn_affine(K.View.full(y), gamma, beta, bound=True, part=gp)
    a0 = K.gn_affine(K.View.full(y), gamma, beta, bound=True)
    for u, v in zip(a1, a0):  # (shift = beta - mean * scale cancels to ~0 for some channels: atol of the
        # output magnitude (~5) x 2e-7)
        assert torch.allclose(u, v, rtol=2e-6, atol=1e-6), (u - v).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize('N,C0,C1', [(128, 32, 0), (64, 48, 32), (192, 16, 64), (256, 128, 128)])
def test_pack_wino_device_bit_identical_to_cpu_definition(N, C0, C1):
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(11)
    w = torch.randn((N, 9 * C0 + C1), generator=g) * torch.rand((N, 1), generator=g) * 3
    w[0] = 0.0  # an all-zero channel: scale 2^0
    w[1, 0] = 2.0**-3  # a channel whose max is an exact power of two
    w[1, 1:] = 0.0
    cpu = K.pack_wino(w, C0, C1, device=False)
    dev = K.pack_wino(w.cuda(), C0, C1, device=True)
    torch.cuda.synchronize()
    assert torch.equal(dev.wsinv.cpu(), cpu.wsinv)
    dd, cd = dev.data.cpu(), cpu.data
    bad = (dd != cd).nonzero()
    assert bad.numel() == 0, (len(bad), bad[:4].tolist(), dd[tuple(bad[:4].t())].tolist(),
                              cd[tuple(bad[:4].t())].tolist())


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Ci,Co', [(2, 16, 32, 128, 64), (1, 8, 16, 48, 128), (2, 32, 16, 64, 64)])
def test_conv3x3_wino_raw_segment_vs_float64(B, H, W, Ci, Co):
    """One raw segment under its per-image bound (the training data gradients: dY (*) W flipped), images
    of different scale."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(47)
    x = torch.randn((B, Ci, H, W), generator=g) * 3
    x[0] *= 1e-3
    w = torch.randn((Co, Ci, 3, 3), generator=g) / (Ci * 9)**0.5
    ref = F.conv2d(x.double(), w.double(), padding=1)
    xn = _nhwc(x).cuda()
    bound = xn.abs().reshape(B, -1).amax(1).contiguous()
    segs = [K.Seg(K.View.full(xn), TAPS3)]
    assert K.wino_eligible(segs, Co, H, W)
    outs = {}
    for mode in ('wino', 'f16x3'):
        out = torch.empty((B, H, W, Co), device='cuda')
        if mode == 'wino':
            K.conv3x3_wino(segs, K.pack_wino(_pack(w).cuda(), Ci), None, K.View.full(out), Hm=H, Wm=W, a_exp=60,
                           a_bound=bound)
        else:
            K.conv3x3_f16x3(segs, K.pack_f16x3(_pack(w).cuda(), Ci), None, K.View.full(out), Hm=H, Wm=W, a_exp=60,
                            a_bound=bound)
        torch.cuda.synchronize()
        outs[mode] = _nchw(out.cpu()).double()
    for b in range(B):  # per image (their scales differ by 1e3)
        ew, ed = rel_l2(outs['wino'][b], ref[b]), rel_l2(outs['f16x3'][b], ref[b])
        assert ew < 1e-5 and ew <= 4 * ed + 2e-7, (b, ew, ed)


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Ci,Co,Cr', [(2, 16, 32, 64, 128, 0), (1, 32, 16, 48, 256, 48), (1, 16, 16, 32, 128, 96),
                                            (2, 32, 32, 128, 128, 128), (2, 16, 16, 64, 256, 0), (1, 8, 16, 32, 512, 512),
                                            (3, 8, 32, 64, 768, 0), (2, 16, 16, 256, 128, 256), (2, 16, 48, 32, 64, 0),
                                            (1, 32, 32, 64, 64, 64), (1, 8, 48, 64, 512, 0), (2, 8, 96, 32, 256, 64),
                                            (1, 16, 80, 32, 128, 0)])
def test_conv3x3_wino_presplit_bit_identical(B, H, W, Ci, Co, Cr):
    """The pre-split form (wc_wino_vsplit_f16x3 once per input, then wc_conv3x3_wino_f16x3_vp copying the
    halo planes by LDS-DMA) against the in-conv prologue: bit-identical output, absmax and GroupNorm
    partials (the same arithmetic in a separate pass); 64- and 128-channel tiles, residual interleaved
    and as a tail, per-image residual exponents.  N % 256 == 0: also the 8-wave 256-channel form
    (wc_conv3x3_wino_f16x3_vp8, kernels.wino_vp_wide)."""
    from weatherconverter_amd import kernels as K
    _compare_forms(B, H, W, Ci, Co, Cr, False, lambda K, m: K.set_wino_vsplit(1 if m else 0),
                   lambda K, v: K.set_wino_vsplit(v))
    if Co % 256 == 0:
        with K.wino_vp_wide():
            names = _compare_forms(B, H, W, Ci, Co, Cr, False, lambda K, m: K.set_wino_vsplit(1 if m else 0),
                                   lambda K, v: K.set_wino_vsplit(v))
        assert names[1].startswith('conv3x3_wino_kernel<8, 256, 3'), names


@pytest.mark.gpu
@pytest.mark.parametrize('line', ['single16', 'bf16'])
@pytest.mark.parametrize('B,H,W,Ci,Co,Cr', [(2, 16, 32, 64, 128, 0), (1, 32, 16, 48, 256, 48), (1, 8, 16, 32, 512, 512),
                                            (2, 8, 96, 32, 256, 64), (1, 16, 80, 32, 128, 0)])
def test_conv3x3_wino_presplit_bit_identical_single_piece_lines(line, B, H, W, Ci, Co, Cr):
    """The single-piece training builds store only the high piece's 8 planes per chunk (their low piece is
    zero) and the conv copies only those: still bit-identical to the in-conv prologue of the same build."""
    from weatherconverter_amd import _native
    with _native.variant(line):
        _compare_forms(B, H, W, Ci, Co, Cr, False, lambda K, m: K.set_wino_vsplit(1 if m else 0),
                       lambda K, v: K.set_wino_vsplit(v))
        n = ctypes.c_int64()
        _native.call('wc_wino_vsplit_bytes', B, Ci, H, W, ctypes.byref(n))
        assert n.value == B * (Ci // 16) * 8 * H * (W // 2) * 16


def _compare_forms(B, H, W, Ci, Co, Cr, raw, select, restore):
    """One conv under select(K, 0) and under select(K, 1): outputs, absmax and GN partials bit-identical;
    restore(K, v) puts back the setting select(K, 0) returned."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(53)
    x = (torch.randn((B, H, W, Ci), generator=g) * 2 + 1).cuda()
    w = (torch.randn((Co, 9 * Ci + Cr), generator=g) / (9 * Ci)**0.5).cuda()
    bias = torch.randn(Co, generator=g).cuda()
    temb = torch.randn((B, Co), generator=g).cuda()
    if raw:
        segs = [K.Seg(K.View.full(x), TAPS3)]
        bound = x.abs().reshape(B, -1).amax(1).contiguous()
        kw = dict(a_exp=60, a_bound=bound)
    else:
        sc = (1 + 0.2 * torch.randn((B, Ci), generator=g)).cuda()
        sh = (0.2 * torch.randn((B, Ci), generator=g)).cuda()
        segs = [K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True)]
        kw = dict(a_exp=6, temb=temb, temb_ld=Co)
        if Cr:
            xr = torch.randn((B, H, W, Cr), generator=g).cuda()
            segs.append(K.Seg(K.View.full(xr), [(0, 0)], kbase=9 * Ci))
            kw['a_bound'] = xr.abs().reshape(B, -1).amax(1).contiguous() * 1.5
    wp = K.pack_wino(w, Ci, Cr)
    res, names = {}, {}
    prev = select(K, 0)
    try:
        for mode in (0, 1):
            select(K, mode)
            y = torch.empty((B, H, W, Co), device='cuda')
            gp = K.GnPart.attach(y, 16)
            amax = torch.zeros(B, device='cuda')
            K.conv3x3_wino(segs, wp, None if raw else bias, K.View.full(y), Hm=H, Wm=W, absmax=amax, gn=gp, **kw)
            names[mode] = K._native.last_kernel_name()
            torch.cuda.synchronize()
            res[mode] = (y.cpu(), amax.cpu(), gp.part.cpu())
    finally:
        restore(K, prev)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b), ((a - b).abs().max(), names)
    return names


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Cg,Co', [(2, 16, 32, 128, 128), (2, 32, 16, 64, 64), (1, 8, 48, 256, 192),
                                         (3, 16, 16, 64, 128)])
def test_dgrad_epilogue_gn_backward_sums(B, H, W, Cg, Co):
    """The training data-gradient conv (raw segment under the per-image bound) forming the GroupNorm+SiLU
    backward's sums of what it writes (wc_conv3x3_wino_f16x3_gnb) instead of a wc_gn_bwd_reduce pass
    over dz: the written dz bit-identical to the plain conv's, and gn_backward's dx, dgamma, dbeta and
    closed-form dx sums equal to the reduce path's to fp32 summation order (rel-L2 <= 1e-6); 64- and
    128-channel tiles (one and two wave rows per tile), several output-channel tiles."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(61)
    gy = (torch.randn((B, H, W, Cg), generator=g) * 1e-2).cuda()
    w = (torch.randn((Co, 9 * Cg), generator=g) / (9 * Cg)**0.5).cuda()
    x = (torch.randn((B, H, W, Co), generator=g) * 2 + 0.5).cuda()
    sc0 = (torch.rand((B, Co), generator=g) + 0.5).cuda()
    sh0 = (torch.randn((B, Co), generator=g) * 0.3).cuda()
    ga = (torch.rand(Co, generator=g) + 0.5).cuda()
    be = (torch.randn(Co, generator=g) * 0.1).cuda()
    bound = gy.abs().reshape(B, -1).amax(1).contiguous()
    segs = [K.Seg(K.View.full(gy), TAPS3)]
    assert K.wino_eligible(segs, Co, H, W)
    wp = K.pack_wino(w, Cg)
    xv = K.View.full(x)
    res = {}
    for mode in ('reduce', 'epilogue'):
        dz = torch.empty((B, H, W, Co), device='cuda')
        pre = K.GnbSums.make(xv, sc0, sh0, ga, be, True, dx_sums=True) if mode == 'epilogue' else None
        assert mode == 'reduce' or pre is not None
        K.conv3x3_wino(segs, wp, None, K.View.full(dz), Hm=H, Wm=W, a_exp=60, a_bound=bound, gnb=pre)
        dx = torch.empty((B, H, W, Co), device='cuda')
        dgam, dbet = torch.zeros(Co, device='cuda'), torch.zeros(Co, device='cuda')
        dsum = K.gn_backward(K.View.full(dz), xv, sc0, sh0, ga, be, True, K.View.full(dx), dgamma=dgam, dbeta=dbet,
                             accumulate=False, dx_sums=True, pre=pre)
        torch.cuda.synchronize()
        res[mode] = [t.cpu() for t in (dz, dx, dgam, dbet, dsum[..., 0])]
    assert torch.equal(res['reduce'][0], res['epilogue'][0])  # the conv's output is unchanged
    for a, b in zip(res['reduce'][1:], res['epilogue'][1:]):
        assert rel_l2(b, a) <= 1e-6, rel_l2(b, a)
