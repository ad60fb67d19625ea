"""The 2D Winograd F(2x2, 3x3) position-major ResBlock conv (csrc/wc_wino2d.hip, kernels.pack_wino2d /
conv3x3_wino2d).

CPU: the weight pack -- the packed fp16 pieces, read back through the kernel's layout, reconstruct the
float64 filter transform U = G g G^T (and the residual columns), and F(2x2, 3x3) evaluated in float64
on them reproduces the direct 3x3 conv.
GPU: the kernel against a float64 direct conv (reference ResBlock convs unet_base.py:87-109, :146-150),
within 4x (+2e-7) of the direct f16x3 kernel's own error and 1e-5, with bias, temb, the fused 1x1
residual under its per-image bound, the epilogue residual view, per-image absmax and GroupNorm tile
partials (against a stats pass over the stored output).
"""
import pytest
import torch
import torch.nn.functional as F

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]
BT = torch.tensor([[1., 0., -1., 0.], [0., 1., 1., 0.], [0., -1., 1., 0.], [0., 1., 0., -1.]], dtype=torch.float64)
AT = torch.tensor([[1., 1., 1., 0.], [0., 1., -1., -1.]], dtype=torch.float64)


def rel_l2(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def _pack(w):  # [Co][Ci][3][3] -> [Co][9 * Ci], K = (ky * 3 + kx, c) (engine.pack_conv)
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


def _unpack(wp, N, C0, C1):
    """Invert pack_wino2d's layout: (U [N][16][C0], residual [N][C1]) in float64 from the pieces."""
    BN, T = wp.BN, wp.data.shape[0]
    d = wp.data.cpu()
    n0 = 16 * C0 * 2 * BN
    seg0 = d[:, :n0].reshape(T, 16, C0 // 16, 2, 2, BN, 8).view(torch.float16).double()
    u = seg0[:, :, :, 0] + seg0[:, :, :, 1]  # [T][16][nc][kh][BN][8]
    u = u.permute(0, 4, 1, 2, 3, 5).reshape(T * BN, 16, C0)
    ws = wp.wsinv.cpu().double()
    U = u[:N] * ws[:N, None, None]
    R = None
    if C1:
        seg1 = d[:, n0:].reshape(T, C1 // 16, 2, 2, BN, 8).view(torch.float16).double()
        r = (seg1[:, :, 0] + seg1[:, :, 1]).permute(0, 3, 1, 2, 4).reshape(T * BN, C1)
        R = r[:N] * ws[:N, None]
    return U, R


def _wino2d_f64(a, U):
    """F(2x2, 3x3) in float64: a [B][C][H][W], U [N][16][C] -> [B][N][H][W]."""
    B, C, H, W = a.shape
    ap = F.pad(a, (1, 1, 1, 1))
    d = torch.stack([torch.stack([ap[:, :, i:i + H:2, j:j + W:2] for j in range(4)], -1) for i in range(4)], -2)
    V = torch.einsum('pi,bcyxij,qj->bpqcyx', BT, d, BT).reshape(B, 16, C, H // 2, W // 2)
    M = torch.einsum('bPcyx,nPc->bnPyx', V, U).reshape(B, U.shape[0], 4, 4, H // 2, W // 2)
    Y = torch.einsum('ip,bnpqyx,jq->bnyixj', AT, M, AT)
    return Y.reshape(B, U.shape[0], H, W)


@pytest.mark.parametrize('N,C0,C1', [(512, 32, 0), (600, 64, 32), (128, 96, 64)])
def test_pack_wino2d_reconstructs_the_filter_transform(N, C0, C1):
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(7)
    w = torch.randn((N, 9 * C0 + C1), generator=g) * torch.rand((N, 1), generator=g) * 3
    wp = K.pack_wino2d(w, C0, C1)
    assert wp.order == 'wino2d' and wp.data.numel() * 2 == wp.data.shape[0] * (16 * C0 // 16 + C1 // 16) * 128 * 64
    U, R = _unpack(wp, N, C0, C1)
    Gm = torch.tensor(K._G2, dtype=torch.float64)
    Uref = torch.einsum('pk,nklc,ql->npqc', Gm, w[:, :9 * C0].double().reshape(N, 3, 3, C0), Gm).reshape(N, 16, C0)
    assert rel_l2(U, Uref) < 3e-7
    if C1:
        assert rel_l2(R, w[:, 9 * C0:].double()) < 3e-7


def test_wino2d_algebra_equals_direct_conv():
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(3)
    a = torch.randn((2, 8, 6, 10), generator=g, dtype=torch.float64)
    w = torch.randn((5, 8, 3, 3), generator=g, dtype=torch.float64)
    Gm = torch.tensor(K._G2, dtype=torch.float64)
    U = torch.einsum('pk,nckl,ql->npqc', Gm, w, Gm).reshape(5, 16, 8)
    assert rel_l2(_wino2d_f64(a, U), F.conv2d(a, w, padding=1)) < 1e-14


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


CASES = [
    # B, H, W, Ci, Co, Cr, gamma scale, outlier
    (2, 16, 32, 64, 512, 0, 1.0, False),     # 4 N tiles
    (1, 32, 32, 96, 640, 64, 1.0, False),    # residual, N not a multiple of 128, K-steps padded
    (2, 16, 16, 32, 512, 128, 1.0, False),   # residual chunks > 3x3 chunks
    (1, 16, 16, 64, 512, 32, 20.0, True),    # Samuelson-extreme outlier + large gamma
    (1, 64, 16, 256, 768, 256, 1.0, False),  # the UNet's 32^2 / 64^2 widths
]


@pytest.mark.gpu
@pytest.mark.parametrize('B,H,W,Ci,Co,Cr,gs,outlier', CASES)
def test_conv3x3_wino2d_vs_float64(B, H, W, Ci, Co, Cr, gs, outlier):
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(41)
    h = torch.randn((B, Ci, H, W), generator=g) * 3 + 0.7
    if outlier:
        h.zero_()
        h[:, ::Ci // 8, 0, 0] = 1e4
    gamma = gs * (1 + 0.3 * torch.randn(Ci, generator=g))
    beta = 0.5 * torch.randn(Ci, generator=g)
    sc, sh = _gn_affine(h, gamma, beta)
    x2 = torch.randn((B, max(Cr, 32), H, W), generator=g) * 5
    w = torch.randn((Co, Ci, 3, 3), generator=g) / (Ci * 9)**0.5
    wr = torch.randn((Co, max(Cr, 32), 1, 1), generator=g) / max(Cr, 32)**0.5
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
        xb = x2.abs().reshape(B, -1).amax(1).cuda() * 1.5
    wp = wp.contiguous().cuda()
    e = K.f16x3_a_exp(float(gamma.abs().max()), float(beta.abs().max()), H * W * Ci // 8)
    tcu = temb.cuda()
    assert K.wino2d_eligible(segs, Co, H, W)
    outs = {}
    for mode in ('wino2d', 'f16x3'):
        out = torch.empty((B, H, W, Co), device='cuda')
        kw = dict(Hm=H, Wm=W, a_exp=e, a_bound=xb, temb=tcu, temb_ld=Co + 8)
        if mode == 'wino2d':
            K.conv3x3_wino2d(segs, K.pack_wino2d(wp, Ci, Cr), b.cuda(), K.View.full(out), **kw)
            assert K._native.last_kernel_name() == f'conv3x3_wino2d_kernel<{"true" if Cr else "false"}>'
        else:
            K.conv3x3_f16x3(segs, K.pack_f16x3(wp, Ci, Cr, res_f16=bool(Cr)), b.cuda(), K.View.full(out), **kw)
        torch.cuda.synchronize()
        outs[mode] = _nchw(out.cpu()).double()
    assert torch.isfinite(outs['wino2d']).all()
    ew, ed = rel_l2(outs['wino2d'], ref), rel_l2(outs['f16x3'], ref)
    assert ew < 1e-5 and ew <= 4 * ed + 2e-7, (ew, ed)


@pytest.mark.gpu
@pytest.mark.parametrize('sw', [8, 32])
def test_conv3x3_wino2d_epilogue_res_absmax_gn_partials(sw):
    """Epilogue residual view, per-image absmax and GroupNorm tile partials of the 2D kernel against the
    values it stored (partials vs a stats pass over the output)."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(43)
    B, H, W, Ci, Co = 2, 32, 48, 64, 512
    x = (torch.randn((B, H, W, Ci), generator=g) * 2 + 3).cuda()
    sc = (1 + 0.2 * torch.randn((B, Ci), generator=g)).cuda()
    sh = (0.2 * torch.randn((B, Ci), generator=g)).cuda()
    w = (torch.randn((Co, 9 * Ci), generator=g) / 24).cuda()
    bias = (torch.randn(Co, generator=g) + 5).cuda()
    r = torch.randn((B, H, W, Co), generator=g).cuda()
    seg = [K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True)]
    wp = K.pack_wino2d(w, Ci)
    y0 = torch.empty((B, H, W, Co), device='cuda')
    K.conv3x3_wino2d(seg, wp, bias, K.View.full(y0), Hm=H, Wm=W, a_exp=6)
    y = torch.empty((B, H, W, Co), device='cuda')
    gp = K.GnPart.attach(y, sw)
    amax = torch.zeros(B, device='cuda')
    K.conv3x3_wino2d(seg, wp, bias, K.View.full(y), Hm=H, Wm=W, a_exp=6, res=K.View.full(r), absmax=amax, gn=gp)
    torch.cuda.synchronize()
    assert torch.equal(y, y0 + r)
    assert torch.equal(amax, y.abs().amax((1, 2, 3)))
    gamma, beta = (1 + torch.randn(Co, generator=g)).cuda(), torch.randn(Co, generator=g).cuda()
    a1 = K.gn_affine(K.View.full(y), gamma, beta, bound=True, part=gp)
    a0 = K.gn_affine(K.View.full(y), gamma, beta, bound=True)
    for u, v in zip(a1, a0):
        assert torch.allclose(u, v, rtol=2e-6, atol=1e-6), (u - v).abs().max()


@pytest.mark.gpu
def test_conv3x3_wino2d_deterministic_and_view_bounds():
    """Two launches give the same bits; the output view's neighbouring channels are not written."""
    from weatherconverter_amd import kernels as K
    g = torch.Generator().manual_seed(5)
    B, H, W, Ci, Co, Cr = 2, 16, 32, 64, 512, 64
    x = (torch.randn((B, H, W, Ci), generator=g) * 2).cuda()
    xr = torch.randn((B, H, W, Cr), generator=g).cuda()
    sc = (1 + 0.2 * torch.randn((B, Ci), generator=g)).cuda()
    sh = (0.2 * torch.randn((B, Ci), generator=g)).cuda()
    w = (torch.randn((Co, 9 * Ci + Cr), generator=g) / 24).cuda()
    segs = [K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True), K.Seg(K.View.full(xr), [(0, 0)], kbase=9 * Ci)]
    wp = K.pack_wino2d(w, Ci, Cr)
    bound = xr.abs().reshape(B, -1).amax(1).contiguous()
    outs = []
    for _ in range(2):
        big = torch.full((B, H, W, Co + 64), 7.0, device='cuda')
        K.conv3x3_wino2d(segs, wp, None, K.View(big, 32, Co), Hm=H, Wm=W, a_exp=6, a_bound=bound)
        torch.cuda.synchronize()
        outs.append(big.cpu())
    assert torch.equal(outs[0], outs[1])
    assert bool((outs[0][..., :32] == 7.0).all()) and bool((outs[0][..., 32 + Co:] == 7.0).all())
