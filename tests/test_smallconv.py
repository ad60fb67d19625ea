"""GPU: the training ends' 3-channel conv kernels (wc_smallconv.hip) against float64 autograd of the
same ops (reference unet_base.py:400 conv_in, :448-449,483-485 norm_out -> SiLU -> conv_out; their
gradients in train_ddpm.py:94-114's loss.backward()).  fp32 VALU kernels: tolerance rel-L2 <= 1e-6
(fp32 accumulation over up to B*H*W = 10^5 pixels), and the weight gradients' fixed-order reduction
must be bitwise repeatable.  Shapes include heights / widths that are not multiples of the 16-pixel
tile or the 64-row band."""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope='module')
def K():
    from weatherconverter_amd import kernels
    kernels._native.load()
    return kernels


SHAPES = [(2, 64, 32, 48), (1, 64, 70, 40), (3, 32, 24, 16), (2, 64, 130, 20)]


@pytest.mark.parametrize('B,C,H,W', SHAPES)
def test_head_dgrad_vs_float64(K, B, C, H, W):
    g = torch.Generator().manual_seed(7)
    gout = torch.randn((B, 3, H, W), generator=g)
    w = torch.randn((3, C, 3, 3), generator=g) / (9 * C)**0.5
    ref = F.conv_transpose2d(gout.double(), w.double(), padding=1)  # d conv2d(act, w, pad 1) / d act
    dz = torch.full((B, H, W, C + 4), float('nan'), device='cuda')  # a view with a wider row stride
    K.head_dgrad(gout.cuda(), w.cuda(), K.View(dz, 0, C))
    got = dz[..., :C].permute(0, 3, 1, 2).cpu()
    assert rel_l2(got, ref) <= TOL
    assert torch.isnan(dz[..., C:]).all()  # nothing written past the view


@pytest.mark.parametrize('B,C,H,W', SHAPES)
def test_head_wgrad_vs_float64(K, B, C, H, W):
    g = torch.Generator().manual_seed(11)
    x = torch.randn((B, H, W, C), generator=g) * 2 + 0.3
    sc = torch.rand((B, C), generator=g) + 0.5
    sh = torch.randn((B, C), generator=g) * 0.2
    gout = torch.randn((B, 3, H, W), generator=g)
    a = x.double() * sc.double()[:, None, None, :] + sh.double()[:, None, None, :]
    act = (a * torch.sigmoid(a)).permute(0, 3, 1, 2)  # the forward's GN affine + SiLU, NCHW
    ref = torch.nn.grad.conv2d_weight(act, (3, C, 3, 3), gout.double(), padding=1)
    dw = torch.zeros((3, C, 3, 3), device='cuda')
    xv = K.View(x.cuda().contiguous(), 0, C)
    args = (xv, sc.cuda(), sh.cuda(), gout.cuda())
    K.head_wgrad(*args, dw)
    assert rel_l2(dw.cpu(), ref) <= TOL
    dw2 = torch.ones_like(dw)
    K.head_wgrad(*args, dw2, accumulate=True)
    assert torch.equal(dw2 - 1, dw) or rel_l2((dw2 - 1).cpu(), dw.cpu()) < 1e-7
    dw3 = torch.empty_like(dw)
    K.head_wgrad(*args, dw3)
    assert torch.equal(dw3, dw)  # fixed-order reduction: bitwise repeatable


@pytest.mark.parametrize('B,C,H,W', SHAPES)
def test_stem_wgrad_vs_float64(K, B, C, H, W):
    g = torch.Generator().manual_seed(13)
    x = torch.rand((B, 3, H, W), generator=g) * 2 - 1
    gy = torch.randn((B, H, W, C), generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (C, 3, 3, 3), gy.double().permute(0, 3, 1, 2), padding=1)
    dw = torch.zeros((C, 3, 3, 3), device='cuda')
    gt = torch.zeros((B, H, W, C + 8), device='cuda')
    gt[..., 4:4 + C] = gy.cuda()
    gv = K.View(gt, 4, C)  # a channel slice of a wider tensor
    K.stem_wgrad(x.cuda(), gv, dw)
    assert rel_l2(dw.cpu(), ref) <= TOL
    dw3 = torch.empty_like(dw)
    K.stem_wgrad(x.cuda(), gv, dw3)
    assert torch.equal(dw3, dw)


def test_smallconv_rejects_bad_shapes(K):
    x = K.View(torch.zeros((1, 16, 16, 48), device='cuda'), 0, 48)
    with pytest.raises(RuntimeError, match='unsupported shape'):
        K.head_wgrad(x, torch.zeros((1, 48), device='cuda'), torch.zeros((1, 48), device='cuda'),
                     torch.zeros((1, 3, 16, 16), device='cuda'), torch.zeros((3, 48, 3, 3), device='cuda'))
