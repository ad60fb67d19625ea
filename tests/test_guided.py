"""Guided path: segmenter / SRGAN parity with the reference modules (CPU, the
segmenter stays PyTorch per north_star) and the HIP guidance update + translation loop (GPU)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2
from weatherconverter_amd.seg_model.inference import compute_gradient_magnitude, input_gradient
from weatherconverter_amd.seg_model.network import deeplabv3plus_resnet101
from weatherconverter_amd.srgan_model.models import Generator
from weatherconverter_amd.synthetic import init_synthetic_, state_dict_digest

G = np.load(os.path.join(GOLDEN, 'guided.npz'))
MAN = json.load(open(os.path.join(GOLDEN, 'guided_manifest.json')))


def _seg():
    net = deeplabv3plus_resnet101(num_classes=19, output_stride=16)
    init_synthetic_(net, seed=0)
    return net.eval()


def _srgan():
    net = Generator()
    init_synthetic_(net, seed=0)
    return net.eval()


def test_state_dict_layouts_match_reference():
    assert [[k, list(v.shape)] for k, v in deeplabv3plus_resnet101(19, 16).state_dict().items()] == \
        MAN['deeplabv3plus_resnet101']
    assert [[k, list(v.shape)] for k, v in Generator().state_dict().items()] == MAN['srgan_generator']


def test_segmenter_logits_and_input_gradient_cpu():
    seg = _seg()
    assert state_dict_digest(seg.state_dict()) == str(G['seg_digest'])
    sr, gt = torch.from_numpy(G['sr']), torch.from_numpy(G['gt'])
    g, logits = input_gradient(seg, sr, gt, want_pred=True)
    assert rel_l2(logits, G['logits']) < 1e-6
    assert rel_l2(g, G['grad']) < 1e-5


def test_srgan_forward_cpu():
    gen = _srgan()
    assert state_dict_digest(gen.state_dict()) == str(G['srgan_digest'])
    with torch.no_grad():
        y = gen(torch.from_numpy(G['srgan_in']))
    assert rel_l2(y, G['srgan_out']) < 1e-6


def test_gradient_magnitude_batch_semantics_cpu():
    g = torch.from_numpy(G['grad'])
    m = compute_gradient_magnitude(torch.nn.functional.avg_pool2d(g, 4, 4))
    assert m.shape == (8, 8) and m.dtype == torch.float64
    m2 = compute_gradient_magnitude(torch.cat([g, g]).mean(dim=(2, 3), keepdim=True).expand(2, 3, 8, 8))
    assert m2.shape == (3, 8, 8)  # D4: batch > 1 sums over the batch axis


@pytest.mark.gpu
def test_apply_gsg_gpu_matches_reference():
    from weatherconverter_amd.sgg import apply_gsg
    torch.backends.cudnn.allow_tf32 = False
    seg = _seg().cuda()
    xt = apply_gsg(seg, torch.from_numpy(G['mu']).cuda(), torch.from_numpy(G['sigma']).cuda(),
                   torch.from_numpy(G['sr']).cuda(), torch.from_numpy(G['gt']).cuda(), 60.0)
    assert xt.dtype == torch.float32
    assert rel_l2(xt.cpu(), G['gsg_xt']) < 1e-5


@pytest.mark.gpu
def test_guided_translation_loop_modes():
    """D1: in 'reference' mode the guidance is discarded, so the result equals plain DDPM from the same
    noised start; 'applied' keeps it.  Tiny UNet, SRGAN x4 to 128 px, DeepLab on 128 px."""
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.translation import sample_with_sgg
    from test_gpu_unet import MANIFEST
    from weatherconverter_amd.diffusion_model.config import ModelConfig
    mc = ModelConfig(**MANIFEST['tiny']['config'])
    unet = Unet(mc)
    init_synthetic_(unet)
    unet = unet.cuda().eval()
    sched = LinearNoiseScheduler(1000, 0.0001, 0.02)
    seg, gen = _seg().cuda(), _srgan().cuda()
    g = torch.Generator().manual_seed(3)
    x = torch.rand((1, 3, 32, 32), generator=g) * 2 - 1
    gt = torch.randint(0, 19, (1, 128, 128), generator=g).cuda()
    noise = torch.randn((1, 3, 32, 32), generator=g)
    kw = dict(N=6, t_start=torch.tensor([5]), noise=noise, LAMBDA=1e6, return_latent=True)  # grads are ~1e-6
    torch.manual_seed(9)
    ref, ref_lat = sample_with_sgg(x, unet, sched, seg, gt, gen, mode='reference', **kw)
    torch.manual_seed(9)
    app, app_lat = sample_with_sgg(x, unet, sched, seg, gt, gen, mode='applied', **kw)
    # plain DDPM from the same start and the same CPU noise stream
    torch.manual_seed(9)
    xt = sched.add_noise2(x.cuda(), noise.cuda(), torch.tensor([5]).cuda())
    with torch.no_grad():
        for i in reversed(range(6)):
            eps = unet(xt, torch.tensor([i]).cuda())
            mu, sz, _ = sched.sample_prev_timestep(xt, eps, i)
            xt = mu if i == 0 else (mu + sz)
        plain = gen(xt)
    assert ref.shape == (1, 3, 128, 128) and torch.isfinite(app).all()
    assert rel_l2(ref, plain) < 1e-6 and rel_l2(ref_lat, xt) < 1e-6
    assert rel_l2(app_lat, ref_lat) > 1e-5  # the applied guidance moved the latent (ref vs plain < 1e-6)


@pytest.mark.gpu
def test_srgan_hip_matches_reference_golden():
    """HIP SRGAN (dwconv + fp32-MFMA pointwise with folded BN / PReLU / PixelShuffle / tanh epilogues)
    against the reference generator's output: rel-L2 <= 1e-5."""
    gen = _srgan().cuda()
    y = gen(torch.from_numpy(G['srgan_in']).cuda())
    assert y.shape == (1, 3, 64, 64)
    assert rel_l2(y.cpu(), G['srgan_out']) < 1e-5


@pytest.mark.gpu
def test_srgan_hip_ragged_tiles_prelu_bn_vs_float64():
    """Ragged spatial tiles (B=2, 20x44), PReLU slopes far from 1 and non-trivial BN statistics,
    against the module's own layers in float64."""
    gen = _srgan()
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():
        for m in gen.modules():
            if isinstance(m, torch.nn.PReLU):
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) * 0.5)
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.3)
                m.running_var.copy_(0.5 + torch.rand(m.running_var.shape, generator=g))
    x = torch.rand((2, 3, 20, 44), generator=g)
    ref = gen.double()(x.double()).float()
    y = gen.float().cuda()(x.cuda())
    assert y.shape == (2, 3, 80, 176)
    assert rel_l2(y.cpu(), ref) < 1e-5
