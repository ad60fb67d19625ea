"""GPU: whole-UNet and sampling parity of the HIP path against golden vectors from the reference.

Tolerances (written here): UNet forward rel-L2 <= 1e-5; trajectory x0 rel-L2 <= 1e-4.
Weights come from the keyed synthetic recipe; the digest check proves they equal the golden run's.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu
MANIFEST = json.load(open(os.path.join(GOLDEN, 'manifest.json')))


def _model(name, seed=0, precision=None):
    from weatherconverter_amd.diffusion_model.config import ModelConfig
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.synthetic import init_synthetic_
    mc = ModelConfig(**MANIFEST[name]['config'])
    net = Unet(mc)
    init_synthetic_(net, seed=seed)
    if precision is not None:
        net.set_conv_precision(precision)
    return mc, net.cuda().eval()


def _x(mc, B, seed):
    from weatherconverter_amd.synthetic import synthetic_images
    return synthetic_images((B, mc.im_channels, mc.im_size, mc.im_size), seed=seed)


def test_unet_tiny_shared_and_per_sample_t():
    from weatherconverter_amd.synthetic import state_dict_digest
    mc, net = _model('tiny')
    g = np.load(os.path.join(GOLDEN, 'unet_tiny.npz'))
    assert state_dict_digest(net.state_dict()) == str(g['digest'])
    with torch.no_grad():
        y1 = net(_x(mc, 2, 101).cuda(), torch.tensor([7]).cuda())
        y2 = net(_x(mc, 2, 102).cuda(), torch.tensor([3, 900]).cuda())
    assert rel_l2(y1.cpu(), g['y_shared_t']) < 1e-5
    assert rel_l2(y2.cpu(), g['y_batch_t']) < 1e-5


@pytest.mark.parametrize('precision', ['f16x3', 'bf16x6', 'fp32'])
def test_unet_64_config1_model(precision):
    mc, net = _model('default_64', precision=precision)
    g = np.load(os.path.join(GOLDEN, 'unet_64.npz'))
    with torch.no_grad():
        y = net(_x(mc, 2, 201).cuda(), torch.tensor([37]).cuda())
    assert rel_l2(y.cpu(), g['y']) < 1e-5


@pytest.mark.parametrize('precision', ['f16x3', 'bf16x6', 'fp32'])
def test_unet_256_baseline_architecture(precision):
    mc, net = _model('default_256', precision=precision)
    g = np.load(os.path.join(GOLDEN, 'unet_256.npz'))
    with torch.no_grad():
        y = net(_x(mc, 1, 301).cuda(), torch.tensor([611]).cuda())
    assert rel_l2(y.cpu(), g['y']) < 1e-5


def test_unet_256_batch16_rows_match_singletons():
    """Full BASELINE batch (B=16 at 256 px): each row equals the same sample run alone."""
    mc, net = _model('default_256')
    x = _x(mc, 16, 301).cuda()
    with torch.no_grad():
        y = net(x, torch.tensor([611]).cuda())
        y0 = net(x[:1].contiguous(), torch.tensor([611]).cuda())
        y9 = net(x[9:10].contiguous(), torch.tensor([611]).cuda())
    assert torch.isfinite(y).all()
    g = np.load(os.path.join(GOLDEN, 'unet_256.npz'))
    assert rel_l2(y[:1].cpu(), g['y']) < 1e-5
    assert rel_l2(y[:1], y0) < 1e-5 and rel_l2(y[9:10], y9) < 1e-5


def test_trajectory_config1_reference_rng():
    """Config 1 end to end: 64 px, B=2, T=50, reference RNG stream (seed 3455) -> golden x0."""
    from weatherconverter_amd.diffusion_model.sample_ddpm import sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    mc, net = _model('default_64')
    g = np.load(os.path.join(GOLDEN, 'traj_64_T50.npz'))
    s = LinearNoiseScheduler(50, 0.0001, 0.02)
    x0 = sample_tensor(net, s, 2, 3, 64, noise='torch_cpu', seed=int(g['seed']))
    assert rel_l2(x0.cpu(), g['x0']) < 1e-4


def test_graph_replay_matches_eager():
    from weatherconverter_amd.diffusion_model.sample_ddpm import sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    mc, net = _model('tiny')
    s = LinearNoiseScheduler(20, 0.0001, 0.02)
    a = sample_tensor(net, s, 2, 3, 32, noise='philox', seed=9)
    b = sample_tensor(net, s, 2, 3, 32, noise='philox', seed=9, graph=True)
    assert torch.equal(a, b)


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_graph_stream_groups_equal_unsplit(precision):
    # the graph step with the batch as 2 / 4 concurrent image groups (bench --split) is bit-exact
    from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep
    mc, net = _model('default_64', precision=precision)
    x = _x(mc, 8, seed=5).cuda()
    t = torch.tensor([321], device='cuda')
    with torch.no_grad():
        ref = _GraphStep(net, x, split=1)(x, t).clone()
        for sp in (2, 4):
            step = _GraphStep(net, x, split=sp)
            assert step.split == sp
            assert torch.equal(step(x, t).clone(), ref)


def test_sharded_sampling_equals_single_rank():
    """Batch sharding with per-sample keyed noise: rows [2, 4) of a B=4 run == a B=2 run at sample0=2."""
    from weatherconverter_amd.diffusion_model.sample_ddpm import sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    mc, net = _model('tiny')
    s = LinearNoiseScheduler(10, 0.0001, 0.02)
    full = sample_tensor(net, s, 4, 3, 32, noise='philox', seed=21)
    part = sample_tensor(net, s, 2, 3, 32, noise='philox', seed=21, sample0=2, total_batch=4)
    assert rel_l2(full[2:], part) < 1e-6
    fc = sample_tensor(net, s, 4, 3, 32, noise='torch_cpu', seed=22)
    pc = sample_tensor(net, s, 2, 3, 32, noise='torch_cpu', seed=22, sample0=2, total_batch=4)
    assert rel_l2(fc[2:], pc) < 1e-6


def test_reference_rng_stream_isolated_from_callbacks():
    """noise='torch_cpu': a progress callback drawing from the global CPU generator leaves the sample
    unchanged, and the global generator ends where the reference's sequential loop leaves it
    (x_T + T - 1 full-batch draws)."""
    from weatherconverter_amd.diffusion_model.sample_ddpm import sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    mc, net = _model('tiny')
    T = 6
    s = LinearNoiseScheduler(T, 0.0001, 0.02)
    a = sample_tensor(net, s, 2, 3, 32, noise='torch_cpu', seed=23)
    after = torch.randn(3)
    b = sample_tensor(net, s, 2, 3, 32, noise='torch_cpu', seed=23, progress=lambda i: torch.rand(7))
    assert torch.equal(a, b)
    torch.manual_seed(23)
    for _ in range(T):  # x_T and the T - 1 z draws of the reference loop
        torch.randn((2, 3, 32, 32))
    assert torch.equal(torch.randn(3), after)


def test_unet_256_batch_above_descriptor_limit_chunks():
    """B=64 at 256 px puts the level-0 skip buffer at 2 GiB (past one buffer descriptor's 32-bit range):
    the engine runs it as chunks of max_batch (63) images; rows equal singleton runs bit for bit."""
    mc, net = _model('default_256')
    eng_cap = net.engine().max_batch(256, 256)
    x = _x(mc, 64, 303).cuda()
    t = torch.tensor([250]).cuda()
    with torch.no_grad():
        y = net(x, t)
        y0 = net(x[:1].contiguous(), t)
        y63 = net(x[63:].contiguous(), t)
    assert eng_cap == 63
    assert torch.isfinite(y).all()
    assert torch.equal(y[:1], y0) and torch.equal(y[63:], y63)


@pytest.mark.parametrize('precision', ['f16x3', 'bf16x6'])
def test_trajectory_T1000_reference_rng(precision):
    """The full T=1000 schedule (64-px default config, B=1, reference RNG stream seed 3455) in the benched
    split-precision arithmetic: x0 (and x at intermediate checkpoints) within SURVEY §8(c)'s trajectory
    tolerance rel-L2 <= 1e-4 of the reference's fp32 CPU trajectory (tests/golden/traj_64_T1000.npz)."""
    from weatherconverter_amd.diffusion_model.sample_ddpm import sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.synthetic import state_dict_digest
    path = os.path.join(GOLDEN, 'traj_64_T1000.npz')
    g = np.load(path)
    mc, net = _model('default_64', precision=precision)
    assert state_dict_digest(net.state_dict()) == str(g['digest'])
    s = LinearNoiseScheduler(1000, 0.0001, 0.02)
    seen = {}

    def grab(i, x):
        if f'x_after_t{i}' in g.files:
            seen[i] = x.cpu().clone()

    x0 = sample_tensor(net, s, 1, 3, 64, noise='torch_cpu', seed=int(g['seed']), graph=True, progress_x=grab)
    errs = {i: rel_l2(v, g[f'x_after_t{i}']) for i, v in sorted(seen.items(), reverse=True)}
    err = rel_l2(x0.cpu(), g['x0'])
    print(f'{precision}: T=1000 trajectory rel-L2 checkpoints {errs}, x0 {err:.3e}')
    assert len(errs) == 4 and all(e < 1e-4 for e in errs.values()), errs
    assert err < 1e-4
