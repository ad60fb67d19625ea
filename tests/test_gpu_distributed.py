"""GPU, world_size 2 over gloo with both ranks on cuda:0: the config-5 product path.

``sample_sharded`` (diffusion_model/distributed.py) runs the HIP sample loop on each rank's block of
global samples and gathers x0 (staged through host memory under gloo).  The gathered batch must be
BIT-equal to one rank sampling the whole batch: noise is keyed per global sample (Philox, or the
reference CPU stream sliced per rank) and every kernel's reduction order is independent of the batch
(GroupNorm splits per image, wc_gn.hip splits_for).  SURVEY.md §8(e).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T_STEPS = 12


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _tiny(cfg='tiny'):
    """The tiny test config, or ('256') config 5's per-rank model: the BASELINE 256-px architecture."""
    import json
    from conftest import GOLDEN
    from weatherconverter_amd.diffusion_model.config import ModelConfig, model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.synthetic import init_synthetic_
    if cfg == '256':
        mc = model_config(256)
    else:
        man = json.load(open(os.path.join(GOLDEN, 'manifest.json')))
        mc = ModelConfig(**man['tiny']['config'])
    net = Unet(mc)
    init_synthetic_(net, seed=0)
    return mc, net.cuda().eval()


def _golden_row_err(net, mc, B, row):
    """rel-L2 of row `row` of a B-image forward (the other rows seeded noise) against the reference's
    256-px forward of the golden input at t = 611."""
    from conftest import GOLDEN
    from weatherconverter_amd.synthetic import synthetic_images
    gd = np.load(os.path.join(GOLDEN, 'unet_256.npz'))
    x = torch.randn((B, mc.im_channels, mc.im_size, mc.im_size), generator=torch.Generator().manual_seed(5))
    x[row] = synthetic_images((1, mc.im_channels, mc.im_size, mc.im_size), seed=301)[0]
    with torch.no_grad():
        y = net(x.cuda(), torch.full((B, ), 611, dtype=torch.long).cuda())[row].double().cpu()
    ref = torch.from_numpy(gd['y'][0]).double()
    return float((y - ref).norm() / ref.norm())


def _worker(rank, world, port, total, noise, q, cfg='tiny', steps=T_STEPS):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from weatherconverter_amd.diffusion_model.distributed import sample_sharded
        from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
        torch.cuda.set_device(0)
        mc, net = _tiny(cfg)
        s = LinearNoiseScheduler(steps, 0.0001, 0.02)
        x0 = sample_sharded(net, s, total, mc.im_channels, mc.im_size, noise=noise, seed=77, graph=True)
        assert x0.is_cuda and x0.shape[0] == total
        eps_err = None
        if cfg == '256':  # the rank's model is the BASELINE UNet: a 16-image forward whose row r holds the
            # 256-px golden input at the golden's t (tests/golden/unet_256.npz, reference forward)
            eps_err = _golden_row_err(net, mc, total // world, rank % (total // world))
        q.put((rank, (x0.cpu().numpy().copy(), eps_err)))
    except BaseException as e:  # surface the failure to the parent instead of hanging its q.get
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('total,noise,cfg,steps', [(4, 'philox', 'tiny', T_STEPS), (5, 'philox', 'tiny', T_STEPS),
                                                   (4, 'torch_cpu', 'tiny', T_STEPS), (1, 'philox', 'tiny', T_STEPS),
                                                   (2, 'philox', '256', 3), (32, 'philox', '256', 2)])
def test_sample_sharded_world2_equals_single_rank(total, noise, cfg, steps):
    """cfg '256': config 5's per-rank workload (the 256-px BASELINE UNet) through sample_sharded ->
    gather_samples: 2 images over 2 ranks at T=3, and config 5's full per-rank batch, 16 images on each
    of 2 ranks at T=2 (BASELINE config 5: 128 images over 8 GPUs); each rank's model also reproduces the
    reference's 256-px forward in one row of a 16-image batch."""
    from weatherconverter_amd.diffusion_model.sample_ddpm import sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, noise, q, cfg, steps)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240 if cfg == '256' else 100) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(res[r], str), f'rank {r}: {res[r]}'
        assert procs[r].exitcode == 0
    mc, net = _tiny(cfg)
    s = LinearNoiseScheduler(steps, 0.0001, 0.02)
    ref = sample_tensor(net, s, total, mc.im_channels, mc.im_size, noise=noise, seed=77, graph=True).cpu()
    for r in range(world):
        got = torch.from_numpy(res[r][0])
        assert torch.isfinite(got).all()
        assert torch.equal(got, ref), f'rank {r}: max |diff| {float((got - ref).abs().max())}'
        if cfg == '256':
            assert res[r][1] < 1e-5, (r, res[r][1])
    assert np.array_equal(res[0][0], res[1][0])
