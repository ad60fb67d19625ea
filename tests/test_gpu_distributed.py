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
        q.put((rank, x0.cpu().numpy().copy()))
    except BaseException as e:  # surface the failure to the parent instead of hanging its q.get
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('total,noise,cfg,steps', [(4, 'philox', 'tiny', T_STEPS), (5, 'philox', 'tiny', T_STEPS),
                                                   (4, 'torch_cpu', 'tiny', T_STEPS), (1, 'philox', 'tiny', T_STEPS),
                                                   (2, 'philox', '256', 3)])
def test_sample_sharded_world2_equals_single_rank(total, noise, cfg, steps):
    """cfg '256': config 5's per-rank workload (the 256-px BASELINE UNet, B=16 per rank in the bench)
    through sample_sharded -> gather_samples at 2 images over 2 ranks, T=3."""
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
        res = dict(q.get(timeout=100) for _ in range(world))
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
        got = torch.from_numpy(res[r])
        assert torch.isfinite(got).all()
        assert torch.equal(got, ref), f'rank {r}: max |diff| {float((got - ref).abs().max())}'
    assert np.array_equal(res[0], res[1])
