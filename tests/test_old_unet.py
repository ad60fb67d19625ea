"""Old 128-px UNet + sample_integrated loop vs reference goldens.

Tolerances: forward rel-L2 <= 1e-5, T=10 trajectory x0 rel-L2 <= 1e-4 (as for the main UNet)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2
from weatherconverter_amd.diffusion_model.models.old_modules import UNet
from weatherconverter_amd.synthetic import init_synthetic_, state_dict_digest, synthetic_images

G = np.load(os.path.join(GOLDEN, 'old_unet.npz'))


def test_old_unet_state_dict_layout():
    man = json.load(open(os.path.join(GOLDEN, 'old_manifest.json')))
    assert [[k, list(v.shape)] for k, v in UNet().state_dict().items()] == man


def _net():
    net = UNet()
    init_synthetic_(net, seed=0)
    assert state_dict_digest(net.state_dict()) == str(G['digest'])
    return net.cuda().eval()


@pytest.mark.gpu
def test_old_unet_forward():
    net = _net()
    with torch.no_grad():
        y = net(synthetic_images((1, 3, 128, 128), seed=501).cuda(), torch.tensor([[[[0.2860]]]]).cuda())
    assert rel_l2(y.cpu(), G['y']) < 1e-5


@pytest.mark.gpu
def test_sample_integrated_trajectory():
    from weatherconverter_amd.diffusion_model.sample_integrated import postprocess, sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    net = _net()
    s = LinearNoiseScheduler(10, 0.0001, 0.02)
    x0 = sample_tensor(net, s, 1, seed=3455)
    assert rel_l2(x0.cpu(), G['traj_x0']) < 1e-4
    img = postprocess(x0)
    assert img.dtype == torch.uint8 and img.shape == (1, 3, 128, 128)
