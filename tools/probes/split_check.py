"""Check: the graph step with the batch split over 2 / 4 streams returns the same eps as the
unsplit graph (bit-exact: every UNet op is per image)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from weatherconverter_amd import kernels  # noqa: E402
from weatherconverter_amd.diffusion_model.config import model_config  # noqa: E402
from weatherconverter_amd.diffusion_model.models.unet_base import Unet  # noqa: E402
from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep  # noqa: E402
from weatherconverter_amd.synthetic import init_synthetic_  # noqa: E402

dev = torch.device('cuda', 0)
mc = model_config(256)
model = Unet(mc)
init_synthetic_(model, seed=0)
model = model.to(dev).eval()
with torch.no_grad():
    x = kernels.philox_normal((16, 3, 256, 256), dev, 3455, sample0=0, step=1000)
    t = torch.tensor([777], device=dev)
    ref = _GraphStep(model, x, split=1)(x, t).clone()
    for sp in (2, 4):
        got = _GraphStep(model, x, split=sp)(x, t).clone()
        torch.cuda.synchronize()
        print(f'split {sp}: max |diff| = {float((got - ref).abs().max()):.3e}, equal = {bool(torch.equal(got, ref))}',
              flush=True)
