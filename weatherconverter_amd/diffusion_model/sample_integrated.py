"""Drop-in for the reference's ``diffusion_model/sample_integrated.py`` (old-UNet sampling).

Loop (reference ``:52-64``): the model gets ``one_minus_cum_prod[t]`` as a (B,1,1,1) noise level and
the scheduler takes the beta-variance step (``sample_prev_timestep2``).  Both run on HIP kernels.
``postprocess`` (dataset-statistics de-normalisation to uint8, ``:32-37``) and the PNG grid match the
reference; exceptions propagate.
"""
import os
from datetime import datetime
from typing import Optional

import torch

from .config import Config, DiffusionConfig, ModelConfig, TrainingConfig, load_config  # noqa: F401
from .models.old_modules import UNet
from .sample_ddpm import load_scheduler, make_grid, save_png  # noqa: F401
from .scheduler.linear_noise_scheduler import LinearNoiseScheduler


def _device() -> torch.device:
    return torch.device('cuda' if torch.cuda.is_available() else 'cpu')


def postprocess(xt, mean=(0.4865, 0.4998, 0.4323), std=(0.2326, 0.2276, 0.2659)):
    """reference :32-37: x*std + mean -> *255 -> clamp -> uint8 (CPU)."""
    m = torch.tensor(mean, device=xt.device).view(1, -1, 1, 1)
    s = torch.tensor(std, device=xt.device).view(1, -1, 1, 1)
    return ((xt * s + m) * 255).clamp(0, 255).type(torch.uint8).detach().cpu()


def save_images(images: torch.Tensor, save_path: str, num_grid_rows: int):
    """reference :23-29 (uint8 grid -> PNG)."""
    from PIL import Image
    grid = make_grid(images, nrow=num_grid_rows)
    now = datetime.now()
    os.makedirs(save_path, exist_ok=True)
    Image.fromarray(grid.permute(1, 2, 0).numpy()).save(
        os.path.join(save_path, f'old_x_{now.hour}:{now.minute}:{now.second}.png'))


@torch.no_grad()
def sample_tensor(model: UNet, scheduler: LinearNoiseScheduler, batch: int, im_channels: int = 3, im_size: int = 128,
                  *, seed: Optional[int] = None, x_T: Optional[torch.Tensor] = None) -> torch.Tensor:
    """reference :52-64 with the reference RNG stream (CPU randn for x_T and every z)."""
    dev = scheduler.device
    if seed is not None:
        torch.manual_seed(seed)
    xt = (torch.randn((batch, im_channels, im_size, im_size)) if x_T is None else x_T).to(dev)
    for i in reversed(range(scheduler.num_timesteps)):
        t = torch.full((xt.size(0), ), i, dtype=torch.long, device=dev)
        noise_pred = model(xt, scheduler.one_minus_cum_prod[t].view(-1, 1, 1, 1))
        mean, sigma, _ = scheduler.sample_prev_timestep2(xt, noise_pred, t)
        xt = mean + sigma if i != 0 else mean
    return xt


def sample(model, scheduler, train_config: TrainingConfig, model_config: ModelConfig, diffusion_config: DiffusionConfig,
           save_path: Optional[str] = 'diffusion_model_v2/outputs/samples', *, seed: Optional[int] = None):
    """reference :40-67; returns the uint8 images."""
    xt = sample_tensor(model, scheduler, train_config.sample_size, model_config.im_channels, model_config.im_size,
                       seed=seed)
    images = postprocess(xt)
    if save_path is not None:
        save_images(images, save_path, train_config.num_grid_rows)
    return images


def load_model(model_path: str) -> torch.nn.Module:
    """reference :70-75 (weights_only checkpoint load)."""
    dev = _device()
    model = UNet().to(dev)
    model.load_state_dict(torch.load(model_path, map_location=dev, weights_only=True)['model_state_dict'])
    return model.eval()


def infer(config: Config):
    """reference :87-97."""
    model = load_model(os.path.join(config.folders.checkpoints, 'old_model/1000-checkpoint.ckpt'))
    scheduler = load_scheduler(config.diffusion)
    with torch.no_grad():
        return sample(model, scheduler, config.training, config.model, config.diffusion,
                      os.path.join(config.folders.samples, 'old_model'))


if __name__ == '__main__':
    infer(load_config())
