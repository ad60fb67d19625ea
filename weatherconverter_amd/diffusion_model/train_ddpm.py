"""Drop-in for the reference's ``diffusion_model/train_ddpm.py`` training-loss path (BASELINE config 3).

One training iteration of the reference (``train_ddpm.py:94-114``) is
    noise = randn_like(images); t = randint(0, T, (B,))
    noisy_im = scheduler.add_noise(images, noise, t)        # :105
    noise_pred = model(noisy_im, t)                         # :106
    loss = criterion(noise_pred, noise)                     # :108, criterion = nn.MSELoss() (:177)
followed by ``loss.backward()`` and ``optimizer.step()``.  All of it runs on HIP kernels except the
Adam update (torch's ``optim.Adam`` on the device): ``wc_add_noise`` (per-sample coefficients), the
UNet forward with per-sample timesteps recording its tape, ``wc_mse_loss`` (fp64-accumulated,
deterministic mean, fused with d loss / d noise_pred), and ``loss.backward()`` through
``UnetTrainFunction`` (models/train_engine.py: data and weight gradients, GroupNorm, attention and
time-embedding backward kernels).  ``training_loss`` is the forward; ``TrainForward`` is the same
captured into a HIP graph for the forward-only line.  Checkpoints keep the reference format (``:56-68``):
``{'model_state_dict', 'optimizer_state_dict', 'epoch'}`` saved as ``f'{epoch}-checkpoint.ckpt'``.
"""
import os
from typing import Optional, Tuple

import torch

from .. import kernels as K
from .config import Config, load_config  # noqa: F401  (reference :19-22)
from .models.unet_base import Unet
from .scheduler.linear_noise_scheduler import LinearNoiseScheduler


def training_loss(model: Unet, scheduler: LinearNoiseScheduler, images: torch.Tensor, noise: torch.Tensor,
                  t: torch.Tensor, *, with_grad: bool = False) -> Tuple[torch.Tensor, ...]:
    """The forward of one training iteration (``train_ddpm.py:105-108``) on the GPU.

    Returns ``(loss, noise_pred)``; with ``with_grad=True`` also d loss / d noise_pred (the seed of
    the backward pass), written by the same MSE sweep.  ``t``: int64 (B,) per-sample timesteps."""
    dev = next(model.parameters()).device
    tt = torch.as_tensor(t).long().reshape(-1).to(dev)
    if tt.numel() != images.shape[0]:
        raise RuntimeError(f'training_loss: {tt.numel()} timesteps for a batch of {images.shape[0]}')
    nz = noise.to(dev, torch.float32).contiguous()
    with torch.no_grad():
        noisy = scheduler.add_noise(images, nz, tt)
        pred = model(noisy, tt)
        out = K.mse_loss(pred, nz, grad=with_grad)
    if with_grad:
        loss, g = out
        return loss, pred, g
    return out, pred


class TrainForward:
    """``training_loss`` captured into a HIP graph over fixed device buffers (images, noise, t):
    copy a batch in, replay, read ``loss``.  Used by the config-3 benchmark."""

    def __init__(self, model: Unet, scheduler: LinearNoiseScheduler, images: torch.Tensor, noise: torch.Tensor,
                 t: torch.Tensor):
        self.model, self.scheduler = model, scheduler
        dev = next(model.parameters()).device
        self.images = images.to(dev, torch.float32).contiguous().clone()
        self.noise = noise.to(dev, torch.float32).contiguous().clone()
        self.t = torch.as_tensor(t).long().reshape(-1).to(dev).clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self.loss, self.pred = training_loss(model, scheduler, self.images, self.noise, self.t)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss, self.pred = training_loss(model, scheduler, self.images, self.noise, self.t)

    def __call__(self, images: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
                 t: Optional[torch.Tensor] = None) -> torch.Tensor:
        if images is not None:
            self.images.copy_(images)
        if noise is not None:
            self.noise.copy_(noise)
        if t is not None:
            self.t.copy_(torch.as_tensor(t).reshape(-1))
        self.graph.replay()
        return self.loss


# ----------------------------------------------------------------------------------- checkpoints
def checkpoint_path(folder: str, run_id, epoch: int) -> str:
    """``train_ddpm.py:57`` naming: <checkpoints>/<run_id>/<epoch>-checkpoint.ckpt."""
    return os.path.join(folder, str(run_id), f'{epoch}-checkpoint.ckpt')


def save_checkpoint(epoch: int, model: Unet, opt: torch.optim.Optimizer, folder: str, run_id=0) -> str:
    """``train_ddpm.py:55-59``: {'model_state_dict', 'optimizer_state_dict', 'epoch'}."""
    path = checkpoint_path(folder, run_id, epoch)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save({'model_state_dict': model.state_dict(), 'optimizer_state_dict': opt.state_dict(), 'epoch': epoch},
               path)
    return path


def load_checkpoint(model: Unet, opt: Optional[torch.optim.Optimizer], checkpoint_path: str):
    """``train_ddpm.py:62-68`` -> (model, opt, epoch).  Tensors and plain containers only
    (``weights_only=True``: nothing in the file is executed)."""
    ck = torch.load(checkpoint_path, map_location='cpu', weights_only=True)
    model.load_state_dict(ck['model_state_dict'])
    if opt is not None and 'optimizer_state_dict' in ck:
        opt.load_state_dict(ck['optimizer_state_dict'])
    return model, opt, ck['epoch']
