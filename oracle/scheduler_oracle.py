"""ORACLE (test infrastructure only) — CPU restatement of the reference linear-beta DDPM scheduler
and reverse loops.

  LinearNoiseScheduler tables   linear_noise_scheduler.py:11-28 (fp32 linspace/cumprod on CPU)
  add_noise2 / add_noise        linear_noise_scheduler.py:30-61
  sample_prev_timestep2         linear_noise_scheduler.py:63-77
  sample_prev_timestep          linear_noise_scheduler.py:79-116
  sample loop                   diffusion_model/sample_ddpm.py:35-44
  sample_integrated loop        diffusion_model/sample_integrated.py:52-64
  apply_gsg math                sgg/sgg.py:16-22 + seg_model/inference.py:39-53
Noise is drawn from torch's CPU generator exactly where the reference draws it, or injected.
"""
import numpy as np
import torch
import torch.nn.functional as F


class OracleScheduler:

    def __init__(self, num_timesteps: int, beta_start: float, beta_end: float):
        self.num_timesteps = num_timesteps
        self.betas = torch.linspace(beta_start, beta_end, num_timesteps)
        self.alphas = 1. - self.betas
        self.alpha_cum_prod = torch.cumprod(self.alphas, dim=0)
        self.sqrt_alpha_cum_prod = torch.sqrt(self.alpha_cum_prod)
        self.one_minus_cum_prod = 1 - self.alpha_cum_prod
        self.sqrt_one_minus_alpha_cum_prod = torch.sqrt(1 - self.alpha_cum_prod)

    def add_noise(self, original, noise, t):
        B = original.shape[0]
        a = self.sqrt_alpha_cum_prod[t].reshape(B, 1, 1, 1)
        b = self.sqrt_one_minus_alpha_cum_prod[t].reshape(B, 1, 1, 1)
        return a * original + b * noise

    def sample_prev_timestep(self, xt, noise_pred, t: int, z=None):
        mean = xt - ((self.betas[t]) * noise_pred) / (self.sqrt_one_minus_alpha_cum_prod[t])
        mean = mean / torch.sqrt(self.alphas[t])
        if t == 0:
            return mean, None
        variance = (1 - self.alpha_cum_prod[t - 1]) / (1.0 - self.alpha_cum_prod[t])
        variance = variance * self.betas[t]
        sigma = variance**0.5
        if z is None:
            z = torch.randn(xt.shape)
        return mean, sigma * z

    def sample_prev_timestep2(self, xt, noise_pred, t: torch.Tensor, z=None):
        beta = self.betas[t].view(-1, 1, 1, 1)
        alpha = self.alphas[t].view(-1, 1, 1, 1)
        s1m = self.sqrt_one_minus_alpha_cum_prod[t].view(-1, 1, 1, 1)
        mean = xt - ((beta * noise_pred) / s1m)
        mean = mean / torch.sqrt(alpha)
        if torch.all(t == 0):
            return mean, None
        sigma = beta**0.5
        if z is None:
            z = torch.randn(xt.shape)
        return mean, sigma * z


def sample_loop(model_fn, sched: OracleScheduler, x_T: torch.Tensor, noises=None):
    """sample_ddpm.py:35-44 with x_T given; noises[i] (if given) replaces the torch.randn at step i."""
    xt = x_T
    for i in reversed(range(sched.num_timesteps)):
        eps = model_fn(xt, torch.as_tensor(i).unsqueeze(0))
        z = None if noises is None else noises[i]
        mean, sz = sched.sample_prev_timestep(xt, eps, i, z=z)
        xt = mean + sz if i != 0 else mean
    return xt


def gsg_update(grad: torch.Tensor, mu: torch.Tensor, sigma: torch.Tensor, lam: float) -> torch.Tensor:
    """apply_gsg after the segmenter backward (sgg.py:18-22, inference.py:39-53), float64 result."""
    pooled = F.avg_pool2d(grad, kernel_size=4, stride=4)
    g = pooled.squeeze(0).cpu().numpy()
    g = g * np.array([0.229, 0.224, 0.225])[:, None, None]
    mag = torch.from_numpy(np.sqrt(np.sum(g**2, axis=0)))
    mu_hat = mu + lam * sigma * mag
    return mu_hat + sigma
