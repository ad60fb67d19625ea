"""Guided weather translation loop (reference ``translation.py:46-97``, ``sample_with_sgg``).

Per reverse step i (N = 500 over the T = 1000 schedule, lambda = 60):
    eps = UNet(xt, i)                                   HIP engine
    mu, sigma*z = scheduler.sample_prev_timestep(...)   HIP kernel (sigma is sigma_t * z, D5)
    sr_xt = SRGAN(xt)                                   PyTorch-ROCm, x4
    odd i: xt = apply_gsg(...)   even i: xt = apply_lcg(...)   (segmenter fwd+input-grad + HIP update)
    xt = mu + sigma                                     reference line 90 (D1: overwrites the guidance)

``mode='reference'`` keeps D1 (guidance computed, then discarded) — the reference's effective output;
``mode='applied'`` keeps the guided xt on guided steps.  D2 (``mu + None`` TypeError at i = 0) is not
reproduced: the last step returns ``mu`` as ``sample_ddpm`` does.  LCG runs only when ``use_lcg``
(the reference's LCG crashes, D3; see ``sgg.apply_lcg``).
"""
from typing import Optional

import torch

from .sgg.sgg import apply_gsg, apply_lcg
from .srgan_model.models import inference as srgan_inference


@torch.no_grad()
def sample_with_sgg(input_tensor: torch.Tensor, diff_model, diff_scheduler, seg_model, gt: torch.Tensor,
                    srgan_model, *, LAMBDA: float = 60.0, N: int = 500, mode: str = 'applied', use_lcg: bool = False,
                    t_start: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
                    progress=None, return_latent: bool = False):
    if mode not in ('reference', 'applied'):
        raise ValueError("mode must be 'reference' or 'applied'")
    dev = diff_scheduler.device
    x0 = input_tensor.to(dev, torch.float32)
    # forward process (translation.py:63-65): random t in [0, N), one noising of the input
    t = torch.randint(0, N, (x0.shape[0], )) if t_start is None else t_start
    nz = torch.randn_like(x0) if noise is None else noise.to(dev)
    xt = diff_scheduler.add_noise2(x0, nz, t.to(dev))
    ts = torch.arange(N, device=dev, dtype=torch.long)
    for i in reversed(range(N)):
        eps = diff_model(xt, ts[i:i + 1])
        mu, sigma, _ = diff_scheduler.sample_prev_timestep(xt, eps, i)
        if i == 0:
            xt = mu
            break
        sr_xt = srgan_inference(srgan_model, xt)
        guided = None
        if i % 2 == 1:
            guided = apply_gsg(seg_model, mu, sigma, sr_xt, gt, LAMBDA)
        elif use_lcg:
            guided = apply_lcg(seg_model, mu, sigma, sr_xt, gt, LAMBDA, mode=mode)
        if mode == 'applied' and guided is not None:
            xt = guided.contiguous()
        else:
            xt = (mu + sigma).contiguous()  # translation.py:90
        if progress is not None:
            progress(i)
    sr_x0 = srgan_inference(srgan_model, xt)  # translation.py:95
    return (sr_x0, xt) if return_latent else sr_x0
