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


class _Replay:
    """fn(x) captured into a HIP graph over a static input buffer: a call copies x in and replays
    (the per-kernel host launch cost of a B=1 UNet / SRGAN forward is most of its eager time).  The
    returned tensor is the graph's static output: consumed before the next call."""

    def __init__(self, fn, x: torch.Tensor):
        self.x = x.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # allocations and weight packing outside the capture
                self.y = fn(self.x)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.y = fn(self.x)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        self.x.copy_(x)
        self.graph.replay()
        return self.y


@torch.no_grad()
def sample_with_sgg(input_tensor: torch.Tensor, diff_model, diff_scheduler, seg_model, gt: torch.Tensor,
                    srgan_model, *, LAMBDA: float = 60.0, N: int = 500, mode: str = 'applied', use_lcg: bool = False,
                    t_start: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
                    progress=None, return_latent: bool = False, graph: bool = True):
    """graph=True replays the UNet and SRGAN forwards from HIP graphs (same kernels, same results);
    the segmenter's autograd pass stays eager."""
    if mode not in ('reference', 'applied'):
        raise ValueError("mode must be 'reference' or 'applied'")
    dev = diff_scheduler.device
    x0 = input_tensor.to(dev, torch.float32)
    # forward process (translation.py:63-65): random t in [0, N), one noising of the input
    t = torch.randint(0, N, (x0.shape[0], )) if t_start is None else t_start
    nz = torch.randn_like(x0) if noise is None else noise.to(dev)
    xt = diff_scheduler.add_noise2(x0, nz, t.to(dev))
    ts = torch.arange(N, device=dev, dtype=torch.long)
    unet_run = sr_run = None
    if graph and xt.is_cuda:
        from .diffusion_model.sample_ddpm import _GraphStep
        unet_run = _GraphStep(diff_model, xt)
        sr_run = _Replay(lambda v: srgan_inference(srgan_model, v), xt)
    for i in reversed(range(N)):
        eps = unet_run(xt, ts[i:i + 1]) if unet_run is not None else diff_model(xt, ts[i:i + 1])
        mu, sigma, _ = diff_scheduler.sample_prev_timestep(xt, eps, i)
        if i == 0:
            xt = mu
            break
        sr_xt = sr_run(xt) if sr_run is not None else srgan_inference(srgan_model, xt)
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
