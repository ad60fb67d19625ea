"""Semantic-gradient guidance (reference ``sgg/sgg.py``).

``apply_gsg``: the segmenter input gradient (PyTorch-ROCm autograd, north_star) followed by ONE HIP
kernel (``wc_sgg_update``) that does the 4x4 average pool, the std-weighted L2 magnitude and the
``mu + lambda*sigma*m + sigma`` update that the reference spreads over ``F.avg_pool2d``, a numpy host
round trip and three float64 tensor ops (``sgg.py:18-22``, ``inference.py:39-43``).

Documented deviations:
  * D4 — the reference's magnitude assumes batch 1; for batch > 1 its numpy sum runs over the batch
    axis.  ``batch_semantics='reference'`` reproduces that; the default ``'per_sample'`` gives each
    sample its own channel magnitude (identical at batch 1).
  * dtype — the reference returns float64 (numpy promotion); here fp32 (the UNet's input dtype).
  * D3 — ``apply_lcg`` as written multiplies (1,3,S,S) by (1,1,4S,4S) masks and raises; ``mode=
    'reference'`` raises the same way, ``mode='applied'`` pools each class mask to the latent grid.
"""
import torch
import torch.nn.functional as F

from .. import kernels as K
from ..seg_model.inference import STD, input_gradient


def _update(grad, mu, sigma, lam, batch_semantics):
    if grad.shape[0] != mu.shape[0]:
        raise RuntimeError('segmenter gradient and mu batch sizes differ')
    xt, _ = K.sgg_update(grad.float(), mu.float(), sigma.float(), float(lam), std=STD,
                         batch_axis_sum=(batch_semantics == 'reference' and mu.shape[0] > 1))
    return xt


def apply_gsg(seg_model: torch.nn.Module, mu: torch.Tensor, sigma: torch.Tensor, sr_xt: torch.Tensor,
              gt: torch.Tensor, _lambda: float, *, batch_semantics: str = 'per_sample') -> torch.Tensor:
    """Global guidance (sgg.py:9-24): xt = mu + lambda*sigma*|avgpool4(dCE/dsr_xt)|_std + sigma."""
    grad, _ = input_gradient(seg_model, sr_xt, gt)
    return _update(grad, mu, sigma, _lambda, batch_semantics)


def apply_lcg(seg_model: torch.nn.Module, mu: torch.Tensor, sigma: torch.Tensor, sr_xt: torch.Tensor,
              gt: torch.Tensor, _lambda: float, *, num_classes: int = 19, mode: str = 'applied') -> torch.Tensor:
    """Local class-wise guidance (sgg.py:27-60): per class c, guide on the class-masked input and blend
    the per-class results with the class masks."""
    S = mu.shape[-1]
    out = torch.zeros_like(mu, dtype=torch.float32)
    for c in range(num_classes):
        mc = (gt == c).to(sr_xt.dtype).unsqueeze(1)  # (B, 1, 4S, 4S)
        grad, _ = input_gradient(seg_model, sr_xt * mc, (gt * mc.squeeze(1).long()))
        xt_c = _update(grad, mu, sigma, _lambda, 'per_sample')
        if mode == 'reference':
            # sgg.py:58 multiplies xt_c (B,3,S,S) by the full-resolution mask -> shape error (D3)
            raise RuntimeError(f'apply_lcg reference semantics: cannot broadcast xt_c {tuple(xt_c.shape)} with '
                               f'mask {tuple(mc.shape)} (reference sgg/sgg.py:58)')
        w = F.avg_pool2d(mc, kernel_size=mc.shape[-1] // S)  # class fraction per latent pixel
        out += xt_c * w
    return out
