"""ORACLE (test infrastructure only) — CPU restatement of the reference's semantic-gradient guidance.

  infer (input gradient)          seg_model/inference.py:118-152 (CE mean, ignore_index=255, backward
                                  to the input; pred / numpy copies dropped)
  compute_gradient_magnitude      seg_model/inference.py:36-53 (numpy float64 host math, batch 1)
  apply_gsg                       sgg/sgg.py:9-24
  apply_lcg                       sgg/sgg.py:27-60, per-class loop :39-56 restated exactly; the final
                                  blend :58-60 cannot run as written (D3: stack of (1,3,S,S) latents
                                  times stack of (1,1,4S,4S) masks does not broadcast), so the
                                  'applied' blend weights xt_c by the class mask average-pooled to the
                                  latent grid (kernel = stride = 4S/S), the fraction of class-c pixels
                                  behind each latent pixel: xt = sum_c pool(mc) * xt_c.

PARITY: apply_gsg is pinned to tests/golden/guided.npz (made by importing the reference's
seg_model.network and restating sgg.py:16-22 there, since sgg/ imports torchvision, absent here).
The per-class loop of apply_lcg reuses that pinned math; the pooled-mask blend is the documented
deviation D3 and is parity-unpinned (the reference raises there).
The segmenter passed in is any nn.Module run on the CPU with plain PyTorch.
"""
import numpy as np
import torch
import torch.nn.functional as F

STD = np.array([0.229, 0.224, 0.225])


def input_gradient(seg_model, x: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
    """inference.py:118-152: d CE(model(x), gt.squeeze(1); ignore 255) / d x."""
    x = x.detach().clone().requires_grad_(True)
    with torch.enable_grad():
        out = seg_model(x)
        loss = torch.nn.CrossEntropyLoss(ignore_index=255)(out, gt.squeeze(1))
        loss.backward()
    return x.grad


def gradient_magnitude(grad: torch.Tensor) -> torch.Tensor:
    """sgg.py:18-19 + inference.py:39-43 (batch 1): avg_pool2d(4, 4), squeeze(0), numpy, * std, L2 over c."""
    pooled = F.avg_pool2d(grad, kernel_size=4, stride=4)
    g = pooled.squeeze(0).cpu().numpy() * STD[:, None, None]
    return torch.from_numpy(np.sqrt(np.sum(g**2, axis=0)))


def apply_gsg(seg_model, mu, sigma, sr_xt, gt, lam: float) -> torch.Tensor:
    """sgg.py:9-24 (float64 result, as the reference's numpy promotion gives)."""
    mag = gradient_magnitude(input_gradient(seg_model, sr_xt, gt))
    return (mu + lam * sigma * mag) + sigma


def apply_lcg_applied(seg_model, mu, sigma, sr_xt, gt, lam: float, num_classes: int = 19) -> torch.Tensor:
    """sgg.py:27-60 with the pooled-mask blend (D3), float64 result."""
    S = mu.shape[-1]
    xt = torch.zeros(mu.shape, dtype=torch.float64)
    for c in range(num_classes):  # sgg.py:39
        mc = (gt == c).long().unsqueeze(1)  # :41 [1,1,4S,4S]
        xt_masked = sr_xt * mc  # :44
        gt_masked = gt * mc.squeeze(0)  # :45
        mag = gradient_magnitude(input_gradient(seg_model, xt_masked, gt_masked))  # :47-50
        xt_c = (mu + lam * sigma * mag) + sigma  # :52-53
        w = F.avg_pool2d(mc.double(), kernel_size=mc.shape[-1] // S)  # D3 blend weight
        xt = xt + w * xt_c
    return xt
