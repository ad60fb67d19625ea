"""Segmenter inference for semantic-gradient guidance (reference ``seg_model/inference.py``).

``infer`` keeps the reference's signature and return triple (``:118-152``) but computes ONLY the
input gradient: ``torch.autograd.grad(loss, input)`` skips every weight-gradient kernel (the
reference's ``loss.backward()`` also accumulates ``.grad`` on all 58.75 M segmenter parameters,
SURVEY §8(f) #3), and it differentiates a detached copy instead of flipping ``requires_grad`` on the
caller's tensor (reference :132).  The pooled-gradient magnitude runs in the ``wc_sgg_update`` HIP
kernel instead of the reference's host numpy round trip (:36-53).
"""
from typing import Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .. import kernels as K
from .network import deeplabv3plus_resnet101, deeplabv3plus_resnet50  # noqa: F401

STD = (0.229, 0.224, 0.225)  # ImageNet std used by the reference's de-normalisation (:42)


def load_model(model_path: str, num_classes: int = 19, output_stride: int = 16, name: str = 'deeplabv3plus_resnet101',
               device=None) -> torch.nn.Module:
    """reference :27-33 — build the net WITHOUT the pretrained-backbone download, load the checkpoint."""
    device = device or torch.device('cuda' if torch.cuda.is_available() else 'cpu')
    ctor = {'deeplabv3plus_resnet101': deeplabv3plus_resnet101, 'deeplabv3plus_resnet50': deeplabv3plus_resnet50}[name]
    model = ctor(num_classes=num_classes, output_stride=output_stride)
    model.load_state_dict(torch.load(model_path, map_location='cpu', weights_only=True)['model_state_dict'])
    return model.to(device).eval()


def input_gradient(model: torch.nn.Module, input_tensor: torch.Tensor, encoded_label_tensor: torch.Tensor,
                   want_pred: bool = False):
    """d CE_mean,ignore255(model(x), y) / d x  (and optionally the logits)."""
    x = input_tensor.detach().requires_grad_(True)
    with torch.enable_grad():
        out = model(x)
        loss = F.cross_entropy(out, encoded_label_tensor.squeeze(1), ignore_index=255)
        (g, ) = torch.autograd.grad(loss, x)
    return g, (out.detach() if want_pred else None)


def infer(model: torch.nn.Module, input_tensor: torch.Tensor, encoded_label_tensor: torch.Tensor,
          verbose: bool = False) -> Tuple[np.ndarray, torch.Tensor, np.ndarray]:
    """reference :118-152 — (pred [H, W] numpy, input gradient tensor, gradient numpy [3, H, W])."""
    g, out = input_gradient(model, input_tensor, encoded_label_tensor, want_pred=True)
    pred = out.argmax(dim=1).squeeze(0).cpu().numpy()
    if verbose:
        print(f'output {tuple(out.shape)}, grad {tuple(g.shape)}')
    return pred, g, g.detach().cpu().squeeze(0).numpy()


def compute_gradient_magnitude(input_gradients: torch.Tensor, denormalize: bool = True, norm: bool = False) -> torch.Tensor:
    """reference :36-53: sqrt(sum_c (g_c * std_c)^2) over axis 0 after ``squeeze(0)`` (float64 result).

    Batch 1 -> (H, W) magnitude over channels; batch > 1 -> the reference's numpy sums over the
    BATCH axis instead (D4), giving (3, H, W); both reproduced.  (Host-free torch float64 ops; the
    fused pool+magnitude+update used by ``apply_gsg`` is the ``wc_sgg_update`` kernel.)
    """
    g = input_gradients.squeeze(0).double()
    if denormalize:
        std = torch.tensor(STD, dtype=torch.float64, device=g.device)
        g = g * (std[:, None, None] if g.dim() == 3 else std[None, :, None, None])
    mag = torch.sqrt(torch.sum(g**2, dim=0))
    if norm:
        mag = (mag - mag.min()) / (mag.max() - mag.min())
    return mag
