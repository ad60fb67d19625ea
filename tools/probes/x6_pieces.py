"""Probe: which operand's third bf16 piece reaches the MFMA in wc_conv3x3_x6.
A or W is rounded to bf16-exact values so only the other operand's pieces matter."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from weatherconverter_amd import kernels as K  # noqa: E402

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]


def bf16_exact(x):
    return ((x.view(torch.int32) >> 16) << 16).view(torch.float32)


def run(a, w):
    B, H, W_, Ci = a.shape
    Co = w.shape[0]
    out = torch.empty((B, H, W_, Co), device='cuda')
    K.conv3x3_x6([K.Seg(K.View.full(a), TAPS3)], K.pack_x6(w, Ci), None, K.View.full(out), Hm=H, Wm=W_)
    wt = w.double().reshape(Co, 3, 3, Ci).permute(0, 3, 1, 2)
    ref = F.conv2d(a.double().permute(0, 3, 1, 2), wt, padding=1).permute(0, 2, 3, 1)
    return float((out.double() - ref).norm() / ref.norm())


g = torch.Generator(device='cuda').manual_seed(0)
a = torch.randn((1, 16, 16, 64), device='cuda', generator=g)
w = torch.randn((128, 9 * 64), device='cuda', generator=g) / 24
print('both fp32        ', run(a, w))
print('A bf16, W fp32   ', run(bf16_exact(a), w))
print('A fp32, W bf16   ', run(a, bf16_exact(w)))
print('both bf16        ', run(bf16_exact(a), bf16_exact(w)))
# piece 2 only: values whose pieces 0 and 1 are fixed and known
p = K.split3_bits(w)
print('W piece-2 nonzero count', int((p[2] != 0).sum()), 'of', p[2].numel())
