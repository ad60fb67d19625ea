"""Digest (sha256 of the fp32 bytes) of the halo 3x3 weight gradient (wc_conv_wgrad3_f16x3, and the
bf16x6 form) on fixed inputs, for bit-identity checks of a kernel change across two libraries:
run it under the tree's library and under WC_KERNEL_LIB=<alt> WC_ALLOW_STALE_LIB=1 and compare.
usage: wgrad3_digest.py [--line f16x3|bf16]   (bf16: the single-piece training build)"""
import argparse
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import _native  # noqa: E402
from weatherconverter_amd import kernels as K  # noqa: E402
from weatherconverter_amd.diffusion_model.models.engine import TAPS3  # noqa: E402

# (B, H, W, C, M, pro): 128-channel M tiles (8-row blocks) and 64-channel tiles (2-row blocks)
CASES = [(2, 32, 32, 128, 128, 2), (3, 16, 48, 64, 256, 1), (2, 16, 16, 64, 64, 0), (1, 64, 32, 32, 128, 2),
         (2, 8, 16, 128, 192, 2)]


def run(x6_f3: bool):
    out = []
    for i, (B, H, W, C, M, pro) in enumerate(CASES):
        g = torch.Generator(device='cuda').manual_seed(100 + i)
        x = torch.randn((B, H, W, C), device='cuda', generator=g)
        gy = torch.randn((B, H, W, M), device='cuda', generator=g) * 1e-2
        sc = torch.rand((B, C), device='cuda', generator=g) + 0.5
        sh = torch.randn((B, C), device='cuda', generator=g) * 0.1
        dw = torch.zeros((M, C, 3, 3), device='cuda')
        seg = K.Seg(K.View.full(x), TAPS3, scale=sc if pro else None, shift=sh if pro else None, silu=pro == 2)
        gb = gy.abs().reshape(B, -1).amax(1).contiguous()
        f3 = K.F3Bounds(gb, 4 if pro else 60, None if pro else x.abs().reshape(B, -1).amax(1).contiguous()) if x6_f3 else None
        K.conv_wgrad(K.View.full(gy), [seg], dw, (C * 9, 9, 1), x6=True, f3=f3)
        torch.cuda.synchronize()
        out.append(hashlib.sha256(dw.cpu().numpy().tobytes()).hexdigest()[:16])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--line', default='f16x3')
    a = ap.parse_args()
    v = 'bf16' if a.line == 'bf16' else ''
    with _native.variant(v):
        print(a.line, 'f16x3', ' '.join(run(True)))
        if not v:
            print(a.line, 'bf16x6', ' '.join(run(False)))


if __name__ == '__main__':
    main()
