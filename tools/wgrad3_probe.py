"""The halo 3x3 weight-gradient kernel (wc_conv_wgrad3_f16x3) alone on the ResBlock shapes of the 256-px
UNet (GN+SiLU prologue), for timing and PMC passes.  usage: wgrad3_probe.py [--only i] [--batch B]
[--line f16x3|bf16|f16] (bf16 / f16: the single-piece training builds' library)"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import TAPS3, timeit  # noqa: E402
from weatherconverter_amd import kernels as K  # noqa: E402

SHAPES = [(16, 256, 128, 128), (16, 128, 256, 256), (16, 64, 512, 512), (16, 32, 768, 768), (16, 128, 128, 256)]


def case(B, S, C, M):
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn((B, S, S, C), device='cuda', generator=g)
    gy = torch.randn((B, S, S, M), device='cuda', generator=g) * 1e-3
    sc = torch.rand((B, C), device='cuda', generator=g) + 0.5
    sh = torch.randn((B, C), device='cuda', generator=g) * 0.1
    dw = torch.empty((M, C, 3, 3), device='cuda')
    gb = gy.abs().reshape(B, -1).amax(1).contiguous()
    seg = K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True)
    fn = lambda: K.conv_wgrad(K.View.full(gy), [seg], dw, (C * 9, 9, 1), x6=True,  # noqa: E731
                              f3=K.F3Bounds(gb, 4))
    t = timeit(fn)
    return t, 2.0 * B * S * S * M * 9 * C / t / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--only', type=int, default=-1)
    ap.add_argument('--batch', type=int, default=0)
    ap.add_argument('--line', default='f16x3', choices=['f16x3', 'bf16', 'f16'])
    a = ap.parse_args()
    var = {'f16x3': '', 'bf16': 'bf16', 'f16': 'single16'}[a.line]
    with K._native.variant(var):
        K._native.load()
        for i, (B, S, C, M) in enumerate(SHAPES):
            if a.only >= 0 and i != a.only:
                continue
            B = a.batch or B
            t, tf = case(B, S, C, M)
            print(f'wgrad3 {a.line} B={B} S={S:3d} C={C} M={M}: {t * 1e3:8.3f} ms  {tf:6.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
