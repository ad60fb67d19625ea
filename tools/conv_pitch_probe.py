"""f16x3 3x3 conv at S=256 with the input's pixel stride (ldc) padded: tests whether the slowdown of
the wide-row layers is an HBM address-mapping effect of the 2^k row pitch.  python tools/conv_pitch_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import timeit, TAPS3  # noqa: E402
from weatherconverter_amd import kernels as K  # noqa: E402

K._native.load()
for (B, H, C, pad) in [(16, 256, 128, 0), (16, 256, 128, 4), (16, 256, 128, 16), (16, 256, 128, 32),
                       (16, 128, 256, 0), (16, 128, 256, 4), (16, 256, 64, 0), (16, 256, 64, 4)]:
    g = torch.Generator(device='cuda').manual_seed(0)
    xt = torch.randn((B, H, H, C + pad), device='cuda', generator=g)
    w = torch.randn((C, 9 * C), device='cuda', generator=g) / (9 * C)**0.5
    b = torch.randn(C, device='cuda', generator=g)
    sc = torch.rand((B, C), device='cuda', generator=g) + 0.5
    sh = torch.randn((B, C), device='cuda', generator=g) * 0.1
    out = torch.empty((B, H, H, C), device='cuda')
    seg = K.Seg(K.View(xt, 0, C), TAPS3, scale=sc, shift=sh, silu=True)
    w3 = K.pack_f16x3(w, C)
    t = timeit(lambda: K.conv3x3_f16x3([seg], w3, b, K.View.full(out), Hm=H, Wm=H, a_exp=4))
    fl = 2.0 * B * H * H * C * 9 * C
    print(f'B={B} S={H} C={C} ldc={C + pad}: {t*1e3:7.3f} ms {fl / t / 1e12:6.1f} TF/s', flush=True)
