"""A/B of the two GN+SiLU 3x3 conv forms (three-wave halo kernel vs the one-wave 16x16 form) on the
256-px UNet conv1 shapes at B=16: per-launch time and TF/s (fp32-equivalent), each form timed
back to back on the same inputs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels as K  # noqa: E402

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]
SHAPES = [(256, 64, 128), (256, 128, 128), (128, 128, 256), (128, 256, 256), (64, 256, 512), (64, 512, 512),
          (32, 512, 768), (32, 768, 768)]


def main():
    B = int(os.environ.get('B', 16))
    g = torch.Generator(device='cuda').manual_seed(0)
    for H, Ci, Co in SHAPES:
        x = torch.randn((B, H, H, Ci), device='cuda', generator=g)
        w = torch.randn((Co, 9 * Ci), device='cuda', generator=g) / (9 * Ci)**0.5
        b = torch.randn(Co, device='cuda', generator=g)
        sc = torch.rand((B, Ci), device='cuda', generator=g) + 0.5
        sh = torch.randn((B, Ci), device='cuda', generator=g)
        w3 = K.pack_f16x3(w, Ci, 0)
        out = torch.empty((B, H, H, Co), device='cuda')
        segs = [K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True)]
        fl = 2.0 * B * H * H * Co * 9 * Ci
        row = [f'{H}^2 {Ci}->{Co}']
        for mode in (0, 1, 0, 1):
            K.set_conv3_onewave(mode)
            fn = lambda: K.conv3x3_f16x3(segs, w3, b, K.View.full(out), Hm=H, Wm=H, a_exp=8)  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 20 * 1e-3
            row.append(f'm{mode} {t * 1e6:7.1f}us {fl / t / 1e12:6.1f}TF')
        print(' | '.join(row), flush=True)
    K.set_conv3_onewave(-1)


if __name__ == '__main__':
    main()
