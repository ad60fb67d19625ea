"""Pre-split projection GEMM (wc_proj_f16x3 / wc_proj_f16x3_qkv) on the UNet attention shapes and
K / N sweeps at B=16: per-launch time, TF/s (fp32-equivalent) and the per-K-step cost, to separate
the K loop from the prologue and epilogue."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels as K  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    B = 16
    g = torch.Generator(device='cuda').manual_seed(0)
    cases = [('out', 64, 512, 512), ('out', 64, 256, 512), ('out', 64, 1024, 512), ('out', 32, 768, 768),
             ('out', 64, 512, 128), ('qkv', 64, 512, 0), ('qkv', 32, 768, 0), ('qkv', 32, 512, 0), ('qkv', 64, 128, 0),
             ('plain', 64, 512, 1536)]
    for kind, H, C, N in cases:
        x = torch.rand((B, H, H, C), device='cuda', generator=g) * 14 - 7
        v = K.View.full(x)
        e = K.f16x3_a_exp(0.0, 7.0, 2)
        a3 = K.split_f16x3_tiled(v, e)
        if kind == 'qkv':
            N = 3 * C
            w = torch.randn((N, C), device='cuda', generator=g) / C**0.5
            w3 = K.pack_f16x3(w, C, ntaps=1, order='natural')
            b = torch.randn(N, device='cuda', generator=g) * 0.1
            qkv3 = torch.empty(B * 6 * C * H * H, dtype=torch.int16, device='cuda')
            fn = lambda: K.proj_f16x3_qkv(v, a3, w3, b, qkv3, a_exp=e, C=C, heads=4, exps=(8, 8, 8))  # noqa: E731
        else:
            w = torch.randn((N, C), device='cuda', generator=g) / C**0.5
            w3 = K.pack_f16x3(w, C, ntaps=1, order='natural')
            b = torch.randn(N, device='cuda', generator=g) * 0.1
            y = torch.randn((B, H, H, N), device='cuda', generator=g)
            yv = K.View.full(y)
            res = yv if kind == 'out' else None
            gp = K.GnPart.attach(y, 16) if kind == 'out' else None
            am = torch.zeros(B, device='cuda')
            fn = lambda: K.proj_f16x3(v, a3, w3, b, yv, a_exp=e, res=res, absmax=am if res is not None else None, gn=gp)  # noqa: E731
        t = timeit(fn)
        M = B * H * H
        fl = 2.0 * M * N * C
        wgs = (M // 128) * ((N + 127) // 128)
        print(f'{kind:5s} {H}^2 C={C:4d} N={N:4d}: {t * 1e6:7.1f} us {fl / t / 1e12:6.1f} TF/s  wgs={wgs} '
              f'steps={C // 16}  us/(wg-step)={t * 1e6 / (wgs / 768.0) / (C // 16):.3f}', flush=True)


if __name__ == '__main__':
    main()
