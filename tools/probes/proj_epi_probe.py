"""Probe: the attention out-projection (1x1 f16x3 implicit GEMM, raw input) as the UNet launches it
-- residual in place, output in a strided (skip-concat) view, GN tile partials, absmax -- with each
epilogue feature toggled, to find what the in-model launch pays over the bare GEMM."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from weatherconverter_amd import kernels as K  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def case(B, H, C, ldo, res, gn, amax):
    g = torch.Generator(device='cuda').manual_seed(0)
    o = torch.randn((B, H, H, C), device='cuda', generator=g)
    w = torch.randn((C, C), device='cuda', generator=g) / C**0.5
    b = torch.randn(C, device='cuda', generator=g)
    buf = torch.randn((B, H, H, ldo), device='cuda', generator=g)
    Y = K.View(buf, 0, C)
    gp = K.GnPart.attach(buf, 16) if gn else None
    am = torch.zeros(B, device='cuda') if amax else None
    w3 = K.pack_f16x3(w, C, ntaps=1, order='natural')
    fn = lambda: K.conv_igemm_f16x3([K.Seg(K.View.full(o), [(0, 0)])], w3, b, Y, Hm=H, Wm=H, a_exp=8,  # noqa: E731
                                    res=Y if res else None, absmax=am, gn=gp)
    t = timeit(fn)
    return t, 2.0 * B * H * H * C * C / t / 1e12


def main():
    K._native.load()
    for (B, H, C) in [(16, 64, 512), (16, 32, 768)]:
        for ldo_mul, res, gn, amax in [(1, False, False, False), (1, False, False, False), (2, False, False, False),
                                       (1, True, False, False), (1, False, True, False), (1, False, False, True),
                                       (2, True, True, False), (2, True, True, True)]:
            t, tf = case(B, H, C, C * ldo_mul, res, gn, amax)
            print(f'B={B} S={H} C={C} ldo={C * ldo_mul} res={res} gn={gn} absmax={amax}: {t * 1e3:7.3f} ms '
                  f'{tf:6.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
