"""Probe: f16x3 3x3 conv time on the in-model shapes with and without the epilogue side outputs
(per-image absmax atomics, GroupNorm tile partials), and on the small-grid 32x32 shapes.

Prints one line per case; run on the GPU box (tools/archive/gpu_probe.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from weatherconverter_amd import kernels as K  # noqa: E402

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def case(B, H, Ci, Co, res, absmax, gn):
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn((B, H, H, Ci), device='cuda', generator=g)
    w = torch.randn((Co, 9 * Ci + res), device='cuda', generator=g) / (9 * Ci)**0.5
    b = torch.randn(Co, device='cuda', generator=g)
    sc = torch.rand((B, Ci), device='cuda', generator=g) + 0.5
    sh = torch.randn((B, Ci), device='cuda', generator=g) * 0.1
    out = torch.empty((B, H, H, Co), device='cuda')
    segs = [K.Seg(K.View.full(x), TAPS3, scale=sc, shift=sh, silu=True)]
    xb = None
    if res:
        xr = torch.randn((B, H, H, res), device='cuda', generator=g)
        segs.append(K.Seg(K.View.full(xr), [(0, 0)], kbase=9 * Ci))
        xb = torch.full((B, ), 8.0, device='cuda')
    w3 = K.pack_f16x3(w, Ci, res, res_f16=bool(res))
    am = torch.zeros(B, device='cuda') if absmax else None
    gp = None
    if gn:
        gp = K.GnPart.alloc(B, H * H, Co, 8, torch.device('cuda')) if hasattr(K.GnPart, 'alloc') else None
    fn = lambda: K.conv3x3_f16x3(segs, w3, b, K.View.full(out), Hm=H, Wm=H, a_exp=4, a_bound=xb,  # noqa: E731
                                 absmax=am, gn=gp)
    t = timeit(fn)
    fl = 2.0 * B * H * H * Co * (9 * Ci + res)
    return t, fl / t / 1e12


def main():
    K._native.load()
    cases = [(16, 256, 128, 128, 128, False, False), (16, 256, 128, 128, 128, True, False),
             (16, 256, 128, 128, 64, False, False), (16, 256, 128, 128, 64, True, False),
             (16, 128, 256, 256, 256, False, False), (16, 128, 256, 256, 256, True, False),
             (16, 32, 1024, 256, 0, False, False), (16, 32, 256, 256, 0, False, False),
             (16, 32, 256, 256, 1024, False, False), (16, 32, 512, 512, 0, False, False),
             (16, 32, 768, 512, 0, False, False)]
    for c in cases:
        t, tf = case(*c)
        print(f'B={c[0]} S={c[1]} {c[2]}->{c[3]} res={c[4]} absmax={c[5]}: {t * 1e3:8.3f} ms {tf:6.1f} TF/s',
              flush=True)


if __name__ == '__main__':
    main()
