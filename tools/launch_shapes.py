"""Every launch of one 256-px sampling forward (B=16) with its shape: the exact instantiation, the entry
point, for conv launches the segments (C x taps, input size), the output size and channels; each launch's
time (HIP events, min over 3 forwards).  `python tools/launch_shapes.py [name-substring]` prints the
launches whose instantiation contains the substring (default: all), in forward order."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import _native, kernels as K  # noqa: E402
from weatherconverter_amd.diffusion_model.config import model_config  # noqa: E402
from weatherconverter_amd.diffusion_model.models.unet_base import Unet  # noqa: E402
from weatherconverter_amd.synthetic import init_synthetic_  # noqa: E402

rec = []
_orig = _native.call


def _shape(args) -> str:
    a = args[0] if args else None
    if isinstance(a, type(ctypes.byref(ctypes.c_int()))):
        a = a._obj
    if isinstance(a, _native.ConvArgs):
        segs = ' + '.join(f'{a.seg[i].C}x{a.seg[i].ntaps}t@{a.seg[i].H}x{a.seg[i].W}' for i in range(a.nseg))
        return f'[{segs}] -> {a.N} @ {a.Hm}x{a.Wm}' + (' +res' if a.res else '')
    return ''


def call(fn, *args):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = _orig(fn, *args)
    e1.record()
    rec.append((fn, _native.last_kernel_name() or fn, _shape(args), e0, e1))
    return r


_native.call = call
net = Unet(model_config(256))
init_synthetic_(net, seed=0)
net = net.cuda().eval()
x = torch.randn((16, 3, 256, 256), device='cuda')
t = torch.full((16, ), 500, device='cuda', dtype=torch.long)
with torch.no_grad():
    net(x, t)
    torch.cuda.synchronize()
    rec.clear()
    for _ in range(3):
        net(x, t)
    torch.cuda.synchronize()
n = len(rec) // 3
sub = sys.argv[1] if len(sys.argv) > 1 else ''
tot = 0.0
for i in range(n):
    fn, name, shape, _, _ = rec[i]
    us = min(rec[i + j * n][3].elapsed_time(rec[i + j * n][4]) for j in range(3)) * 1e3
    tot += us
    if sub in name:
        print(f'{i:3d} {us:8.1f} us  {name[:60]:60s} {fn:32s} {shape}', flush=True)
print(f'total {tot / 1e3:.3f} ms over {n} launches (events around each call)')
