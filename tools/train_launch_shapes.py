"""Every launch of one config-3 training iteration (add_noise + UNet forward + MSE + backward, no Adam) at
256 px, B=32, with its shape and its time (HIP events around each call, min over 2 iterations): the
per-shape view of the training line.  `python tools/train_launch_shapes.py [--precision bf16] [--top 40]`
prints the launches grouped by (instantiation, shape), largest total first."""
import argparse
import ctypes
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import _native, kernels  # noqa: E402
from weatherconverter_amd.diffusion_model.config import model_config  # noqa: E402
from weatherconverter_amd.diffusion_model.models.unet_base import Unet  # noqa: E402
from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler  # noqa: E402
from weatherconverter_amd.synthetic import init_synthetic_  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--precision', default='bf16', choices=['fp32-class', 'f16', 'bf16'])
ap.add_argument('--batch', type=int, default=32)
ap.add_argument('--top', type=int, default=40)
args = ap.parse_args()

rec = []
_orig = _native.call
_ref_t = type(ctypes.byref(ctypes.c_int()))


def _shape(args_) -> str:
    a = args_[0] if args_ else None
    if isinstance(a, _ref_t):
        a = a._obj
    if isinstance(a, _native.ConvArgs):
        segs = ' + '.join(f'{a.seg[i].C}x{a.seg[i].ntaps}t' for i in range(a.nseg))
        return f'[{segs}] -> {a.N} @ {a.Hm}x{a.Wm}' + (' +res' if a.res else '')
    if isinstance(a, _native.WgradArgs):
        segs = ' + '.join(f'{a.seg[i].C}x{a.seg[i].ntaps}t' for i in range(a.nseg))
        return f'dW {a.M} x [{segs}] @ {a.Hm}x{a.Wm}'
    return ''


def call(fn, *a):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = _orig(fn, *a)
    e1.record()
    rec.append((fn, _native.last_kernel_name() or fn, _shape(a), e0, e1))
    return r


dev = torch.device('cuda', 0)
net = Unet(model_config(256))
init_synthetic_(net, seed=0)
if args.precision in ('f16', 'bf16'):
    net.set_train_precision(args.precision)
net = net.to(dev).train()
sched = LinearNoiseScheduler(1000, 0.0001, 0.02)
B = args.batch
g = torch.Generator().manual_seed(5)
img = (torch.rand((B, 3, 256, 256), generator=g) * 2 - 1).to(dev)
noise = torch.randn((B, 3, 256, 256), generator=g).to(dev)
t = torch.randint(0, 1000, (B, ), generator=g).to(dev)
crit = torch.nn.MSELoss()


def step():
    for p in net.parameters():
        p.grad = None
    loss = crit(net(sched.add_noise(img, noise, t), t), noise)
    loss.backward()


step()
torch.cuda.synchronize()
_native.call = call
runs = []
for _ in range(2):
    rec.clear()
    step()
    torch.cuda.synchronize()
    runs.append([(fn, name, shape, e0.elapsed_time(e1) * 1e3) for fn, name, shape, e0, e1 in rec])
n = min(len(r) for r in runs)
agg = defaultdict(lambda: [0, 0.0])
total = 0.0
for i in range(n):
    fn, name, shape, _ = runs[0][i]
    us = min(r[i][3] for r in runs)
    total += us
    k = (name[:64], shape)
    agg[k][0] += 1
    agg[k][1] += us
print(f'{n} launches, {total / 1e3:.2f} ms (events around each call)')
for (name, shape), (cnt, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
    print(f'{us / 1e3:8.3f} ms {cnt:4d} x {us / cnt:8.1f} us  {name:64s} {shape}')
