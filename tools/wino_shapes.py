"""The Winograd conv launches of one 256-px sampling forward (B=16): input / residual channels, output
channels and size, and each launch's time (events), to see where the residual tail forms sit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels as K  # noqa: E402
from weatherconverter_amd.diffusion_model.config import model_config  # noqa: E402
from weatherconverter_amd.diffusion_model.models.unet_base import Unet  # noqa: E402
from weatherconverter_amd.synthetic import init_synthetic_  # noqa: E402

rec = []


def tracer(fn, tag):
    def traced(segs, w, bias, out, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn(segs, w, bias, out, **kw)
        e1.record()
        rec.append((tag, segs[0].view.C, segs[1].view.C if len(segs) > 1 else 0, out.C, kw['Hm'], e0, e1))
        return r
    return traced


# the Winograd convs and the direct halo convs (WINO_SHAPES_DIRECT=1 adds the latter)
K.conv3x3_wino = tracer(K.conv3x3_wino, 'wino')
if os.environ.get('WINO_SHAPES_DIRECT', '0') == '1':
    K.conv3x3_f16x3 = tracer(K.conv3x3_f16x3, 'direct')
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
agg = {}
for i, (tag, c0, c1, co, h, e0, e1) in enumerate(rec):
    k = (i % n, tag, c0, c1, co, h)
    agg.setdefault(k, []).append(e0.elapsed_time(e1) * 1e3)
tot = 0
for (i, tag, c0, c1, co, h), ts in sorted(agg.items()):
    m = min(ts)
    tot += m
    fl = 2.0 * 16 * h * h * co * (9 * c0 + c1)
    print(f'{i:2d} {tag:6s} {h:4d}^2 {c0:4d} (+res {c1:4d}) -> {co:4d}: {m:7.1f} us  {fl / m / 1e6:6.1f} TF/s', flush=True)
print(f'total {tot / 1e3:.3f} ms over {n} launches')
