"""Where the training iteration's small torch kernels (fills, copies, elementwise) come from: one iteration
under torch.profiler with Python stacks, device time of the non-HIP-extension kernels grouped by the
innermost repo source line that launched them."""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels  # noqa: E402
from weatherconverter_amd.diffusion_model.config import model_config  # noqa: E402
from weatherconverter_amd.diffusion_model.models.unet_base import Unet  # noqa: E402
from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler  # noqa: E402
from weatherconverter_amd.synthetic import init_synthetic_  # noqa: E402

dev = torch.device('cuda', 0)
net = Unet(model_config(256))
init_synthetic_(net, seed=0)
net = net.to(dev).train()
opt = torch.optim.Adam(net.parameters(), lr=1e-4)
crit = torch.nn.MSELoss()
sched = LinearNoiseScheduler(1000, 0.0001, 0.02)
B = 32
g = torch.Generator().manual_seed(0)
img = (torch.rand((B, 3, 256, 256), generator=g) * 2 - 1).to(dev)
noise = kernels.philox_normal((B, 3, 256, 256), dev, 0, step=0)
ts = torch.randint(0, 1000, (B, ), generator=g).to(dev)


def step():
    opt.zero_grad(set_to_none=True)
    pred = net(sched.add_noise(img, noise, ts), ts)
    crit(pred, noise).backward()
    opt.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
rows = []
for e in prof.key_averages(group_by_stack_n=12):
    dt = getattr(e, 'self_device_time_total', None)
    if dt is None:
        dt = e.self_cuda_time_total
    if dt <= 0 or not e.key.startswith('aten::'):
        continue
    st = [f for f in (e.stack or []) if 'weatherconverter_amd' in f or 'tools/' in f]
    rows.append((dt, e.count, e.key, st[0] if st else '?'))
rows.sort(reverse=True)
print(f'aten ops with device time: {sum(r[0] for r in rows) / 1e3:.2f} ms')
for dt, c, k, site in rows[:45]:
    print(f'{c:5d} {dt / 1e3:8.3f} ms  {k:28s} {site[-100:]}')
