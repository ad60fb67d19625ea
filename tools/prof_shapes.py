"""Per-launch-shape event times of one UNet forward (256 px, B=16): groups the profiled launches by
(kernel instantiation, algorithmic work per launch) and prints ms, launches and the achieved rate."""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from weatherconverter_amd import kernels
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.synthetic import init_synthetic_
    mc = model_config(256)
    net = Unet(mc)
    init_synthetic_(net, seed=0)
    net = net.cuda().eval()
    x = kernels.philox_normal((16, 3, 256, 256), torch.device('cuda'), 1)
    t = torch.tensor([500], device='cuda')
    with torch.no_grad():
        net(x, t)
        torch.cuda.synchronize()
        prof = kernels.profile_conv(True)
        torch.cuda._sleep(1 << 28)
        net(x, t)
        torch.cuda.synchronize()
        kernels.profile_conv(False)
    agg = defaultdict(lambda: [0, 0.0])
    for name, work, e0, e1, *_ in prof:
        a = agg[(name, work)]
        a[0] += 1
        a[1] += e0.elapsed_time(e1)
    tot = sum(v[1] for v in agg.values())
    print(f'total event ms {tot:.3f}')
    for (name, work), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        unit = 'GB/s' if name.startswith('gn_') else 'TF/s'
        rate = work * n / (ms * 1e-3) / (1e9 if unit == 'GB/s' else 1e12)
        print(f'{ms:8.3f} ms  {n:3d}x  {work / (1e9 if unit == "GB/s" else 1e9):9.3f} G/launch  {rate:8.1f} {unit}  {name}')


if __name__ == '__main__':
    main()
