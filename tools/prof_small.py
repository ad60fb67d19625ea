"""Small-batch UNet forward for a kernel trace: python tools/prof_small.py [size] [batch] [steps]."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd.diffusion_model.config import model_config  # noqa: E402
from weatherconverter_amd.diffusion_model.models.unet_base import Unet  # noqa: E402
from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep  # noqa: E402
from weatherconverter_amd.synthetic import init_synthetic_  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
net = Unet(model_config(S))
init_synthetic_(net, seed=0)
net = net.cuda().eval()
x = torch.randn((B, 3, S, S), device='cuda')
t = torch.tensor([10], device='cuda')
with torch.no_grad():
    run = _GraphStep(net, x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        run(x, t)
    torch.cuda.synchronize()
print(f'S={S} B={B}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per forward (graph)')
