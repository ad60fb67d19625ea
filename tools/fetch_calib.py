"""FETCH_SIZE calibration on this box: wc_absmax_images reads a 4 GiB fp32 tensor once with 16-byte
loads per lane (nothing else); run under rocprofv3 --pmc FETCH_SIZE and compare the counter with 4 GiB
(MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of such reads).  A 2 GiB write between launches
evicts the tensor from L2 / MALL."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels as K  # noqa: E402
from weatherconverter_amd.kernels import View  # noqa: E402

x = torch.randn((16, 256, 256, 1024), device='cuda')  # 4 GiB
junk = torch.empty(1 << 29, device='cuda')  # 2 GiB
for _ in range(3):
    junk.fill_(1.0)
    K.absmax_images(View.full(x))
torch.cuda.synchronize()
print('bytes per launch', x.numel() * 4)
