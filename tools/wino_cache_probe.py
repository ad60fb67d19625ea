"""Winograd conv time per image against the batch (input tensor 34 MB ... 537 MB at 256 px, 128 channels):
whether the K loop waits on HBM for its halo loads once the input no longer fits the 256 MB Infinity
Cache.  Each launch is timed back to back 10x (the input stays wherever the previous launch left it)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import conv_case  # noqa: E402

for (H, Ci, Co) in ((256, 128, 128), (128, 256, 256), (64, 512, 512)):
    for B in (1, 2, 4, 8, 16, 32):
        t, fl, _ = conv_case(B, H, Ci, Co, mode='wino')
        mb = B * H * H * Ci * 4 / 2**20
        print(f'{H}^2 {Ci}->{Co} B={B:2d} input {mb:7.1f} MiB: {t * 1e6:8.1f} us  {t * 1e6 / B:7.2f} us/image  '
              f'{fl / t / 1e12:6.1f} TF/s', flush=True)
