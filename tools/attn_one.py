"""One pre-split f16x3 attention shape (argv: N C heads B [reps]) launched `reps` times on random fp16
pieces (the product entry point wc_attention_fwd_f16x3_presplit_a3): the single-kernel subject of a PMC
pass or an A/B.  Default: the 64x64 attention of the 256-px UNet (N 4096, C 512, 4 heads, B 16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels as K  # noqa: E402

a = [int(x) for x in sys.argv[1:]]
N, C, heads, B = (a + [4096, 512, 4, 16][len(a):])[:4]
reps = a[4] if len(a) > 4 else 10
g = torch.Generator(device='cuda').manual_seed(0)
qkv3 = torch.randn(B * 6 * C * N, device='cuda', generator=g).half().view(torch.int16)
exps = (0, 0, 0)
K.attention_presplit_a3(qkv3, B, N, C, heads, exps)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    K.attention_presplit_a3(qkv3, B, N, C, heads, exps)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / reps
fl = 4.0 * B * N * N * C
print(f'N {N} C {C} heads {heads} B {B}: {us:.1f} us  {fl / us / 1e6:.1f} TF/s fp32-equivalent  '
      f'{3 * fl / us / 1e6:.1f} TF/s f16 issued')
