"""Per-shape f16x3 3x3 conv timing (same per-workgroup work, different tensor sizes / batch) to
separate per-step cost from memory-system effects.  python tools/conv_shape_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import conv_case  # noqa: E402
from weatherconverter_amd import kernels as K  # noqa: E402

K._native.load()
for c in [(16, 256, 128, 128), (4, 256, 128, 128), (1, 256, 128, 128), (64, 128, 128, 128), (256, 64, 128, 128),
          (16, 128, 128, 128), (16, 64, 512, 512), (64, 64, 512, 512), (16, 256, 256, 128)]:
    t, tf, _ = conv_case(*c, prologue=True, res=0, mode='f3')
    B, H, Ci, Co = c
    wgs = B * (H // 8) * (H // 16) * ((Co + 127) // 128)
    print(f'B={B:3d} S={H:3d} {Ci}->{Co}: {t*1e3:7.3f} ms {tf:6.1f} TF/s  WGs={wgs}  act={B*H*H*Ci*4/1e6:.0f} MB', flush=True)
