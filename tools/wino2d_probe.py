"""EXPERIMENTAL 2D Winograd F(2x2,3x3) conv1 against the shipped F(2,3)-along-x kernel and the
direct f16x3 kernel on the ResBlock conv1 shapes of the 256x256 UNet at B=16 (GN+SiLU prologue, no
residual), with each one's rel-L2 against torch's fp32 conv (tf32 off) as a sanity column."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import conv_case  # noqa: E402
from weatherconverter_amd import kernels as K  # noqa: E402

K._native.load()
for B, S, Ci, Co in ((16, 256, 128, 128), (16, 128, 128, 256), (16, 128, 256, 256), (16, 64, 256, 512),
                     (16, 64, 512, 512), (16, 32, 512, 768), (16, 32, 768, 768), (16, 32, 1024, 256)):
    for mode in ('wino2d', 'wino', 'f3'):
        t, tf, err = conv_case(B, S, Ci, Co, True, 0, check=True, mode=mode)
        print(f'{mode:7s} B={B} S={S:3d} {Ci}->{Co}: {t * 1e3:8.3f} ms  {tf:6.1f} TF/s(direct-eq)  err {err:.2e}',
              flush=True)
