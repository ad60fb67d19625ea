"""Cost of the Winograd conv's residual chunks: the same 3x3 conv with no residual, a residual of as many
chunks as the 3x3 segment (all interleaved) and of twice as many (half of them in the serial tail)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import conv_case  # noqa: E402
from weatherconverter_amd import kernels as K  # noqa: E402

K._native.load()
for B, S, C in ((16, 128, 128), (16, 64, 256), (16, 32, 512)):
    for res in (0, C, 2 * C):
        t, tf, _ = conv_case(B, S, C, C, True, res, mode='wino')
        print(f'wino B={B} S={S} {C}->{C} res={res}: {t * 1e3:8.3f} ms  {tf:6.1f} TF/s', flush=True)
