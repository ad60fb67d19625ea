"""One Winograd conv shape (argv: H Ci Co B [res]) launched 10x: the single-kernel subject of a PMC pass."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import conv_case  # noqa: E402

H, Ci, Co, B = (int(a) for a in sys.argv[1:5])
res = int(sys.argv[5]) if len(sys.argv) > 5 else 0
t, _, _ = conv_case(B, H, Ci, Co, res=res, mode='wino')
print(f'{H}^2 {Ci}->{Co} (+res {res}) B={B}: {t * 1e6:.1f} us')
