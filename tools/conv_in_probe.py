"""conv_in in the sampling step vs isolated: time wc_conv_in (B=16, 256 px, 3 -> 64 into a 128-channel
skip buffer) back to back, after a 1 GiB write that flushes L2 / MALL, and after a head-conv-sized read."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels as K  # noqa: E402


def ev_time(fn, pre=None, n=10):
    ts = []
    for _ in range(n):
        if pre:
            pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    B, S = 16, 256
    x = torch.randn((B, 3, S, S), device='cuda')
    w = torch.randn((64, 3, 3, 3), device='cuda').contiguous()
    b = torch.randn(64, device='cuda')
    U = torch.empty((B, S, S, 128), device='cuda')
    dense = torch.empty((B, S, S, 64), device='cuda')
    junk = torch.empty(1 << 28, device='cuda')
    big = torch.randn((B, S, S, 128), device='cuda')

    def flush():
        junk.fill_(1.0)

    def readbig():
        big.sum()

    for name, out in (('ldo128', K.View(U, 64, 64)), ('dense', K.View.full(dense))):
        f = lambda: K.conv_in(x, w, b, out)
        f()
        gp = K.GnPart.attach(out.t, 8) if name == 'ldo128' else None
        fg = lambda: K.conv_in(x, w, b, out, gn=gp)
        if gp is not None:
            print(f'{name}+gn: back-to-back {ev_time(fg):8.1f} us   after 1 GiB fill {ev_time(fg, flush):8.1f} us   '
                  f'after 512 MB read {ev_time(fg, readbig):8.1f} us   (separate gn_partials pass: '
                  f'{ev_time(lambda: K.gn_partials(out, gp)):8.1f} us)')
        torch.cuda.synchronize()
        print(f'{name}: back-to-back {ev_time(f):8.1f} us   after 1 GiB fill {ev_time(f, flush):8.1f} us   '
              f'after 512 MB read {ev_time(f, readbig):8.1f} us')
    gb = (x.numel() * 4 + dense.numel() * 4) / 1e9
    print(f'algorithmic {gb * 1e3:.1f} MB')


if __name__ == '__main__':
    main()
