"""Swift-SRGAN x4 generator timing on the HIP engine (256 -> 1024 and 128 -> 512, B=1, the guided
translation loop's shapes, translation.py:81); prints one line per shape."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from weatherconverter_amd.srgan_model.models import Generator
    from weatherconverter_amd.synthetic import init_synthetic_
    gen = Generator()
    init_synthetic_(gen, seed=0)
    gen = gen.cuda().eval()
    for S in (128, 256):
        x = torch.rand((1, 3, S, S), device='cuda')
        for _ in range(3):
            gen(x)
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            y = gen(x)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        print(f'srgan x4 {S}->{4 * S}: {ms:.3f} ms/image  out {tuple(y.shape)} finite={bool(torch.isfinite(y).all())}',
              flush=True)


if __name__ == '__main__':
    main()
