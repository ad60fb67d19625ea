"""Where the training step's small torch ops come from: one config-3 training step under torch.profiler
(with_stack), the aten fill / zero / copy / cat / flip / elementwise ops counted by their innermost
weatherconverter_amd frame.  usage: train_op_sources.py [--batch 32]"""
import argparse
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = ('aten::fill_', 'aten::zero_', 'aten::copy_', 'aten::cat', 'aten::flip', 'aten::add', 'aten::mul', 'aten::sub',
       'aten::div', 'aten::clamp', 'aten::ones_like', 'aten::_to_copy', 'aten::where', 'aten::abs', 'aten::amax',
       'aten::ldexp', 'aten::stack', 'aten::floor', 'aten::log2', 'aten::zeros', 'aten::zeros_like', 'aten::full',
       'aten::ones', 'aten::new_zeros', 'aten::fill', 'aten::masked_fill_', 'aten::index_put_', 'aten::scatter_')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    a = ap.parse_args()
    from weatherconverter_amd import kernels
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.synthetic import init_synthetic_
    dev = torch.device('cuda', 0)
    net = Unet(model_config(256))
    init_synthetic_(net, seed=0)
    net = net.to(dev).train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    crit = torch.nn.MSELoss()
    sched = LinearNoiseScheduler(1000, 0.0001, 0.02)
    B = a.batch
    img = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1
    noise = kernels.philox_normal((B, 3, 256, 256), dev, 1, step=0)
    t = torch.randint(0, 1000, (B, ), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = crit(net(sched.add_noise(img, noise, t), t), noise)
        loss.backward()
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    cnt = Counter()

    class Count(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.overloadpacket.__name__)
            if any(name == o.split('::')[1] for o in OPS):
                frame = '?'
                for fr in reversed(traceback.extract_stack()):
                    f = fr.filename
                    if ('weatherconverter_amd' in f or '/tools/' in f or 'torch/optim' in f) \
                            and '_python_dispatch' not in f and 'train_op_sources' not in f:
                        frame = f"{f.split('repo/')[-1]}:{fr.lineno}"
                        break
                cnt[(name, frame)] += 1
            return func(*args, **(kwargs or {}))

    with Count():
        step()
        torch.cuda.synchronize()
    for (name, frame), n in cnt.most_common(60):
        print(f'{n:5d}  {name:18s} {frame}', flush=True)


if __name__ == '__main__':
    main()
