"""DeepLabV3+ R101 (OS16, 19 classes) forward + input gradient at 1024^2, B=1 (the config-4 guidance
pass): eager vs captured into a HIP graph over static input / label buffers.  Prints both times and
whether the gradients agree bitwise."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd.seg_model.inference import input_gradient  # noqa: E402
from weatherconverter_amd.seg_model.network import deeplabv3plus_resnet101  # noqa: E402
from weatherconverter_amd.synthetic import init_synthetic_  # noqa: E402


def ev(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device('cuda', 0)
    seg = deeplabv3plus_resnet101(num_classes=19, output_stride=16, pretrained_backbone=False)
    init_synthetic_(seg, seed=2)
    seg = seg.to(dev).eval()
    g = torch.Generator().manual_seed(5)
    x = (torch.rand((1, 3, 1024, 1024), generator=g) * 2 - 1).to(dev)
    gt = torch.randint(0, 19, (1, 1024, 1024), generator=g)
    gt[torch.rand(gt.shape, generator=g) < 0.05] = 255
    gt = gt.to(dev)
    eager_ms = ev(lambda: input_gradient(seg, x, gt), 8)
    ref, _ = input_gradient(seg, x, gt)
    xs, gs = x.clone(), gt.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            out, _ = input_gradient(seg, xs, gs)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out, _ = input_gradient(seg, xs, gs)
    graph_ms = ev(graph.replay, 8)
    graph.replay()
    torch.cuda.synchronize()
    d = (out - ref).abs().max().item()
    print(f'deeplab fwd + input grad 1024^2: eager {eager_ms:.3f} ms, graph {graph_ms:.3f} ms, '
          f'bitwise {torch.equal(out, ref)}, max |diff| {d:.3e}, |ref| max {ref.abs().max().item():.3e}', flush=True)


if __name__ == '__main__':
    main()
