"""BASELINE config 4 at length: one complete guided translation (reference translation.py:46-97,
``sample_with_sgg``) timed end to end on one MI355X.

Workload: 256-px UNet (config.yaml model) + scheduler on the HIP engine, Swift-SRGAN x4 (256 -> 1024)
and DeepLabV3+ R101 (19 classes, OS16) input gradient at 1024^2 in PyTorch-ROCm (north_star), the
wc_sgg_update kernel; N = 500 reverse steps over the T = 1000 schedule, lambda = 60, GSG on every odd
step (translation.py:84-87), B = 1 (the reference's batch-1 semantics, D4).  Synthetic keyed weights
(no checkpoints ship), input image U[-1, 1], gt ~ randint(0, 19) with 5 % ignore (255).

Prints one JSON line per run: the whole sample_with_sgg call (both modes: 'reference' = the
reference's effective output, guidance computed then overwritten, D1; 'applied' = the guided latent
kept), plus a bounded LCG sample (apply_lcg mode 'applied', 19 class-masked DeepLab passes per even
step; the reference crashes there, D3) extrapolated to the 250 even steps.
    python tools/bench_guided.py [--n 500] [--miopen-benchmark 1] [--lcg-steps 2]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=500)
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--miopen-benchmark', type=int, default=1,
                    help='torch.backends.cudnn.benchmark for the segmenter (MIOpen find with its own workspace)')
    ap.add_argument('--lcg-steps', type=int, default=2)
    ap.add_argument('--modes', default='reference,applied')
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.miopen_benchmark)
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.seg_model.network import deeplabv3plus_resnet101
    from weatherconverter_amd.sgg.sgg import apply_lcg
    from weatherconverter_amd.srgan_model.models import Generator
    from weatherconverter_amd.srgan_model.models import inference as srgan_inference
    from weatherconverter_amd.synthetic import init_synthetic_
    from weatherconverter_amd.translation import sample_with_sgg
    dev = torch.device('cuda', 0)
    S = a.size
    unet = Unet(model_config(S))
    init_synthetic_(unet, seed=0)
    unet = unet.to(dev).eval()
    sr = Generator()
    init_synthetic_(sr, seed=1)
    sr = sr.to(dev).eval()
    seg = deeplabv3plus_resnet101(num_classes=19, output_stride=16, pretrained_backbone=False)
    init_synthetic_(seg, seed=2)
    seg = seg.to(dev).eval()
    sched = LinearNoiseScheduler(1000, 0.0001, 0.02, device=dev)
    g = torch.Generator().manual_seed(3455)
    x_in = torch.rand((1, 3, S, S), generator=g) * 2 - 1
    gt = torch.randint(0, 19, (1, 4 * S, 4 * S), generator=g)
    gt[torch.rand(gt.shape, generator=g) < 0.05] = 255
    gt = gt.to(dev)
    t_start = torch.tensor([a.n - 1])  # the full N-step loop (translation.py:63 draws t ~ U[0, N))
    noise = torch.randn((1, 3, S, S), generator=g)
    # warm-up: MIOpen find / kernel loads / graph capture outside the timed call (N=4 loop)
    sample_with_sgg(x_in, unet, sched, seg, gt, sr, N=4, mode='applied', t_start=torch.tensor([3]), noise=noise)
    torch.cuda.synchronize()
    for mode in a.modes.split(','):
        steps = {'n': 0}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out, lat = sample_with_sgg(x_in, unet, sched, seg, gt, sr, N=a.n, mode=mode, t_start=t_start, noise=noise,
                                   return_latent=True, progress=lambda i: steps.__setitem__('n', steps['n'] + 1))
        torch.cuda.synchronize()
        sec = time.perf_counter() - t0
        print(json.dumps({
            'config': 4, 'metric': 'guided translation wall time (sample_with_sgg, complete N-step loop)',
            'value': round(sec, 3), 'unit': 's', 'higher_is_better': False, 'mode': mode, 'N': a.n,
            'gsg_steps': a.n // 2, 'steps_run': steps['n'] + 1, 'ms_per_step': round(sec / a.n * 1e3, 2),
            'workload': f'{S}-px UNet (HIP, HIP graph) + Swift-SRGAN x4 to {4 * S}^2 + DeepLabV3+ R101 input gradient '
                        f'at {4 * S}^2 (PyTorch-ROCm) + wc_sgg_update, B=1, lambda=60, GSG on odd steps',
            'miopen_benchmark': bool(a.miopen_benchmark), 'sr_out_shape': list(out.shape),
            'out_finite': bool(torch.isfinite(out).all() and torch.isfinite(lat).all()),
            'data': 'synthetic keyed weights, U[-1,1] input, gt randint(0,19) + 5% ignore'}), flush=True)
    if a.lcg_steps > 0:
        xt = torch.randn((1, 3, S, S), device=dev)
        mu, sigma = xt * 0.9, xt * 0.01
        with torch.no_grad():
            sr_xt = srgan_inference(sr, xt)
        apply_lcg(seg, mu, sigma, sr_xt, gt, 60.0, mode='applied')
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.lcg_steps):
            apply_lcg(seg, mu, sigma, sr_xt, gt, 60.0, mode='applied')
        torch.cuda.synchronize()
        lcg = (time.perf_counter() - t0) / a.lcg_steps
        print(json.dumps({'config': 4, 'metric': 'apply_lcg (applied mode) per even step', 'value': round(lcg * 1e3, 1),
                          'unit': 'ms', 'timed_calls': a.lcg_steps,
                          'extrapolated_lcg_s_for_N': round(lcg * (a.n - a.n // 2), 1),
                          'note': 'reference apply_lcg crashes at sgg/sgg.py:58 (D3); 19 class-masked DeepLab '
                                  'input-gradient passes per call'}), flush=True)


if __name__ == '__main__':
    main()
