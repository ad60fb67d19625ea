"""BASELINE config 3 measurement: one training-loss iteration (train_ddpm.py:94-108: add_noise + UNet
forward + MSE) at 256 px, B=32, per-sample timesteps, HIP-graph replay; prints one JSON line.

  python tools/bench_train.py [--batch 32] [--steps 20] [--warmup 3]

The backward and the optimizer step are not part of config 3 as BASELINE.json states it ("forward
add_noise + UNet + MSE"); the arithmetic is the engine's fp32-class mode (>= the config's bf16).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GFLOP_PER_IMAGE_STEP_256 = 590.61


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--seed', type=int, default=3455)
    args = ap.parse_args()
    from weatherconverter_amd import kernels
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.diffusion_model.train_ddpm import TrainForward
    from weatherconverter_amd.synthetic import init_synthetic_
    dev = torch.device('cuda', 0)
    mc = model_config(args.size)
    net = Unet(mc)
    init_synthetic_(net, seed=0)
    net = net.to(dev).train()
    sched = LinearNoiseScheduler(1000, 0.0001, 0.02)
    B, S = args.batch, args.size
    g = torch.Generator().manual_seed(args.seed)
    # a few distinct synthetic batches (images ~ U[-1, 1], noise ~ N(0, 1), t ~ U[0, 1000)), resident on
    # the device before the timed region
    nb = 4
    imgs = [(torch.rand((B, 3, S, S), generator=g) * 2 - 1).to(dev) for _ in range(nb)]
    noises = [kernels.philox_normal((B, 3, S, S), dev, args.seed, step=i) for i in range(nb)]
    ts = [torch.randint(0, 1000, (B, ), generator=g).to(dev) for _ in range(nb)]
    step = TrainForward(net, sched, imgs[0], noises[0], ts[0])
    losses = []
    for i in range(args.warmup):
        step(imgs[i % nb], noises[i % nb], ts[i % nb])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        losses.append(step(imgs[i % nb], noises[i % nb], ts[i % nb]).clone())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = el / args.steps * 1e3
    print(json.dumps({
        'metric': 'train_ddpm config 3: training-loss iterations/s (add_noise + UNet fwd + MSE)',
        'value': round(args.steps / el, 3), 'unit': 'iter/s', 'ms_per_iter': round(ms, 3),
        'images_per_s': round(B * args.steps / el, 2), 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
        'higher_is_better': True, 'dtype': 'f32 (fp32-class split-precision MFMA, f16x3/bf16x6)',
        'data': 'synthetic (keyed random-init weights; images U[-1,1], Philox N(0,1) noise, t ~ U[0,1000))',
        'config': {'workload': 'BASELINE config 3 forward', 'global_batch': B, 'image_size': S,
                   'hip_graph': True, 'backward': False},
        'unet_tflops_algorithmic': round(GFLOP_PER_IMAGE_STEP_256 * B / (ms * 1e-3) / 1e3, 1) if S == 256 else None,
        'loss_finite': bool(torch.isfinite(torch.stack(losses)).all()),
        'loss_mean': float(torch.stack(losses).mean()),
    }))


if __name__ == '__main__':
    main()
