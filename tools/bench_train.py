"""BASELINE config 3 measurement at 256 px, B=32, per-sample timesteps; prints one JSON line.

  python tools/bench_train.py [--mode step|forward] [--batch 32] [--steps 10] [--warmup 2]

mode 'step' (default): the reference's whole training iteration (train_ddpm.py:94-114) —
    opt.zero_grad(); noisy = scheduler.add_noise(images, noise, t); pred = model(noisy, t);
    loss = MSELoss()(pred, noise); loss.backward(); opt.step()
  with the HIP forward-with-tape and HIP backward (models/train_engine.py) and torch Adam, timed per
  phase with events.  Arithmetic (the model's conv precision, f16x3 by default): forward convs,
  projections and attention f16x3 under static range bounds (GroupNorm, in-projection row norms),
  data-gradient convs f16x3 under per-image absmax bounds of the gradient, weight gradients and the
  attention backward bf16x6 (fp32 MFMA at head dim 192); all fp32-class and checked against float64
  autograd.
mode 'forward': the training-loss forward only (add_noise + UNet fwd + MSE), HIP-graph replay (the
  round-1 line).
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
    ap.add_argument('--mode', default='step', choices=['step', 'forward'])
    ap.add_argument('--profile', action='store_true', help='per-kernel-class event times of one step')
    ap.add_argument('--no-roofline', action='store_true', help='skip the per-kernel roofline leg')
    ap.add_argument('--no-cpu-baseline', action='store_true', help='skip the CPU reference-iteration leg')
    ap.add_argument('--cpu-batch', type=int, default=1, help='CPU baseline batch (a bounded sample of B)')
    ap.add_argument('--precision', default='fp32-class', choices=['fp32-class', 'f16', 'bf16'],
                    help="'bf16' / 'f16': the 16-bit training lines (Unet.set_train_precision, single-piece builds)")
    args = ap.parse_args()
    if args.mode == 'step':
        return train_step(args)
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


DTYPES = {
    'fp32-class': 'fp32-class (f16x3: forward convs, projections, attention; data and weight gradients and the '
                  'attention backward under per-image range bounds raised by the gradients\' writers; bf16x6 where '
                  'no bound exists; fp32 MFMA for the dK/dV of head dim 192)',
    'f16': '16-bit line (the f16x3 kernels with one fp16 piece per operand, fp32 accumulation, power-of-two range '
           'scaling; bf16x6 / fp32 MFMA where no bound exists)',
    'bf16': 'bf16 (BASELINE config 3): the f16x3 kernels with one bf16 piece per operand on the bf16 MFMA, fp32 '
            'accumulation; bf16x6 / fp32 MFMA where no bound exists',
}


def train_step(args):
    from weatherconverter_amd import kernels
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.synthetic import init_synthetic_
    dev = torch.device('cuda', 0)
    mc = model_config(args.size)
    net = Unet(mc)
    init_synthetic_(net, seed=0)
    if args.precision in ('f16', 'bf16'):
        net.set_train_precision(args.precision)
    net = net.to(dev).train()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)  # train_ddpm.py:176 (lr from config.yaml)
    crit = torch.nn.MSELoss()
    sched = LinearNoiseScheduler(1000, 0.0001, 0.02)
    B, S = args.batch, args.size
    g = torch.Generator().manual_seed(args.seed)
    nb = 4
    imgs = [(torch.rand((B, 3, S, S), generator=g) * 2 - 1).to(dev) for _ in range(nb)]
    noises = [kernels.philox_normal((B, 3, S, S), dev, args.seed, step=i) for i in range(nb)]
    ts = [torch.randint(0, 1000, (B, ), generator=g).to(dev) for _ in range(nb)]

    def step(i, ev=None):
        opt.zero_grad(set_to_none=True)
        noisy = sched.add_noise(imgs[i % nb], noises[i % nb], ts[i % nb])
        pred = net(noisy, ts[i % nb])
        loss = crit(pred, noises[i % nb])
        if ev:
            ev[0].record()
        loss.backward()
        if ev:
            ev[1].record()
        opt.step()
        return loss.detach()

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    losses, evs = [], []
    t0 = time.perf_counter()
    for i in range(args.steps):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[2].record()
        losses.append(step(i, (e[0], e[1])))
        evs.append(e)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = el / args.steps * 1e3
    fwd = sum(e[2].elapsed_time(e[0]) for e in evs) / len(evs)
    bwd = sum(e[0].elapsed_time(e[1]) for e in evs) / len(evs)
    roof = None if args.no_roofline else roofline_leg(kernels, step, args.precision, ms)
    cpu = None if args.no_cpu_baseline else cpu_baseline_leg(args)
    prof = None
    if args.profile:
        rec = kernels.profile_conv(True)
        step(0)
        torch.cuda.synchronize()
        kernels.profile_conv(False)
        per = {}
        for name, flops, e0, e1, *_ in rec:
            key = name.split('<')[0].split(' ')[0]
            d = per.setdefault(key, [0, 0.0, 0.0])
            d[0] += 1
            d[1] += flops
            d[2] += e0.elapsed_time(e1)
        prof = {k: {'launches': v[0], 'ms': round(v[2], 2), 'tflops_or_gbs': round(v[1] / (v[2] * 1e-3) / 1e12, 1)}
                for k, v in sorted(per.items(), key=lambda kv: -kv[1][2])}
    ls = torch.stack(losses)
    print(json.dumps({
        'metric': 'train_ddpm config 3: training iterations/s (add_noise + UNet fwd + MSE + backward + Adam)',
        'value': round(args.steps / el, 4), 'unit': 'iter/s', 'ms_per_iter': round(ms, 2),
        'ms_forward': round(fwd, 2), 'ms_backward': round(bwd, 2), 'ms_adam_and_host': round(ms - fwd - bwd, 2),
        'images_per_s': round(B * args.steps / el, 2), 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
        'higher_is_better': True,
        'dtype': DTYPES[args.precision],
        'data': 'synthetic (keyed random-init weights; images U[-1,1], Philox N(0,1) noise, t ~ U[0,1000))',
        'config': {'workload': 'BASELINE config 3 full training iteration', 'global_batch': B, 'image_size': S,
                   'backward': True, 'optimizer': 'torch.optim.Adam lr 1e-4', 'precision': args.precision},
        'train_tflops_algorithmic': round(3 * GFLOP_PER_IMAGE_STEP_256 * B / (ms * 1e-3) / 1e3, 1) if S == 256 else None,
        'loss_finite': bool(torch.isfinite(ls).all()), 'loss_first': float(ls[0]), 'loss_last': float(ls[-1]),
        'roofline': roof,
        'cpu_baseline': cpu,
        'kernel_classes': prof,
    }))


def roofline_leg(kernels, step, precision: str, ms_iter: float):
    """One training iteration with HIP events around every named launch (kernels.profile_conv): the
    dominant instantiation by time is the roofline kernel; achieved = its algorithmic FLOPs per launch
    (fp32-equivalent) / its mean duration, against its arithmetic's ceiling on this line: on the 16-bit
    lines the split-precision templates compute with ONE 16-bit piece (the dense bf16 / f16 MFMA peak,
    2516.6 TF/s); on the fp32-class line f16x3 (/3), bf16x6 (/6) or fp32 MFMA (bench.py _mode_peak).
    Beside it the whole iteration's algorithmic rate (3x the forward's FLOPs) against the same peak."""
    import bench
    rec = kernels.profile_conv(True)
    torch.cuda._sleep(1 << 28)  # the host enqueues the whole iteration ahead of the GPU: events bracket kernels
    step(0)
    torch.cuda.synchronize()
    kernels.profile_conv(False)
    per = {}
    for name, flops, e0, e1, *_ in rec:
        d = per.setdefault(name, [0, 0.0, 0.0])
        d[0] += 1
        d[1] += flops
        d[2] += e0.elapsed_time(e1) * 1e-3

    def peak(name):
        p = bench._mode_peak(name)
        return bench.DENSE16_PEAK_TFLOPS if (precision in ('bf16', 'f16') and p == bench.F16X3_PEAK_TFLOPS) else p
    mfma = {k: v for k, v in per.items() if v[1] > 0 and ('conv' in k or 'attn' in k or 'attention' in k
                                                          or 'proj' in k or 'wgrad' in k)}
    name = max(mfma, key=lambda k: mfma[k][2])
    n, fl, sec = mfma[name]
    ach = fl / n / (sec / n) / 1e12
    top = sorted(mfma.items(), key=lambda kv: -kv[1][2])[:12]
    iter_peak = bench.DENSE16_PEAK_TFLOPS if precision in ('bf16', 'f16') else bench.F16X3_PEAK_TFLOPS
    it = 3 * GFLOP_PER_IMAGE_STEP_256 * 32 / (ms_iter * 1e-3) / 1e3
    return {
        'kernel': name, 'bound': 'mfma', 'achieved': round(ach, 1), 'peak': peak(name), 'unit': 'TFLOP/s',
        'frac': round(ach / peak(name), 4), 'traffic': None, 'launches_per_iter': n,
        'mean_launch_ms': round(sec / n * 1e3, 4), 'gflop_per_launch': round(fl / n / 1e9, 2),
        'mean_launch_ms_source': 'HIP events around each launch of one iteration (kernels.profile_conv), host '
                                 'enqueue ahead of the GPU',
        'iteration': {'tflops_algorithmic': round(it, 1), 'peak': iter_peak, 'frac': round(it / iter_peak, 4),
                      'flops': '3 x the forward (590.61 GFLOP per 256-px image, SURVEY.md 8(d)) x 32 images'},
        'top_kernels': {k: {'launches': v[0], 'ms': round(v[2] * 1e3, 2), 'tflops': round(v[1] / v[2] / 1e12, 1),
                            'peak': peak(k), 'frac': round(v[1] / v[2] / 1e12 / peak(k), 4)} for k, v in top},
        'named_launch_ms': round(sum(v[2] for v in per.values()) * 1e3, 2),
    }


def cpu_baseline_leg(args):
    """The reference training iteration (train_ddpm.py:94-114: add_noise, UNet forward, MSE, backward;
    Adam excluded) on the CPU: the oracle's op-for-op PyTorch restatement of unet_base.Unet with autograd,
    fp32, at a bounded sample of the batch (--cpu-batch images at the same size), on the CPUs this process
    may use, one timed iteration after one warm-up; value = iterations/s scaled to the GPU line's batch."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from oracle.unet_oracle import unet_forward, unet_state_dict_keys
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.synthetic import synth_tensor
    share = bench._cpu_share()
    torch.set_num_threads(share['usable_cpus'])
    mc = model_config(args.size)
    sd = {k: synth_tensor(k, s).requires_grad_() for k, s in unet_state_dict_keys(mc).items()}
    B = args.cpu_batch
    g = torch.Generator().manual_seed(5)
    x0 = torch.rand((B, 3, args.size, args.size), generator=g) * 2 - 1
    nz = torch.randn(x0.shape, generator=g)
    t = torch.randint(0, 1000, (B, ), generator=g)
    acp = torch.cumprod(1 - torch.linspace(0.0001, 0.02, 1000), 0)

    def it():
        noisy = acp[t].sqrt()[:, None, None, None] * x0 + (1 - acp[t]).sqrt()[:, None, None, None] * nz
        loss = torch.nn.functional.mse_loss(unet_forward(sd, mc, noisy, t), nz)
        loss.backward()
        for v in sd.values():
            v.grad = None
    it()
    t0 = time.perf_counter()
    it()
    dt = time.perf_counter() - t0
    return {'value': round(B / args.batch / dt, 6), 'unit': 'iter/s', 'cores': share['usable_cpus'], 'kind': 'port',
            'ms_per_iter_sample': round(dt * 1e3, 1), 'host': share,
            'sample': f'oracle PyTorch-CPU restatement of the reference iteration (add_noise + UNet forward + MSE + '
                      f'autograd backward, no Adam), {args.size}px, B={B} of the line\'s {args.batch}, 1 timed '
                      f'iteration after 1 warm-up; iterations/s scaled by {B}/{args.batch}'}


if __name__ == '__main__':
    main()
