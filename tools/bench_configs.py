"""BASELINE.json configs 1, 3 and 4 on one MI355X (config 2 is bench.py's line; config 5 is bench.py
under torch.distributed.run on 8 GPUs).  Prints one JSON object per config.

  config 1  64 px UNet, B=2, T=50 full sample (sample_ddpm.py) on the HIP engine; beside it the
            oracle's PyTorch-CPU restatement of the same loop (the reference's own CPU path).
  config 3  train_ddpm.py forward at 256 px, B=32 (tools/bench_train.py).
  config 4  sample_integrated/translation guided step at 256 px: UNet + scheduler (HIP), Swift-SRGAN
            x4 256 -> 1024 (HIP), DeepLabV3+ R101 forward + input gradient at 1024^2 (PyTorch-ROCm,
            north_star) + the wc_sgg_update kernel; N=500 steps (GSG on odd steps, translation.py:56),
            reported per step kind and extrapolated to the N=500 loop.
Synthetic keyed weights everywhere (no checkpoints offline).

  python tools/bench_configs.py [--configs 1,3,4] [--guided-steps 4]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _sync():
    torch.cuda.synchronize()


def run_config1(dev):
    from oracle.unet_oracle import unet_forward
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.sample_ddpm import sample_tensor
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.synthetic import init_synthetic_
    mc = model_config(64)
    net = Unet(mc)
    init_synthetic_(net, seed=0)
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    net = net.to(dev).eval()
    T, B = 50, 2
    sched = LinearNoiseScheduler(T, 0.0001, 0.02, device=dev)
    with torch.no_grad():
        sample_tensor(net, sched, B, 3, 64, noise='philox', seed=3455, graph=True)  # warm (capture)
        _sync()
        t0 = time.perf_counter()
        x0 = sample_tensor(net, sched, B, 3, 64, noise='philox', seed=3455, graph=True)
        _sync()
        gpu_s = time.perf_counter() - t0
        # steady state: one captured runner, T reverse steps
        from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep
        from weatherconverter_amd.kernels import philox_normal
        xs = philox_normal((B, 3, 64, 64), dev, 3455, step=T)
        run = _GraphStep(net, xs)
        nxt = torch.empty_like(xs)
        ts = torch.arange(T, device=dev)
        _sync()
        t0 = time.perf_counter()
        for i in reversed(range(T)):
            eps = run(xs, ts[i:i + 1])
            sched.step(xs, eps, i, out=nxt, noise='philox', seed=3455) if i else sched.step(xs, eps, 0, out=nxt)
            xs, nxt = nxt, xs
        _sync()
        steady = (time.perf_counter() - t0) / T
    # CPU: the oracle's UNet step (the reference's unet_base restated op for op) x T
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    x = torch.randn((B, 3, 64, 64), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        unet_forward(sd, mc, x, torch.tensor([25]))
        t0 = time.perf_counter()
        for _ in range(3):
            unet_forward(sd, mc, x, torch.tensor([25]))
        cpu_step = (time.perf_counter() - t0) / 3
    return {
        'config': 1, 'workload': 'sample_ddpm 64 px UNet, B=2, T=50 (full sample, HIP graph, Philox noise)',
        'gpu_s_per_sample_batch': round(gpu_s, 4), 'gpu_ms_per_step': round(gpu_s / T * 1e3, 3),
        'gpu_images_per_s': round(B / gpu_s, 2), 'gpu_ms_per_step_steady': round(steady * 1e3, 3),
        'note': 'gpu_s_per_sample_batch includes the HIP-graph capture of sample_tensor(graph=True)',
        'cpu_ms_per_step': round(cpu_step * 1e3, 2), 'cpu_s_per_sample_batch': round(cpu_step * T, 3),
        'cpu_threads': threads, 'cpu_kind': 'oracle UNet step (reference unet_base restated), x T',
        'x0_finite': bool(torch.isfinite(x0).all()),
    }


def run_config3():
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'bench_train.py'), '--steps', '20'],
                       capture_output=True, text=True, timeout=600)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    if r.returncode != 0 or not line:
        raise RuntimeError(f'bench_train failed: {r.stderr[-2000:]}')
    d = json.loads(line[-1])
    d['config'] = {'id': 3, **d['config']}
    return d


def run_config4(dev, steps):
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.seg_model.network import deeplabv3plus_resnet101
    from weatherconverter_amd.sgg.sgg import apply_gsg
    from weatherconverter_amd.srgan_model.models import Generator
    from weatherconverter_amd.srgan_model.models import inference as srgan_inference
    from weatherconverter_amd.synthetic import init_synthetic_
    S = 256
    mc = model_config(S)
    unet = Unet(mc)
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
    xt = (torch.rand((1, 3, S, S), generator=g) * 2 - 1).to(dev)
    gt = torch.randint(0, 19, (1, 4 * S, 4 * S), generator=g)
    gt[torch.rand(gt.shape, generator=g) < 0.05] = 255
    gt = gt.to(dev)
    ts = torch.arange(1000, device=dev)

    from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep
    from weatherconverter_amd.translation import _Replay
    with torch.no_grad():  # the product loop's runners (translation.sample_with_sgg, graph=True)
        unet_run = _GraphStep(unet, xt)
        sr_run = _Replay(lambda v: srgan_inference(sr, v), xt)

    def step(i, guided):
        with torch.no_grad():
            eps = unet_run(xt, ts[i:i + 1])
            mu, sigma, _ = sched.sample_prev_timestep(xt, eps, i)
            sr_xt = sr_run(xt)
        if guided:
            return apply_gsg(seg, mu, sigma, sr_xt, gt, 60.0)
        return mu + sigma

    times = {}
    for kind, guided in (('unguided', False), ('gsg', True)):
        for _ in range(2):
            step(499, guided)
        _sync()
        t0 = time.perf_counter()
        for j in range(steps):
            out = step(499 - j, guided)
        _sync()
        times[kind] = (time.perf_counter() - t0) / steps
    # the component times of one guided step (graph replays; eager UNet beside them)
    with torch.no_grad():
        _sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            unet_run(xt, ts[100:101])
        _sync()
        t_unet = (time.perf_counter() - t0) / steps
        t0 = time.perf_counter()
        for _ in range(steps):
            unet(xt, ts[100:101])
        _sync()
        t_unet_eager = (time.perf_counter() - t0) / steps
        t0 = time.perf_counter()
        for _ in range(steps):
            sr_run(xt)
        _sync()
        t_sr = (time.perf_counter() - t0) / steps
    N = 500
    loop_s = (N // 2) * times['gsg'] + (N - N // 2) * times['unguided']
    return {
        'config': 4, 'workload': 'guided translation step, 256 px UNet + SRGAN x4 (1024^2) + DeepLabV3+ R101 '
                                 'input gradient at 1024^2 + sgg update, B=1; N=500 (GSG on odd steps)',
        'ms_per_unguided_step': round(times['unguided'] * 1e3, 2), 'ms_per_gsg_step': round(times['gsg'] * 1e3, 2),
        'ms_unet_forward_b1': round(t_unet * 1e3, 2), 'ms_unet_forward_b1_eager': round(t_unet_eager * 1e3, 2),
        'ms_srgan_256_to_1024': round(t_sr * 1e3, 2),
        'ms_deeplab_grad_and_update': round((times['gsg'] - times['unguided']) * 1e3, 2),
        'extrapolated_s_per_translation_N500': round(loop_s, 2),
        'out_finite': bool(torch.isfinite(out).all()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='1,3,4')
    ap.add_argument('--guided-steps', type=int, default=4)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    want = set(int(c) for c in a.configs.split(','))
    res = []
    if 1 in want:
        res.append(run_config1(dev))
        print(json.dumps(res[-1]), flush=True)
    if 3 in want:
        res.append(run_config3())
        print(json.dumps(res[-1]), flush=True)
    if 4 in want:
        res.append(run_config4(dev, a.guided_steps))
        print(json.dumps(res[-1]), flush=True)


if __name__ == '__main__':
    main()
