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
A final line (--breakdown, default on) splits one guided step into its parts, each timed alone over
--reps repetitions with HIP events: the UNet forward (graph replay, B=1), the scheduler step, the SRGAN
x4 forward (graph replay), the DeepLab forward + input gradient and the wc_sgg_update kernel; per-step
= UNet + scheduler + SRGAN + (DeepLab + update) / 2 (GSG on odd steps).  It carries a `roofline` object
(the SRGAN's kernels timed inside a replayed graph by wc_stamp nodes, against the fp32-MFMA peak for
the pointwise GEMMs and HBM for the depthwise convs; the update kernel against HBM; the B=1 UNet's
dominant kernel as bench.py reports it) and a `cpu_baseline` (the same step on the host cores: the
oracle UNet, the CPU SRGAN, the oracle GSG with the CPU DeepLab -- one odd and one even step,
extrapolated x N).
    python tools/bench_guided.py [--n 500] [--miopen-benchmark 1] [--lcg-steps 2] [--breakdown 1]
"""
import argparse
import copy
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
    ap.add_argument('--breakdown', type=int, default=1)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--cpu-baseline', type=int, default=1)
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
    unet_sd_cpu = {k: v.detach().clone() for k, v in unet.state_dict().items()}
    unet = unet.to(dev).eval()
    sr = Generator()
    init_synthetic_(sr, seed=1)
    sr_cpu = copy.deepcopy(sr).eval()
    sr = sr.to(dev).eval()
    seg = deeplabv3plus_resnet101(num_classes=19, output_stride=16, pretrained_backbone=False)
    init_synthetic_(seg, seed=2)
    seg_cpu = copy.deepcopy(seg).eval()
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

    if a.breakdown:
        line = breakdown(a, unet, sched, sr, seg, gt, noise.to(dev))
        if a.cpu_baseline:
            line['cpu_baseline'] = cpu_baseline(a, unet_sd_cpu, sr_cpu, seg_cpu, gt.cpu(), noise)
            line['cpu_baseline']['vs_gpu_per_step'] = round(line['cpu_baseline']['ms_per_step'] / line['ms_per_step'], 1)
        print(json.dumps(line), flush=True)


def _events(fn, reps):
    """Mean seconds of fn() over reps back-to-back calls between one HIP event pair (after one warm call)."""
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def stamped_kernels(fn, x, reps=3):
    """Per-instantiation in-graph table of fn(x) (bench.ingraph_timing for any callable): every named
    launch between two wc_stamp nodes inside one captured graph, replayed `reps` times.  Returns
    {name: [launches, flops, sec, bytes]} per call."""
    import bench
    from weatherconverter_amd import kernels
    hz = kernels.wall_clock_hz()
    x_in = x.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn(x_in)
    torch.cuda.current_stream().wait_stream(side)
    slots = torch.zeros(16384, dtype=torch.int64, device=x.device)
    over = bench._stamp_overhead(slots)
    g = torch.cuda.CUDAGraph()
    st = kernels.stamp_timing(slots)
    try:
        with torch.cuda.graph(g):
            fn(x_in)
    finally:
        kernels.stamp_timing(None)
    per = {}
    for name, flops, nbytes, _ in st['launches']:
        d = per.setdefault(name, [0, 0.0, 0.0, 0.0])
        d[0] += 1
        d[1] += flops
        d[3] += nbytes
    for _ in range(reps):
        g.replay()
        torch.cuda.synchronize()
        v = slots[:2 * len(st['launches'])].cpu().tolist()
        for i, (name, *_) in enumerate(st['launches']):
            per[name][2] += ((v[2 * i + 1] - v[2 * i]) / hz - over) / reps
    del g
    return per


def _kernel_rows(per):
    import bench
    rows = {}
    for k, (n, fl, sec, nb) in sorted(per.items(), key=lambda kv: -kv[1][2]):
        r = {'launches': n, 'ms': round(sec * 1e3, 4)}
        if k.startswith('conv_igemm_kernel'):
            tf = fl / sec / 1e12
            r.update({'bound': 'mfma', 'achieved': round(tf, 2), 'peak': bench.FP32_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                      'frac': round(tf / bench.FP32_PEAK_TFLOPS, 4), 'gflop': round(fl / 1e9, 3)})
        elif nb:
            gbs = nb / sec / 1e9
            r.update({'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': bench.HBM_PEAK_GBS, 'unit': 'GB/s',
                      'frac': round(gbs / bench.HBM_PEAK_GBS, 4), 'gbytes': round(nb / 1e9, 4)})
        rows[k] = r
    return rows


def breakdown(a, unet, sched, sr, seg, gt, noise):
    """One guided step split into its parts (module docstring)."""
    import bench
    from weatherconverter_amd import kernels as K
    from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep
    from weatherconverter_amd.seg_model.inference import input_gradient
    from weatherconverter_amd.sgg.sgg import _update
    from weatherconverter_amd.srgan_model.models import inference as srgan_inference
    from weatherconverter_amd.translation import _Replay
    dev = noise.device
    S = a.size
    xt = noise.clone()
    i = a.n // 2 + 1  # an odd (GSG) step of the loop
    run = _GraphStep(unet, xt)
    t_dev = torch.tensor([i], device=dev)
    unet_s = _events(lambda: run(xt, t_dev), a.reps)
    eps = run(xt, t_dev).clone()
    sched_s = _events(lambda: sched.sample_prev_timestep(xt, eps, i), a.reps)
    mu, sigma, _ = sched.sample_prev_timestep(xt, eps, i)
    sr_run = _Replay(lambda v: srgan_inference(sr, v), xt)
    sr_s = _events(lambda: sr_run(xt), a.reps)
    sr_xt = sr_run(xt).clone()
    seg_s = _events(lambda: input_gradient(seg, sr_xt, gt), max(2, a.reps // 4))
    grad, _ = input_gradient(seg, sr_xt, gt)
    grad = grad.float().contiguous()
    upd_s = _events(lambda: _update(grad, mu, sigma, 60.0, 'per_sample'), a.reps)
    # kernels of the SRGAN forward and the update, timed inside replayed graphs
    sr_rows = _kernel_rows(stamped_kernels(lambda v: srgan_inference(sr, v), xt))
    upd_rows = _kernel_rows(stamped_kernels(lambda g: K.sgg_update(g, mu, sigma, 60.0), grad))
    sr_mfma = {k: v for k, v in sr_rows.items() if v.get('bound') == 'mfma'}
    dom = max(sr_mfma, key=lambda k: sr_mfma[k]['ms']) if sr_mfma else None
    uroof = bench.roofline_leg(unet, xt, t_dev)
    per_step = unet_s + sched_s + sr_s + 0.5 * (seg_s + upd_s)
    return {
        'config': 4, 'metric': 'guided translation ms per reverse step (sample_with_sgg parts)',
        'value': round(per_step * 1e3, 3), 'unit': 'ms/step', 'higher_is_better': False,
        'ms_per_step': round(per_step * 1e3, 3), 'projected_s_for_N': round(per_step * a.n, 2), 'N': a.n,
        'parts_ms': {'unet_forward_graph_B1': round(unet_s * 1e3, 3), 'scheduler_step': round(sched_s * 1e3, 4),
                     'srgan_x4_graph': round(sr_s * 1e3, 3), 'deeplab_fwd_input_grad_1024': round(seg_s * 1e3, 3),
                     'wc_sgg_update': round(upd_s * 1e3, 4)},
        'per_step_model': 'unet + scheduler + srgan + (deeplab + sgg_update) / 2: GSG on the odd steps '
                          '(translation.py:84-87), plain reverse step on the even ones',
        'reps': a.reps,
        'roofline': {
            'srgan_dominant': dict(sr_mfma[dom], kernel=dom) if dom else None,
            'srgan_kernels': sr_rows,
            'sgg_update': upd_rows,
            'unet_B1': {k: uroof[k] for k in ('kernel', 'achieved', 'peak', 'unit', 'frac', 'mean_launch_ms',
                                              'mfma_ms_per_forward')},
            'source': 'wc_stamp GPU wall-clock nodes around each launch inside a replayed HIP graph (bench.py '
                      'ingraph_timing); SRGAN pointwise GEMMs on fp32 MFMA (157.3 TF/s), depthwise convs and the '
                      'update on HBM (8 TB/s, algorithmic bytes: each input and output element once)'},
        'workload': f'{S}-px UNet B=1 + Swift-SRGAN x4 to {4 * S}^2 + DeepLabV3+ R101 OS16 input gradient at '
                    f'{4 * S}^2 + wc_sgg_update, lambda=60',
        'data': 'synthetic keyed weights, N(0,1) latent, gt randint(0,19) + 5% ignore'}


def cpu_baseline(a, unet_sd, sr_cpu, seg_cpu, gt, noise):
    """The guided step on the host cores: oracle UNet (reference unet_base restated op for op), the
    scheduler oracle's reverse step, the SRGAN's CPU forward (the reference module tree), the oracle
    GSG (reference sgg.py:9-24, inference.py:118-152) with the CPU DeepLab; one odd (GSG) and one
    even step, the mean extrapolated x N."""
    sys.path.insert(0, ROOT)
    import bench
    from oracle.scheduler_oracle import OracleScheduler
    from oracle.sgg_oracle import apply_gsg as gsg_oracle
    from oracle.unet_oracle import unet_forward
    from weatherconverter_amd.diffusion_model.config import model_config
    share = bench._cpu_share()
    torch.set_num_threads(share['usable_cpus'])
    mc = model_config(a.size)
    sched = OracleScheduler(1000, 0.0001, 0.02)
    xt = noise.clone()
    times = {}
    with torch.no_grad():
        for odd in (True, False):
            i = a.n // 2 + (1 if odd else 0)
            t0 = time.perf_counter()
            eps = unet_forward(unet_sd, mc, xt, torch.tensor([i]))
            mu, sigma = sched.sample_prev_timestep(xt, eps, i)
            sr_xt = sr_cpu(xt)
            if odd:
                with torch.enable_grad():
                    out = gsg_oracle(seg_cpu, mu, sigma, sr_xt, gt, 60.0)
            else:
                out = mu + sigma
            times['odd' if odd else 'even'] = time.perf_counter() - t0
            del out
    step = 0.5 * (times['odd'] + times['even'])
    return {'ms_per_step': round(step * 1e3, 1), 'value_s_for_N': round(step * a.n, 1), 'unit': 's', 'cores': share['usable_cpus'],
            'kind': 'port', 'host': share,
            'sample': f'one odd (GSG) step {times["odd"]:.2f} s and one even step {times["even"]:.2f} s at N={a.n}, '
                      f'{a.size}-px UNet B=1, on {share["usable_cpus"]} threads; extrapolated x{a.n} -- not a full loop'}


if __name__ == '__main__':
    main()
