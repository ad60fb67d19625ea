"""Generate golden vectors by importing the REFERENCE (xXCoffeeColaXc/WeatherConverter) on CPU.

Run in the build container only (the reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--reference /root/reference]

Outputs (committed; inputs are regenerated from seeds, weights from the keyed recipe in
weatherconverter_amd/synthetic.py, so only outputs + digests are stored):
  manifest.json         state_dict key->shape for the 64/128/256 default configs and the tiny config
  sched.npz             scheduler tables (T=50, T=1000), reverse-step / add_noise vectors
  temb.npz              get_time_embedding for several t
  unet_tiny.npz         tiny-config Unet forward, B=2, shared t and per-sample t
  unet_64.npz           64-px default-config Unet forward, B=2 (config 1 model)
  unet_256.npz          256-px default-config Unet forward, B=1 (BASELINE architecture)
  traj_64_T50.npz       config 1: 64 px, B=2, T=50 reverse trajectory (sample_ddpm.py:35-44 loop)
  traj_64_T1000.npz     64 px default config, B=1, the full T=1000 schedule, same loop and RNG stream
                        (--only-traj1000; ~5 min on 8 CPU threads)
The reference modules imported: diffusion_model.models.unet_base, diffusion_model.scheduler.
linear_noise_scheduler, diffusion_model.config.models.  ``Tensor.cuda`` is shimmed to a no-op
(unet_base.py:461 hard-codes .cuda()); nothing in the reference is modified.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from weatherconverter_amd.synthetic import synthetic_images, synthetic_state_dict, state_dict_digest  # noqa: E402

TINY = dict(name='ddpm', im_channels=3, im_size=32, down_channels=[32, 64, 64, 128], mid_channels=[128, 128, 64],
            down_sample=[True, True, False], time_emb_dim=128, num_down_layers=2, num_mid_layers=1,
            num_up_layers=2, num_heads=4, attn_resolutions=[16, 8])


def default_model(ref_models, im_size):
    import yaml
    with open(os.path.join(ROOT, 'weatherconverter_amd/diffusion_model/config/config.yaml')) as fh:
        m = yaml.safe_load(fh)['model']
    m['im_size'] = im_size
    return ref_models.ModelConfig(**m)


# Reverse-step t: the ends and the middle, plus every t whose step scalars the reference host's MKL sqrt
# rounds 1 ulp below the correctly rounded root: sqrt(1 - acp) at 14, 308, 611, 867 (and 310), sqrt(alpha)
# at 710, the posterior sigma at 85, 490 (weatherconverter_amd/diffusion_model/scheduler/vml_sqrt.py).
STEP_T = (0, 1, 37, 500, 999, 14, 308, 310, 611, 867, 710, 85, 490)
# sample_prev_timestep2 (beta variance): t = 3, and the beta sigmas MKL rounds down (190, 222)
STEP2_T = (3, 190, 222)


def sched_steps(s, sched):
    """Reverse-step vectors of the reference scheduler s (T = 1000) into sched."""
    g = torch.Generator().manual_seed(11)
    xt = torch.randn((2, 3, 16, 16), generator=g) * 3
    eps = torch.randn((2, 3, 16, 16), generator=g)
    sched['step_xt'] = xt.numpy()
    sched['step_eps'] = eps.numpy()
    for t in STEP_T:
        torch.manual_seed(1000 + t)
        mean, sz, _ = s.sample_prev_timestep(xt, eps, torch.as_tensor(t))
        sched[f'step{t}_mean'] = mean.numpy()
        if sz is not None:
            sched[f'step{t}_sigz'] = sz.numpy()
            torch.manual_seed(1000 + t)
            sched[f'step{t}_z'] = torch.randn(xt.shape).numpy()
    for t in STEP2_T:
        tb = torch.tensor([t, t])
        torch.manual_seed(77 + (t if t != 3 else 0))
        mean2, sz2, _ = s.sample_prev_timestep2(xt, eps, tb)
        key = 'step2' if t == 3 else f'step2_{t}'
        sched[f'{key}_t'] = tb.numpy()
        sched[f'{key}_mean'] = mean2.numpy()
        sched[f'{key}_sigz'] = sz2.numpy()
        torch.manual_seed(77 + (t if t != 3 else 0))
        sched[f'{key}_z'] = torch.randn(xt.shape).numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', default='/root/reference')
    ap.add_argument('--skip-traj', action='store_true')
    ap.add_argument('--only-guided', action='store_true')
    ap.add_argument('--only-old', action='store_true')
    ap.add_argument('--only-traj1000', action='store_true')
    ap.add_argument('--only-sched-steps', action='store_true',
                    help='add the reverse-step vectors at STEP_T / STEP2_T to the existing sched.npz')
    args = ap.parse_args()
    sys.path.insert(0, args.reference)
    torch.Tensor.cuda = lambda self, *a, **k: self  # harness shim for unet_base.py:461
    torch.set_num_threads(8)
    if args.only_guided:
        return guided(args)
    if args.only_old:
        return old_unet(args)
    if args.only_traj1000:
        return traj1000(args)
    if args.only_sched_steps:
        from diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
        path = os.path.join(HERE, 'sched.npz')
        with np.load(path, allow_pickle=False) as z:
            sched = dict(z)
        sched_steps(LinearNoiseScheduler(1000, 0.0001, 0.02), sched)
        np.savez(path, **sched)
        return
    from diffusion_model.config import models as ref_models
    from diffusion_model.models.unet_base import Unet, get_time_embedding
    from diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler

    out = {}
    # ------------------------------------------------------------- manifest
    manifest = {}
    cfgs = {'tiny': ref_models.ModelConfig(**TINY)}
    for s in (64, 128, 256):
        cfgs[f'default_{s}'] = default_model(ref_models, s)
    for name, mc in cfgs.items():
        net = Unet(mc)
        manifest[name] = {'config': mc.model_dump(), 'keys': [[k, list(v.shape)] for k, v in net.state_dict().items()]}
    with open(os.path.join(HERE, 'manifest.json'), 'w') as fh:
        json.dump(manifest, fh)
    print('manifest:', {k: len(v['keys']) for k, v in manifest.items()})

    # ------------------------------------------------------------- scheduler
    sched = {}
    for T in (50, 1000):
        s = LinearNoiseScheduler(T, 0.0001, 0.02)
        for n in ('betas', 'alphas', 'alpha_cum_prod', 'sqrt_alpha_cum_prod', 'one_minus_cum_prod',
                  'sqrt_one_minus_alpha_cum_prod'):
            sched[f'T{T}_{n}'] = getattr(s, n).numpy()
    s = LinearNoiseScheduler(1000, 0.0001, 0.02)
    sched_steps(s, sched)
    xt, eps = torch.from_numpy(sched['step_xt']), torch.from_numpy(sched['step_eps'])
    tn = torch.tensor([5, 880])
    sched['addnoise_t'] = tn.numpy()
    sched['addnoise_out'] = s.add_noise(xt, eps, tn).numpy()
    sched['addnoise2_out'] = s.add_noise2(xt, eps, tn).numpy()
    np.savez(os.path.join(HERE, 'sched.npz'), **sched)

    # ------------------------------------------------------------- time embedding
    ts = torch.tensor([0, 1, 17, 500, 999])
    np.savez(os.path.join(HERE, 'temb.npz'), t=ts.numpy(), emb=get_time_embedding(ts, 128).numpy())

    # ------------------------------------------------------------- UNet forwards
    def run_forward(mc, B, t, xseed, wseed=0):
        net = Unet(mc)
        sd = synthetic_state_dict(net.state_dict(), seed=wseed)
        net.load_state_dict(sd)
        net.eval()
        x = synthetic_images((B, mc.im_channels, mc.im_size, mc.im_size), seed=xseed)
        with torch.no_grad():
            y = net(x, torch.as_tensor(t))
        return net, y, state_dict_digest(sd)

    net, y1, dg = run_forward(cfgs['tiny'], 2, [7], 101)
    _, y2, _ = run_forward(cfgs['tiny'], 2, [3, 900], 102)
    np.savez(os.path.join(HERE, 'unet_tiny.npz'), y_shared_t=y1.numpy(), y_batch_t=y2.numpy(), digest=dg)
    print('tiny done', float(y1.abs().max()))
    _, y64, dg64 = run_forward(cfgs['default_64'], 2, [37], 201)
    np.savez(os.path.join(HERE, 'unet_64.npz'), y=y64.numpy(), digest=dg64)
    print('64 done', float(y64.abs().max()))
    _, y256, dg256 = run_forward(cfgs['default_256'], 1, [611], 301)
    np.savez(os.path.join(HERE, 'unet_256.npz'), y=y256.numpy(), digest=dg256)
    print('256 done', float(y256.abs().max()))

    # ------------------------------------------------------------- config-1 trajectory
    if not args.skip_traj:
        mc = cfgs['default_64']
        net = Unet(mc)
        net.load_state_dict(synthetic_state_dict(net.state_dict(), seed=0))
        net.eval()
        s50 = LinearNoiseScheduler(50, 0.0001, 0.02)
        torch.manual_seed(3455)
        xt = torch.randn((2, 3, 64, 64))  # sample_ddpm.py:35-36
        eps_first = None
        with torch.no_grad():
            for i in reversed(range(50)):  # sample_ddpm.py:37-44
                noise_pred = net(xt, torch.as_tensor(i).unsqueeze(0))
                if eps_first is None:
                    eps_first = noise_pred.clone()
                mean, sigma, _ = s50.sample_prev_timestep(xt, noise_pred, torch.as_tensor(i))
                xt = mean + sigma if i != 0 else mean
        np.savez(os.path.join(HERE, 'traj_64_T50.npz'), x0=xt.numpy(), eps_first=eps_first.numpy(), seed=3455)
        print('traj done', float(xt.abs().max()))


def traj1000(args):
    """traj_64_T1000.npz: the sample_ddpm.py:35-44 loop over the full T=1000 schedule (64-px default
    config, B=1, torch.manual_seed(3455) CPU stream), x at a few checkpoints and the final x0."""
    from diffusion_model.config import models as ref_models
    from diffusion_model.models.unet_base import Unet
    from diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    mc = default_model(ref_models, 64)
    net = Unet(mc)
    sd = synthetic_state_dict(net.state_dict(), seed=0)
    net.load_state_dict(sd)
    net.eval()
    s = LinearNoiseScheduler(1000, 0.0001, 0.02)
    torch.manual_seed(3455)
    xt = torch.randn((1, 3, 64, 64))  # sample_ddpm.py:35-36
    out = {'seed': 3455, 'digest': state_dict_digest(sd)}
    marks = {999, 900, 500, 100}
    with torch.no_grad():
        for i in reversed(range(1000)):  # sample_ddpm.py:37-44
            noise_pred = net(xt, torch.as_tensor(i).unsqueeze(0))
            mean, sigma, _ = s.sample_prev_timestep(xt, noise_pred, torch.as_tensor(i))
            xt = mean + sigma if i != 0 else mean
            if i in marks:
                out[f'x_after_t{i}'] = xt.numpy().copy()
    out['x0'] = xt.numpy()
    np.savez(os.path.join(HERE, 'traj_64_T1000.npz'), **out)
    print('traj1000 done', float(xt.abs().max()))


def old_unet(args):
    """old_unet.npz: old_modules.UNet (128 px) forward and a sample_integrated.py:52-64 trajectory
    (T=10 schedule, B=1, reference RNG stream), plus the key manifest."""
    from diffusion_model.models.old_modules import UNet
    from diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    net = UNet()
    sd = synthetic_state_dict(net.state_dict(), seed=0)
    net.load_state_dict(sd)
    net.eval()
    out = {'digest': state_dict_digest(sd)}
    x = synthetic_images((1, 3, 128, 128), seed=501)
    lvl = torch.tensor([[[[0.2860]]]])
    with torch.no_grad():
        out['y'] = net(x, lvl).numpy()
    s10 = LinearNoiseScheduler(10, 0.0001, 0.02)
    torch.manual_seed(3455)
    xt = torch.randn((1, 3, 128, 128))  # sample_integrated.py:52-53
    with torch.no_grad():
        for i in reversed(range(10)):  # :55-64
            t = torch.full((xt.size(0), ), i, dtype=torch.long)
            noise_pred = net(xt, s10.one_minus_cum_prod[t].view(-1, 1, 1, 1))
            mean, sigma, _ = s10.sample_prev_timestep2(xt, noise_pred, t)
            xt = mean + sigma if i != 0 else mean
    out['traj_x0'] = xt.numpy()
    np.savez(os.path.join(HERE, 'old_unet.npz'), **out)
    with open(os.path.join(HERE, 'old_manifest.json'), 'w') as fh:
        json.dump([[k, list(v.shape)] for k, v in net.state_dict().items()], fh)
    print('old unet done', float(np.abs(out['y']).max()), float(np.abs(out['traj_x0']).max()))


def guided(args):
    """guided.npz + guided_manifest.json: DeepLabV3+ R101 OS16 (seg_model.network) logits and input
    gradient, the apply_gsg update (sgg.py:16-22 + inference.py:39-53 restated: those modules import
    torchvision, absent here), and the Swift-SRGAN generator (srgan_model.models)."""
    import torch.nn.functional as F
    from seg_model.network.modeling import deeplabv3plus_resnet101
    from srgan_model.models import Generator
    torch.set_num_threads(8)
    out, manifest = {}, {}
    seg = deeplabv3plus_resnet101(num_classes=19, output_stride=16, pretrained_backbone=False)
    sd = synthetic_state_dict(seg.state_dict(), seed=0)
    seg.load_state_dict(sd)
    seg.eval()
    manifest['deeplabv3plus_resnet101'] = [[k, list(v.shape)] for k, v in seg.state_dict().items()]
    out['seg_digest'] = state_dict_digest(sd)
    g = torch.Generator().manual_seed(41)
    sr = torch.randn((1, 3, 32, 32), generator=g)
    gt = torch.randint(0, 19, (1, 32, 32), generator=g)
    gt[torch.rand((1, 32, 32), generator=g) < 0.05] = 255
    x = sr.clone().requires_grad_(True)  # inference.py:118-152 restated
    logits = seg(x)
    loss = torch.nn.CrossEntropyLoss(ignore_index=255)(logits, gt.squeeze(1))
    loss.backward()
    out['sr'] = sr.numpy()
    out['gt'] = gt.numpy()
    out['logits'] = logits.detach().numpy()
    out['grad'] = x.grad.numpy()
    mu = torch.randn((1, 3, 8, 8), generator=g)
    sigma = torch.randn((1, 3, 8, 8), generator=g) * 0.05
    pooled = F.avg_pool2d(x.grad, kernel_size=4, stride=4)  # sgg.py:18
    gn = pooled.squeeze(0).numpy() * np.array([0.229, 0.224, 0.225])[:, None, None]  # inference.py:39-42
    mag = torch.from_numpy(np.sqrt(np.sum(gn**2, axis=0)))  # :43
    out['mu'], out['sigma'] = mu.numpy(), sigma.numpy()
    out['gsg_xt'] = ((mu + 60.0 * sigma * mag) + sigma).numpy()  # sgg.py:21-22, float64
    gen = Generator(upscale_factor=4)
    gsd = synthetic_state_dict(gen.state_dict(), seed=0)
    gen.load_state_dict(gsd)
    gen.eval()
    manifest['srgan_generator'] = [[k, list(v.shape)] for k, v in gen.state_dict().items()]
    out['srgan_digest'] = state_dict_digest(gsd)
    lr = torch.rand((1, 3, 16, 16), generator=g)
    with torch.no_grad():
        out['srgan_in'], out['srgan_out'] = lr.numpy(), gen(lr).numpy()
    np.savez(os.path.join(HERE, 'guided.npz'), **out)
    with open(os.path.join(HERE, 'guided_manifest.json'), 'w') as fh:
        json.dump(manifest, fh)
    print('guided done', float(out['grad'].std()), float(np.abs(out['gsg_xt']).max()))


if __name__ == '__main__':
    main()
