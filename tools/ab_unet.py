"""Same-box A/B of UNet-forward variants (HIP-graph replay, 256px B=16 by default).

Box-to-box clock differences (power cap) are larger than most single-kernel changes, so a variant is
only judged against the baseline captured in the same process: each variant is an engine mutation
applied after packing, captured into its own graph, and the graphs are replayed alternately.

  python tools/ab_unet.py [--variants base,no_f3_resample] [--reps 10] [--rounds 4]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def no_f3_resample(eng):
    """Down-sampling / transposed convs back on bf16x6 (no producer-bound f16x3)."""
    eng.down_convs = [None if d is None else (d[0], d[1], d[2], None) for d in eng.down_convs]
    eng.up_convs = [None if u is None else ([(t, w, w6, None) for t, w, w6, _ in u[0]], u[1]) for u in eng.up_convs]


def no_gn_partials(eng):
    """One GroupNorm stats pass per GN instead of the producers' epilogue tile partials."""
    eng.gn_partials = False


VARIANTS = {'base': lambda eng: None, 'no_f3_resample': no_f3_resample, 'no_gn_partials': no_gn_partials}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--variants', default='base,no_f3_resample')
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=4)
    args = ap.parse_args()
    from weatherconverter_amd import kernels
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep
    from weatherconverter_amd.synthetic import init_synthetic_
    dev = torch.device('cuda', 0)
    mc = model_config(args.size)
    model = Unet(mc)
    init_synthetic_(model, seed=0)
    model = model.to(dev).eval()
    names = args.variants.split(',')
    x = kernels.philox_normal((args.batch, mc.im_channels, mc.im_size, mc.im_size), dev, 0, sample0=0, step=1000)
    t = torch.full((1, ), 500, dtype=torch.long, device=dev)
    runners, outs, engines = {}, {}, []
    with torch.no_grad():
        for n in names:
            model._engine = None
            engines.append(model.engine())  # each graph keeps reading its own engine's packed weights
            VARIANTS[n](engines[-1])
            runners[n] = _GraphStep(model, x)
            outs[n] = runners[n](x, t).clone()
        times = {n: [] for n in names}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.rounds):
            for n in names:
                runners[n](x, t)
                ev0.record()
                for _ in range(args.reps):
                    runners[n](x, t)
                ev1.record()
                torch.cuda.synchronize()
                times[n].append(ev0.elapsed_time(ev1) / args.reps)
    base = names[0]
    for n in names:
        d = (outs[n] - outs[base]).double()
        rel = float(d.norm() / outs[base].double().norm())
        print(f'{n:20s} median {statistics.median(times[n]):8.3f} ms  min {min(times[n]):8.3f} ms  '
              f'rel-diff vs {base} {rel:.2e}  rounds {["%.3f" % v for v in times[n]]}', flush=True)


if __name__ == '__main__':
    main()
