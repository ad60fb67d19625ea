"""CPU-baseline provenance: the oracle's PyTorch-CPU UNet step against the imported
REFERENCE ``unet_base.Unet`` on the same weights, input, t and thread count, in this build container.

Prints one JSON line: bitwise equality of the two outputs, their rel-L2, and the per-forward CPU
times (median of --reps after one warmup) and their ratio.  The reference is imported read-only from
/root/reference with the harness's ``Tensor.cuda`` no-op shim for unet_base.py:461 (as
tests/golden/make_golden.py); it never goes to the GPU box.
    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_provenance.py [--size 256 --batch 2 --threads 8 --reps 3]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', default='/root/reference')
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--batch', type=int, default=2)
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--reps', type=int, default=3)
    a = ap.parse_args()
    sys.path.insert(0, a.reference)
    torch.Tensor.cuda = lambda self, *x, **k: self  # harness shim for unet_base.py:461
    torch.set_num_threads(a.threads)
    from diffusion_model.models.unet_base import Unet as RefUnet
    from oracle.unet_oracle import unet_forward
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.synthetic import synthetic_images, synthetic_state_dict
    from diffusion_model.config import models as ref_models
    mc = model_config(a.size)
    ref = RefUnet(ref_models.ModelConfig(**mc.model_dump())).eval()
    sd = synthetic_state_dict(ref.state_dict(), seed=0)
    ref.load_state_dict(sd)
    x = synthetic_images((a.batch, 3, a.size, a.size), seed=301)
    t = torch.tensor([611])
    times = {'reference': [], 'oracle': []}
    outs = {}
    with torch.no_grad():
        for name, fn in (('reference', lambda: ref(x, t)), ('oracle', lambda: unet_forward(sd, mc, x, t))):
            fn()
        for _ in range(a.reps):  # interleaved rounds
            for name, fn in (('reference', lambda: ref(x, t)), ('oracle', lambda: unet_forward(sd, mc, x, t))):
                t0 = time.perf_counter()
                outs[name] = fn()
                times[name].append(time.perf_counter() - t0)
    r, o = outs['reference'], outs['oracle']
    med = {k: statistics.median(v) for k, v in times.items()}
    res = {'case': f'{a.size}px default config.yaml UNet, B={a.batch}, t=611, keyed synthetic weights (seed 0)',
           'threads': a.threads, 'cpu_model': _cpu(), 'bitwise_equal': bool(torch.equal(r, o)),
           'rel_l2': float((o.double() - r.double()).norm() / r.double().norm()),
           'max_abs_diff': float((o - r).abs().max()),
           'reference_ms_per_forward': round(med['reference'] * 1e3, 1), 'oracle_ms_per_forward': round(med['oracle'] * 1e3, 1),
           'oracle_over_reference_time': round(med['oracle'] / med['reference'], 4),
           'reps': a.reps, 'all_ms': {k: [round(v * 1e3, 1) for v in vs] for k, vs in times.items()}}
    print(json.dumps(res))


def _cpu():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == '__main__':
    main()
