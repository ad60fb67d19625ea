"""Builds weatherconverter_amd/diffusion_model/scheduler/vrsqrt14.npz from this CPU's VRSQRT14
(tools/vml/dump_vrsqrt14.c, AVX-512F), then checks the restatement vml_sqrt.sqrt_f32 against this host's
torch.sqrt bit for bit (every float32 in [0.25, 1) and a sample of [2^-30, 2^8)).  Run on the reference
host, the one whose torch.sqrt made tests/golden/sched.npz:  python tools/vml/make_table.py"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, 'weatherconverter_amd', 'diffusion_model', 'scheduler', 'vrsqrt14.npz')


def main():
    with tempfile.TemporaryDirectory() as d:
        exe, raw = os.path.join(d, 'dump'), os.path.join(d, 'tab.bin')
        subprocess.run(['gcc', '-O2', '-mavx512f', os.path.join(ROOT, 'tools', 'vml', 'dump_vrsqrt14.c'), '-o', exe],
                       check=True)
        subprocess.run([exe, raw], check=True)
        tab = np.fromfile(raw, dtype='<u2')
    assert tab.size == 65536
    # stored as first differences per parity half (they lie in [-3, 0]: the table is monotone)
    halves = tab.reshape(2, 32768).astype(np.int32)
    np.savez_compressed(OUT, first=halves[:, 0].astype(np.uint16), diff=np.diff(halves, axis=1).astype(np.int8))
    print('wrote', OUT, os.path.getsize(OUT), 'bytes')
    sys.path.insert(0, ROOT)
    import torch

    from weatherconverter_amd.diffusion_model.scheduler import vml_sqrt
    vml_sqrt._table.cache_clear()
    u = np.arange(0x3e800000, 0x3f800000, dtype=np.uint32)
    x = u.view(np.float32)
    bad = int((vml_sqrt.sqrt_f32(x) != torch.sqrt(torch.from_numpy(x)).numpy()).sum())
    rng = np.random.default_rng(0)
    xs = np.exp2(rng.uniform(-30, 8, 4_000_000)).astype(np.float32)
    bad2 = int((vml_sqrt.sqrt_f32(xs) != torch.sqrt(torch.from_numpy(xs)).numpy()).sum())
    print(f'restatement vs this host torch.sqrt: {bad} of {x.size} in [0.25, 1), {bad2} of {xs.size} sampled')
    assert bad == 0 and bad2 == 0


if __name__ == '__main__':
    main()
