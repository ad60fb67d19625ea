"""CPU: the scheduler tables and step scalars are the reference host's bits on every host (reference
diffusion_model/scheduler/linear_noise_scheduler.py:16-21, :63-116)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from weatherconverter_amd.diffusion_model.scheduler import vml_sqrt
from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import (LinearNoiseScheduler, table_linspace,
                                                                                    tables)

TABLES = ('betas', 'alphas', 'alpha_cum_prod', 'sqrt_alpha_cum_prod', 'one_minus_cum_prod',
          'sqrt_one_minus_alpha_cum_prod')


@pytest.mark.parametrize('T', [50, 1000])
def test_tables_bit_exact_vs_reference_host(T):
    """All six tables equal the reference's own (imported on the golden host, tests/golden/make_golden.py)
    bit for bit, the two square-root tables included: MKL VML's sqrt on the reference host is 1 ulp below
    the correctly rounded root at t = 143, 181, 218, 258, 327, 334 (sqrt_alpha_cum_prod) and 14, 308,
    310, 611, 867 (sqrt_one_minus_alpha_cum_prod) at T = 1000, and the restatement has those bits."""
    gd = np.load(os.path.join(GOLDEN, 'sched.npz'))
    s = LinearNoiseScheduler(T, 0.0001, 0.02, device=torch.device('cpu'))
    for n in TABLES:
        assert np.array_equal(getattr(s, n).numpy(), gd[f'T{T}_{n}']), n
    if T == 1000:  # the entries where the reference's root is not the correctly rounded one
        for n, src, ts in (('sqrt_alpha_cum_prod', 'alpha_cum_prod', [143, 181, 218, 258, 327, 334]),
                           ('sqrt_one_minus_alpha_cum_prod', 'one_minus_cum_prod', [14, 308, 310, 611, 867])):
            cr = np.sqrt(gd[f'T{T}_{src}'])
            assert np.nonzero(cr != gd[f'T{T}_{n}'])[0].tolist() == ts, n


def test_step_scalars_vs_reference_expressions():
    """step_scalars' (beta, sqrt(1 - acp), sqrt(alpha), sigma) for every t in both variance modes equal the
    reference's 0-d float32 torch expressions (:96-110, :63-75) evaluated on this host, wherever this
    host's torch.sqrt is the reference host's (the MKL VML AVX-512 path; else the bits are pinned by the
    golden step vectors in test_oracle_golden / test_gpu_kernels)."""
    x = np.linspace(0.01, 1.0, 20001, dtype=np.float32)
    if not np.array_equal(torch.sqrt(torch.from_numpy(x)).numpy(), vml_sqrt.sqrt_f32(x)):
        pytest.skip("this host's torch.sqrt is not the reference host's")
    s = LinearNoiseScheduler(1000, 0.0001, 0.02, device=torch.device('cpu'))
    be, al, acp = s._cpu['betas'], s._cpu['alphas'], s._cpu['alpha_cum_prod']
    for t in range(1000):
        ref_sqa = torch.sqrt(al[t]).item()
        ref_post = 0.0 if t == 0 else (((1 - acp[t - 1]) / (1.0 - acp[t])) * be[t]) ** 0.5
        for variance, ref_sig in (('posterior', ref_post), ('beta', 0.0 if t == 0 else be[t] ** 0.5)):
            beta, s1m, sqa, sigma = s.step_scalars(t, variance)
            assert (beta, s1m, sqa) == (be[t].item(), s._cpu['sqrt_one_minus_alpha_cum_prod'][t].item(), ref_sqa), t
            assert sigma == float(ref_sig), (t, variance)


def test_vml_sqrt_properties():
    """The restated MKL sqrt: never above the correctly rounded root and at most 1 ulp below it; exact on
    squares and powers of four; IEEE values at 0, inf, NaN and negative inputs; subnormals refused."""
    rng = np.random.default_rng(5)
    x = np.exp2(rng.uniform(-40, 40, 200_000)).astype(np.float32)
    got, cr = vml_sqrt.sqrt_f32(x), np.sqrt(x)
    d = cr.view(np.int32).astype(np.int64) - got.view(np.int32).astype(np.int64)
    assert d.min() == 0 and d.max() == 1 and 0.002 < (d != 0).mean() < 0.02
    sq = np.arange(1, 4097, dtype=np.float32)
    assert np.array_equal(vml_sqrt.sqrt_f32(sq * sq), sq)
    p4 = np.float32(4.0)**np.arange(-30, 30, dtype=np.float32)
    assert np.array_equal(vml_sqrt.sqrt_f32(p4), np.sqrt(p4))
    sp = np.array([0.0, -0.0, np.inf, np.nan, -1.0], np.float32)
    out = vml_sqrt.sqrt_f32(sp)
    assert out[0] == 0 and out[2] == np.inf and np.isnan(out[3]) and np.isnan(out[4])
    assert vml_sqrt.sqrt_f32(np.float32(0.25)) == np.float32(0.5)
    with pytest.raises(ValueError):
        vml_sqrt.sqrt_f32(np.array([1e-40], np.float32))


def test_tables_independent_of_torch_linspace_path():
    """The restatement agrees with torch.linspace wherever torch's result is the per-element fused form,
    and never depends on torch: the same call gives the same bits in a fresh computation."""
    for (T, a, b) in ((1000, 0.0001, 0.02), (50, 0.0001, 0.02), (250, 1e-4, 0.03), (7, 0.5, -0.25)):
        x = table_linspace(a, b, T)
        assert x.dtype == np.float32 and x.shape == (T, )
        assert x[0] == np.float32(a) and x[-1] == np.float32(b)
        assert np.array_equal(x, table_linspace(a, b, T))
        assert np.all(np.abs(x - torch.linspace(a, b, T).numpy()) <= np.spacing(np.abs(x)))
    t = tables(1000, 0.0001, 0.02)
    assert all(v.dtype == np.float32 for v in t.values())
    assert np.all(np.diff(t['alpha_cum_prod']) < 0)
