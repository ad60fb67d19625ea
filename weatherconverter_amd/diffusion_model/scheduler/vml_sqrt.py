"""torch.sqrt of a float32 CPU tensor, as the reference host computes it -- restated host-independently.

The reference evaluates its scheduler's square roots with torch on the CPU
(``diffusion_model/scheduler/linear_noise_scheduler.py:19,21``, the per-step ``torch.sqrt(alpha)`` at
``:69,100`` and ``variance ** 0.5`` at ``:75,109``).  ATen sends float32 ``sqrt`` (and ``pow(x, 0.5)``)
through MKL VML, whose AVX-512 path is not correctly rounded.  Pinned on the reference host (every
float32 in [0.25, 1) and 4 M samples over [2^-30, 2^8), ``tools/vml/make_table.py``) it is

    r = VRSQRT14(x);  y = x * r;  e = fma(-y, y, x);  sqrt(x) = fma(e, r / 2, y)      (float32 ops)

which is 1 ulp below the correctly rounded root for 0.59 % of inputs (those whose exact root lies within
~0.06 ulp below a rounding midpoint).  Which ones depends on VRSQRT14's approximation bits, which differ
between CPU implementations and code paths, so the reference's own tables depend on the host.  This
module evaluates the formula with exact IEEE arithmetic in numpy and VRSQRT14 from the reference host's
table (``vrsqrt14.npz``: the approximation is a function of the exponent parity and the top 15 mantissa
bits, exact at powers of four -- checked over every normal float by ``tools/vml/dump_vrsqrt14.c``), so
every host gets the reference host's bits: the scheduler tables equal ``tests/golden/sched.npz`` exactly.
"""
import functools
import os

import numpy as np

_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'vrsqrt14.npz')


@functools.lru_cache(maxsize=None)
def _table() -> np.ndarray:
    with np.load(_TABLE, allow_pickle=False) as z:
        first, diff = z['first'].astype(np.int64), z['diff'].astype(np.int64)
    halves = np.concatenate([first[:, None], diff], axis=1).cumsum(axis=1)
    return halves.reshape(-1).astype(np.uint32)  # [parity 2][top15 32768]: significand bits 22..7


def vrsqrt14(x: np.ndarray) -> np.ndarray:
    """VRSQRT14 of positive normal float32 x, from the reference host's table."""
    u = np.asarray(x, np.float32).view(np.uint32)
    e = (u >> 23) & 0xff
    # parity index 1 for even biased exponents ([0.5, 1) is 126), 0 for odd ([0.25, 0.5) is 125)
    par = (e + 1) & 1
    top = (u >> 8) & 0x7fff
    sig = _table()[par * 32768 + top]
    # x = x' 4^k with x' in [0.25, 1) (biased exponent 125 + par): 1/sqrt(x') in (1, 2], r = r' 2^-k
    k = (e.astype(np.int64) - (125 + par.astype(np.int64))) // 2
    rexp = 127 - k
    r = ((rexp.astype(np.uint32) << 23) | (sig << 7)).view(np.float32)
    exact4 = (par == 0) & ((u & 0x7fffff) == 0)  # powers of four: the exact root (2 x 2^-k)
    r = np.where(exact4, ((rexp + 1).astype(np.uint32) << 23).view(np.float32), r)
    return r


def _fma_f32(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """float32 fma(a, b, c) with one rounding: a*b is exact in float64, the sum's float64 rounding error
    is recovered exactly (TwoSum) and decides the float32 rounding where the float64 sum sits on a
    float32 midpoint."""
    p = a.astype(np.float64) * b.astype(np.float64)
    c64 = c.astype(np.float64)
    s = p + c64
    bb = s - p
    err = (p - (s - bb)) + (c64 - bb)
    f = s.astype(np.float32)
    d = s - f.astype(np.float64)
    toward = np.where(d > 0, np.float32(np.inf), np.float32(-np.inf)).astype(np.float32)
    nb = np.nextafter(f, toward)
    half = np.abs(nb.astype(np.float64) - f.astype(np.float64)) / 2
    tie = (d != 0) & (np.abs(d) == half)
    away = tie & (np.sign(err) == np.sign(d)) & (err != 0)
    return np.where(away, nb, f)


def sqrt_f32(x) -> np.ndarray:
    """The reference host's float32 torch.sqrt(x), elementwise (0 -> 0, +inf -> +inf, negative / NaN ->
    NaN).  Subnormal inputs are refused (the scheduler never produces them, and the table was not
    pinned there)."""
    x = np.asarray(x, np.float32)
    scalar = x.ndim == 0
    x = np.atleast_1d(x)
    u = x.view(np.uint32)
    e = (u >> 23) & 0xff
    normal = (e > 0) & (e < 255) & ((u >> 31) == 0)
    sub = (e == 0) & ((u & 0x7fffff) != 0)
    if np.any(sub):
        raise ValueError('vml_sqrt.sqrt_f32: subnormal input')
    xs = np.where(normal, x, np.float32(1.0))
    r = vrsqrt14(xs)
    y = (xs * r).astype(np.float32)
    ee = (xs.astype(np.float64) - y.astype(np.float64) * y.astype(np.float64)).astype(np.float32)  # exact, one rounding
    out = _fma_f32(ee, (np.float32(0.5) * r).astype(np.float32), y)
    with np.errstate(invalid='ignore'):
        ieee = np.sqrt(x)
    out = np.where(normal, out, ieee)  # 0, +-0, inf, nan, negative: IEEE sqrt's values
    return out[0] if scalar else out
