"""Micro-benchmark of wc_conv_igemm / wc_attention_fwd on the 256-px UNet shapes (B=16), with a
correctness spot check against torch fp32 on the GPU (torch conv: tf32 disabled)."""
import argparse
import sys
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd import kernels as K  # noqa: E402

TAPS3 = [(ky - 1, kx - 1) for ky in range(3) for kx in range(3)]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


ZEROS = False


def conv_case(B, H, Ci, Co, prologue=True, res=0, check=False, mode='fp32', taps=None):
    taps = TAPS3 if taps is None else taps
    nt = len(taps)
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn((B, H, H, Ci), device='cuda', generator=g)
    if ZEROS:
        x.zero_()
    w = torch.randn((Co, nt * Ci + res), device='cuda', generator=g) / (nt * Ci)**0.5
    b = torch.randn(Co, device='cuda', generator=g)
    sc = torch.rand((B, Ci), device='cuda', generator=g) + 0.5
    sh = torch.randn((B, Ci), device='cuda', generator=g) * 0.1
    out = torch.empty((B, H, H, Co), device='cuda')
    segs = [K.Seg(K.View.full(x), taps, scale=sc if prologue else None, shift=sh if prologue else None,
                  silu=prologue and nt > 1)]
    if res:
        xr = torch.randn((B, H, H, res), device='cuda', generator=g)
        segs.append(K.Seg(K.View.full(xr), [(0, 0)], kbase=nt * Ci))
    if mode in ('x6', 'f3', 'wino') and nt != 9 or mode in ('f3', 'wino') and not prologue:
        return None, None, None
    if mode == 'wino':
        ww = K.pack_wino(w, Ci, res)
        xb = torch.full((B, ), 8.0, device='cuda') if res else None
        fn = lambda: K.conv3x3_wino(segs, ww, b, K.View.full(out), Hm=H, Wm=H, a_exp=4, a_bound=xb)  # noqa: E731
    elif mode == 'f3':  # a_exp 4 keeps |x*sc + sh| * 16 far inside fp16 for these synthetic inputs
        w3 = K.pack_f16x3(w, Ci, res, res_f16=bool(res))
        xb = torch.full((B, ), 8.0, device='cuda') if res else None  # |randn| residual input < 8
        fn = lambda: K.conv3x3_f16x3(segs, w3, b, K.View.full(out), Hm=H, Wm=H, a_exp=4, a_bound=xb)  # noqa: E731
    elif mode == 'igx6':
        w6 = K.pack_x6(w, Ci, res, ntaps=nt, order='natural')
        fn = lambda: K.conv_igemm_x6(segs, w6, b, K.View.full(out), Hm=H, Wm=H)  # noqa: E731
    elif mode == 'x6':
        w6 = K.pack_x6(w, Ci, res)
        fn = lambda: K.conv3x3_x6(segs, w6, b, K.View.full(out), Hm=H, Wm=H)  # noqa: E731
    else:
        fn = lambda: K.conv_igemm(segs, w, b, K.View.full(out), Hm=H, Wm=H)  # noqa: E731
    t = timeit(fn)
    fl = 2.0 * B * H * H * Co * (nt * Ci + res)
    err = None
    if check:
        xx = x.permute(0, 3, 1, 2)
        a = xx * sc[:, :, None, None] + sh[:, :, None, None] if prologue else xx
        if prologue and nt > 1:
            a = F.silu(a)
        k = 3 if nt == 9 else 1
        wt = w[:, :nt * Ci].reshape(Co, k, k, Ci).permute(0, 3, 1, 2)
        torch.backends.cudnn.allow_tf32 = False
        ref = F.conv2d(a, wt, b, padding=k // 2)
        if res:
            ref = ref + F.conv2d(xr.permute(0, 3, 1, 2), w[:, nt * Ci:].reshape(Co, res, 1, 1))
        fn()
        torch.cuda.synchronize()
        got = out.permute(0, 3, 1, 2)
        err = float((got.double() - ref.double()).norm() / ref.double().norm())
    return t, fl / t / 1e12, err


TAPS4S2 = [(ky - 1, kx - 1) for ky in range(4) for kx in range(4)]


def igf3_case(B, H, Ci, Co, prologue, kind, check=False):
    """wc_conv_igemm_f16x3 on the projection / down-conv shapes: kind '1x1' (attention in/out
    projection) or 'down' (4x4 stride-2 pad-1, output H/2)."""
    g = torch.Generator(device='cuda').manual_seed(0)
    taps, st = ([(0, 0)], 1) if kind == '1x1' else (TAPS4S2, 2)
    Hm = H // st
    nt = len(taps)
    x = torch.randn((B, H, H, Ci), device='cuda', generator=g)
    w = torch.randn((Co, nt * Ci), device='cuda', generator=g) / (nt * Ci)**0.5
    b = torch.randn(Co, device='cuda', generator=g)
    sc = torch.rand((B, Ci), device='cuda', generator=g) + 0.5 if prologue else None
    sh = torch.randn((B, Ci), device='cuda', generator=g) * 0.1 if prologue else None
    out = torch.empty((B, Hm, Hm, Co), device='cuda')
    seg = K.Seg(K.View.full(x), taps, stride=st, scale=sc, shift=sh)
    w3 = K.pack_f16x3(w, Ci, ntaps=nt, order='natural')
    bound = None if prologue else torch.full((B, ), 8.0, device='cuda')
    fn = lambda: K.conv_igemm_f16x3([seg], w3, b, K.View.full(out), Hm=Hm, Wm=Hm, a_exp=4 if prologue else 60,  # noqa: E731
                                    a_bound=bound)
    t = timeit(fn)
    fl = 2.0 * B * Hm * Hm * Co * nt * Ci
    err = None
    if check:
        xx = x.permute(0, 3, 1, 2)
        a = xx * sc[:, :, None, None] + sh[:, :, None, None] if prologue else xx
        k = 1 if kind == '1x1' else 4
        wt = w.reshape(Co, k, k, Ci).permute(0, 3, 1, 2)
        torch.backends.cudnn.allow_tf32 = False
        ref = F.conv2d(a, wt, b, stride=st, padding=0 if k == 1 else 1)
        fn()
        torch.cuda.synchronize()
        err = float((out.permute(0, 3, 1, 2).double() - ref.double()).norm() / ref.double().norm())
    return t, fl / t / 1e12, err


IGF3_CASES = [(16, 64, 512, 1536, True, '1x1'), (16, 32, 768, 2304, True, '1x1'), (16, 64, 128, 384, True, '1x1'),
              (16, 64, 512, 512, False, '1x1'), (16, 32, 768, 768, False, '1x1'), (16, 256, 128, 128, False, 'down'),
              (16, 128, 256, 256, False, 'down'), (16, 64, 512, 512, False, 'down')]


def gn_case(B, H, C, ldc=None):
    ldc = ldc or C
    x = torch.randn((B, H, H, ldc), device='cuda')
    g = torch.ones(C, device='cuda')
    v = K.View(x, 0, C)
    t = timeit(lambda: K.gn_affine(v, g, g))
    return t, B * H * H * C * 4 / t / 1e9


def attn_case(B, N, C, prec='fp32'):
    qkv = torch.randn((B * N, 3 * C), device='cuda')
    o = torch.empty((B * N, C), device='cuda')
    exps = (10, 10, 10) if prec == 'f16x3' else None  # |randn| * 2^10 stays far inside fp16
    t = timeit(lambda: K.attention(qkv, o, B, N, C, 4, prec, exps))
    fl = 4.0 * B * N * N * C
    return t, fl / t / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--check', action='store_true')
    ap.add_argument('--only', type=int, default=-1, help='run a single conv case (for PMC profiling)')
    ap.add_argument('--modes', default='fp32,x6,f3,igx6',
                    help='conv kernels to time: fp32, x6 (halo 3x3 bf16x6), f3 (halo 3x3 f16x3), igx6, igf3 (projections / down convs)')
    ap.add_argument('--attn-only', type=int, default=-1, help='time only this f16x3 attention case (PMC)')
    ap.add_argument('--no-misc', action='store_true', help='skip the GroupNorm / attention timings')
    ap.add_argument('--zeros', action='store_true', help='all-zero activations (clock/power experiment)')
    a = ap.parse_args()
    global ZEROS
    ZEROS = a.zeros
    K._native.load()
    if a.attn_only >= 0:
        c = [(16, 4096, 512), (16, 1024, 768), (16, 1024, 512), (16, 4096, 128), (16, 1024, 256)][a.attn_only]
        t, tf = attn_case(*c, prec='f16x3')
        print(f'attn f16x3 B={c[0]} N={c[1]} C={c[2]}: {t*1e3:8.3f} ms  {tf:6.1f} TF/s', flush=True)
        return
    cases = [(16, 256, 128, 128, True, 0), (16, 256, 128, 128, True, 64), (16, 256, 64, 64, True, 0),
             (16, 128, 256, 256, True, 0), (16, 64, 512, 512, True, 0), (16, 32, 768, 768, True, 0),
             (16, 32, 1024, 256, True, 0), (16, 256, 64, 128, False, 0),
             (16, 64, 512, 1536, True, 0, [(0, 0)]), (16, 32, 768, 768, False, 0, [(0, 0)])]
    tot_t = tot_f = 0
    if a.only >= 0:
        cases = [cases[a.only]]
    for mode in a.modes.split(','):
        tot_t = tot_f = 0
        if mode == 'igf3':
            for c in (IGF3_CASES if a.only < 0 else [IGF3_CASES[a.only]]):
                t, tf, err = igf3_case(*c, check=a.check)
                tot_t += t
                tot_f += tf * t
                print(f'igf3 {c[5]:4s} B={c[0]} S={c[1]} {c[2]}->{c[3]} prologue={c[4]}: {t*1e3:8.3f} ms  {tf:6.1f} TF/s'
                      + (f'  relL2={err:.2e}' if err is not None else ''), flush=True)
            print(f'igf3 conv aggregate {tot_f / tot_t:.1f} TF/s')
            continue
        for c in cases:
            t, tf, err = conv_case(*c[:6], check=a.check, mode=mode, taps=c[6] if len(c) > 6 else None)
            if t is None:
                continue
            tot_t += t
            tot_f += tf * t
            print(f'{mode:4s} conv{"1x1" if len(c) > 6 else "3x3"} B={c[0]} S={c[1]} {c[2]}->{c[3]} prologue={c[4]} res={c[5]}: {t*1e3:8.3f} ms  '
                  f'{tf:6.1f} TF/s' + (f'  relL2={err:.2e}' if err is not None else ''), flush=True)
        print(f'{mode} conv aggregate {tot_f / tot_t:.1f} TF/s')
    if a.only >= 0 or a.no_misc:
        return
    for c in [(16, 256, 128), (16, 256, 64), (16, 128, 256), (16, 64, 512), (16, 32, 768), (16, 256, 128, 256)]:
        t, gbs = gn_case(*c)
        print(f'gn B={c[0]} S={c[1]} C={c[2]} ldc={c[3] if len(c) > 3 else c[2]}: {t*1e3:8.3f} ms  {gbs:7.1f} GB/s',
              flush=True)
    for prec in ('fp32', 'bf16x6', 'f16x3'):
        for c in [(16, 4096, 512), (16, 1024, 768), (16, 1024, 512), (16, 4096, 128), (16, 1024, 256)]:
            t, tf = attn_case(*c, prec=prec)
            print(f'attn {prec:6s} B={c[0]} N={c[1]} C={c[2]}: {t*1e3:8.3f} ms  {tf:6.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
