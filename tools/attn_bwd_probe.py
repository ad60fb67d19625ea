"""The training attention backward in isolation (PMC / timing probe): B x N tokens, C channels, heads,
f16x3 (wc_attention_bwd_f16x3) after the f16x3 LSE forward, on random inputs.
    python tools/attn_bwd_probe.py [--B 32 --N 4096 --C 512 --heads 4 --reps 3]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--B', type=int, default=32)
    ap.add_argument('--N', type=int, default=4096)
    ap.add_argument('--C', type=int, default=512)
    ap.add_argument('--heads', type=int, default=4)
    ap.add_argument('--reps', type=int, default=3)
    a = ap.parse_args()
    from weatherconverter_amd import kernels as K
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, N, C, H = a.B, a.N, a.C, a.heads
    qkv = torch.randn((B * N, 3 * C), device=dev, generator=g)
    do = torch.randn((B * N, C), device=dev, generator=g)
    o = torch.empty((B * N, C), device=dev)
    lse = torch.empty((B, H, N), device=dev)
    exps = (10, 10, 10)
    K.attention_fwd_lse(qkv, o, lse, B, N, C, H, precision='f16x3', exps=exps)
    dob = do.abs().reshape(B, -1).amax(1)
    dqkv = torch.empty_like(qkv)
    K.attention_bwd(qkv, o, do, lse, dqkv, B, N, C, H, precision='f16x3', exps=exps, dout_bound=dob)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        K.attention_bwd(qkv, o, do, lse, dqkv, B, N, C, H, precision='f16x3', exps=exps, dout_bound=dob)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    flops = 10.0 * B * N * N * C
    print(json.dumps({'B': B, 'N': N, 'C': C, 'heads': H, 'ms': round(ms, 3),
                      'tflops_algorithmic': round(flops / (ms * 1e-3) / 1e12, 1)}))


if __name__ == '__main__':
    main()
