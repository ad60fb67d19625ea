#!/usr/bin/env python
"""bench.py — BASELINE.json metric: 256x256 images/sec for T=1000 DDPM sampling (+ ms/UNet-step).

One "step" = one reverse-diffusion step over the per-GPU batch: a full UNet forward on the HIP
engine + the fused scheduler update (reference sample_ddpm.py:37-44).  The timed region runs
EXACTLY --steps consecutive steps of the T=1000 schedule starting at t=999 (default 1000 = one
complete sample, x_T -> x_0, including the final all-gather of x_0 when N>1); images/s =
(images in flight) * (steps / T) / elapsed, so a full run is the literal job throughput.

Workload (BASELINE config 2 at N=1, config 5 at N=8): S=256, 16 images per GPU (weak scaling),
fp32, the default config.yaml UNet (110.08 M params) with keyed synthetic weights, Philox device
noise keyed by (seed, global sample, step).

Launch: python bench.py [--gpus N --steps K --warmup W].  N>1: under torch.distributed.run (RCCL,
WORLD_SIZE must equal --gpus); without WORLD_SIZE in the environment bench.py starts
``torch.distributed.run --nproc-per-node N`` itself as a child process (before any GPU call) and exits
with its code.  Rank 0 prints ONE JSON line.  Extra legs (rank 0, after the timed region):
  roofline      per-launch HIP events around every conv of one UNet forward; the dominant kernel
                is the conv instantiation with the most time (the GN+SiLU-prologue 3x3 convs) —
                achieved = its algorithmic (fp32-equivalent) FLOPs per launch / its mean launch
                duration, against its own ceiling: 157.3 TF for the fp32-MFMA conv, 2516.6/6 =
                419.4 TF for bf16x6 kernels (6 bf16 MFMAs per fp32 product), 2516.6/3 = 838.9 TF
                for the f16x3 conv (3 f16 MFMAs per product; MI355X_MICROARCH.md).
  parity        the committed 256-px golden input (reference unet_base.Unet output, tests/golden/
                unet_256.npz) through the same engine / arithmetic that was timed: rel-L2 vs the golden.
  cpu_baseline  the oracle's PyTorch-CPU restatement of the reference UNet step (N=1 only), at the
                timed batch (B=16) on every CPU this process may use, a bounded sample (1-3 steps
                after one warmup, ~10-30 s), extrapolated x T.
"""
import argparse
import glob
import json
import math
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 MFMA (= vector) peak, MI355X_MICROARCH.md
# bf16x6 conv: every fp32-equivalent 32x32x16 block costs 6 bf16 MFMAs, so its ceiling is the dense
# bf16 MFMA peak (256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz = 2516.6 TF/s) / 6.
BF16X6_PEAK_TFLOPS = round(2516.6 / 6, 1)
# f16x3 conv: 3 f16 MFMAs (same rate as bf16) per fp32-equivalent block.
F16X3_PEAK_TFLOPS = round(2516.6 / 3, 1)
DENSE16_PEAK_TFLOPS = 2516.6  # dense f16 / bf16 MFMA peak (256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz)
HBM_PEAK_GBS = 8000.0
GFLOP_PER_IMAGE_STEP_256 = 590.61  # SURVEY.md §8(d) algorithmic FLOPs (probe hook count)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='GPUs of this node (default: WORLD_SIZE, else 1); N>1 without WORLD_SIZE self-launches')
    ap.add_argument('--steps', type=int, default=1000)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=16, help='images per GPU')
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--timesteps', type=int, default=1000)
    ap.add_argument('--seed', type=int, default=3455)
    ap.add_argument('--graph', type=int, default=1, help='replay the UNet forward from a HIP graph')
    ap.add_argument('--split', type=int, default=None,
                    help='image groups per GPU run concurrently on their own streams inside the graph '
                         '(default: _GraphStep\'s, 2 at >= 16 images per GPU; WC_GRAPH_SPLIT)')
    ap.add_argument('--vp-wide', type=int, default=0,
                    help='eager runs (--graph 0): the pre-split convs in the form the two-group graph uses '
                         '(kernels.wino_vp_wide), so a PMC pass at --batch B/2 sees the timed instantiations')
    ap.add_argument('--no-roofline', action='store_true')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-batch', type=int, default=None, help='CPU baseline batch (default: --batch)')
    ap.add_argument('--cpu-steps', type=int, default=3, help='at most this many timed CPU steps')
    ap.add_argument('--cpu-budget', type=float, default=20.0, help='stop timing CPU steps after ~this many s')
    ap.add_argument('--no-parity', action='store_true')
    ap.add_argument('--precision', default=None, choices=['f16x3', 'bf16x6', 'fp32'],
                    help='conv/attention arithmetic (default: kernels.default_conv_precision(), i.e. f16x3)')
    ap.add_argument('--pg', action='store_true',
                    help='initialise the process group and run the N-rank code (collectives included) even at '
                         'world size 1 (exercises the RCCL branch on a one-GPU box)')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='process-group backend for N>1: nccl (= RCCL over xGMI, the benched path) or gloo '
                         '(x0 gather staged through host memory; lets N ranks share one GPU for rehearsal)')
    return ap.parse_args(argv)


KERNEL_DESC = {
    'conv3x3_x6': 'split-precision MFMA 3x3 conv, halo-tiled, GN+SiLU prologue',
    'conv_igemm_x6': 'split-precision MFMA implicit-GEMM conv / projection',
    'attention_x6': 'split-precision MFMA flash attention',
    'conv_igemm_kernel': 'fp32 MFMA implicit-GEMM conv',
    'attention_kernel': 'fp32 MFMA flash attention',
    'proj_pa_kernel': 'split-precision MFMA pre-split projection GEMM',
    'conv3x3_w1_kernel': 'split-precision MFMA 3x3 conv, one wave per SIMD, 16 x 16-pixel tiles',
    'conv3x3_wino_kernel': 'split-precision MFMA 3x3 conv through Winograd F(2,3) along x (12 K-steps per 16-channel '
                           'chunk and output pair instead of 18: 2/3 of the direct MFMA work), GN+SiLU prologue',
}


def _describe(name: str) -> str:
    """Human description of a kernel instantiation (rocprofv3 name, all template arguments)."""
    base = name.split('<')[0]
    targs = name[name.index('<') + 1:name.rindex('>')].split(', ') if '<' in name else []
    mode = 'f16x3' if _mode_peak(name) == F16X3_PEAK_TFLOPS else ('bf16x6' if _mode_peak(name) == BF16X6_PEAK_TFLOPS
                                                                   else 'fp32')
    d = KERNEL_DESC.get(base, base)
    if base == 'conv3x3_wino_kernel' and len(targs) >= 4 and targs[3] == 'true':
        d += ', fused 1x1 residual in positions 0 / 3'
    if base == 'conv3x3_x6_kernel' and len(targs) >= 9:
        if targs[7] == '1':
            d = 'split-precision MFMA 4x4/s2 down conv over the space-to-depth input (halo-tiled)'
        elif targs[7] == '2':
            d = 'split-precision MFMA ConvTranspose 4x4/s2, four parities per halo'
        elif targs[3] == 'true':
            d += ', fused 1x1 residual' + (' interleaved per chunk' if targs[8] == '3' else '') + (
                ' in f16x3 under the per-image GN bound' if targs[5] == 'true' else ' in bf16x6')
        if targs[8] != '0':
            d += ', weights in registers'
    return f'{mode}: {d}'


def _is_hbm(name: str) -> bool:
    return name.startswith(('gn_', 'split_', 'wino_vsplit'))


def _stamp_overhead(slots, n: int = 65) -> float:
    """Seconds one wc_stamp node adds to a replayed graph: n stamps captured back to back, the median
    interval between consecutive ones."""
    from weatherconverter_amd import _native, kernels
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(n):
            _native.call('wc_stamp', slots.data_ptr(), i, kernels._stream())
    g.replay()
    torch.cuda.synchronize()
    v = slots[:n].cpu().tolist()
    del g
    d = sorted(b - a for a, b in zip(v, v[1:]))
    return d[len(d) // 2] / kernels.wall_clock_hz()


def ingraph_timing(model, x, t_dev, reps: int = 3):
    """Per-launch durations INSIDE a replayed HIP graph, as the timed steps run them.  One UNet forward is
    captured with a wc_stamp node (a one-wave kernel writing the GPU wall clock, kernels.stamp_timing) on
    each side of every named launch and replayed `reps` times; a launch's duration = the clock
    difference of its two stamps minus one stamp node's own share of the graph (measured by
    _stamp_overhead), averaged over the replays.  (torch refuses timed event-record nodes in ROCm graph
    capture, so the clock is read by the graph itself.)  Returns ({instantiation: [launches, flops, sec,
    bytes, issued mfma flops]} per forward, the stamped graph's wall per replay, the sum of the
    per-launch durations, the stamp overhead)."""
    from weatherconverter_amd import kernels
    hz = kernels.wall_clock_hz()
    x_in, t_in = x.clone(), t_dev.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        model(x_in, t_in)  # allocations / packs outside the capture
    torch.cuda.current_stream().wait_stream(side)
    slots = torch.zeros(16384, dtype=torch.int64, device=x.device)
    over = _stamp_overhead(slots)
    g = torch.cuda.CUDAGraph()
    st = kernels.stamp_timing(slots)
    try:
        with torch.cuda.graph(g):
            model(x_in, t_in)
    finally:
        kernels.stamp_timing(None)
    launches = st['launches']
    per, walls = {}, []
    for name, flops, nbytes, mfma in launches:
        d = per.setdefault(name, [0, 0.0, 0.0, 0.0, 0.0])
        d[0] += 1
        d[1] += flops
        d[3] += nbytes
        d[4] += mfma if mfma is not None else flops * _pieces(name)
    for _ in range(reps):
        w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        w0.record()
        g.replay()
        w1.record()
        torch.cuda.synchronize()
        walls.append(w0.elapsed_time(w1) * 1e-3)
        v = slots[:2 * len(launches)].cpu().tolist()
        for i, (name, *_) in enumerate(launches):
            per[name][2] += ((v[2 * i + 1] - v[2 * i]) / hz - over) / reps
    del g
    total = sum(v[2] for v in per.values())
    return per, sum(walls) / len(walls), total, over


def reissue_timing(model, x, t_dev):
    """Every conv / projection / attention launch of one eager forward re-issued 5x back to back right
    after itself between one HIP event pair (kernels.replay_timing('*')): the per-instantiation table
    of rounds 3-5, kept beside the in-graph one."""
    from weatherconverter_amd import kernels
    rep = kernels.replay_timing('*', reps=5)
    torch.cuda._sleep(1 << 28)
    with torch.no_grad():
        model(x, t_dev)
    torch.cuda.synchronize()
    kernels.replay_timing(None)
    per = {}
    for name, flops, r0, r1, reps, nbytes, mfma in rep['events']:
        d = per.setdefault(name, [0, 0.0, 0.0, 0.0, 0.0])
        d[0] += 1
        d[1] += flops
        d[2] += r0.elapsed_time(r1) * 1e-3 / reps
        d[3] += nbytes
        d[4] += mfma if mfma is not None else flops * _pieces(name)
    return per


def roofline_leg(model, x, t_dev, groups: int = 1):
    """Per-kernel timing of one UNet forward as the timed graph runs it.

    Primary: ingraph_timing -- a HIP event pair around every named launch inside a replayed graph of
    the forward (same kernels, arguments and order as the timed steps), keyed by the exact
    instantiation the library reports (rocprofv3's name), so the table lines up with the rocprofv3
    trace of the timed replays (tools/step_table.py).  The dominant kernel = the MFMA instantiation
    with the most in-graph time per forward; achieved = its algorithmic (fp32-equivalent) FLOPs per
    launch / its in-graph mean duration, against its arithmetic mode's ceiling.  The round-3..5
    re-issue table (reissue_timing) rides along as mean_launch_ms_reissue."""
    with torch.no_grad():
        model(x, t_dev)  # packs / allocations outside the measured forward
    torch.cuda.synchronize()
    src = ('in-graph: GPU wall-clock stamps (wc_stamp nodes) around each launch inside a replayed HIP graph of '
           'the forward, minus one stamp node; mean of 3 replays')
    graph_wall = graph_sum = over = None
    try:
        with torch.no_grad():
            per_all, graph_wall, graph_sum, over = ingraph_timing(model, x, t_dev)
    except Exception as e:  # noqa: BLE001 -- report the fallback in the line instead of failing the bench
        per_all = None
        src = f'in-graph stamps failed ({type(e).__name__}: {e}); each launch re-issued 5x between one event pair'
    rei = reissue_timing(model, x, t_dev)
    if per_all is None:
        per_all = rei
    per = {k: v for k, v in per_all.items() if not _is_hbm(k)}
    hbm = {k: v for k, v in per_all.items() if _is_hbm(k)}
    name = max(per, key=lambda k: per[k][2])
    n, fl, sec, abytes, issued = per[name]
    mean_dur = sec / n
    achieved = (fl / n) / mean_dur / 1e12
    peak = _mode_peak(name)
    total_mfma = sum(v[2] for v in per.values())
    # HBM bytes per launch of this kernel from the committed two-pass PMC measurement
    # (tools/pmc_traffic.sh: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM), if present
    traffic, traffic_src = None, None
    for path in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles',
                                              '*_hbm_traffic.json')))[-1:]:
        recs = json.load(open(path))
        rec = recs.get(name)
        if rec:
            traffic = round(rec['total_bytes'] / 1e9, 4)
            traffic_src = (f'{os.path.relpath(path, os.path.dirname(os.path.abspath(__file__)))}: GB per launch '
                           f'(read {rec["read_bytes"] / 1e9:.3f} + write {rec["write_bytes"] / 1e9:.3f}), '
                           f'mean over {rec["launches"]} launches'
                           + (f'; algorithmic {rec["algorithmic_bytes"] / 1e9:.3f}' if 'algorithmic_bytes' in rec
                              else ''))
    rn = rei.get(name)
    if not abytes and rn and rn[3]:  # the stamped launches carry no byte count: the re-issue table's, per launch
        abytes = rn[3] / rn[0] * n
    # what a bare f16 MFMA stream sustains on this power-capped chip: the MAXIMUM over the committed
    # waves-per-SIMD sweep (tools/probes/mfma_peak.hip, median of each point's three launches; the
    # best point is one wave per SIMD issuing back to back), the split-precision kernels' work
    # against it, beside the data-sheet peak
    sustained = None
    probe = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'r04a_mfma_sweep.jsonl')
    if peak == F16X3_PEAK_TFLOPS and os.path.exists(probe):
        pts = {}
        for r in map(json.loads, open(probe)):
            if r.get('mfma') == 'f32_32x32x16_f16':
                pts.setdefault(r['waves_per_simd'], []).append(r['tflops'])
        if pts:
            med = {w: sorted(v)[len(v) // 2] for w, v in pts.items()}
            wbest = max(med, key=med.get)
            f16 = med[wbest]
            sustained = {'f16_mfma_tflops': f16, 'fp32_equiv_tflops': round(f16 / 3, 1),
                         'frac': round(achieved / (f16 / 3), 4), 'waves_per_simd': wbest,
                         'sweep_f16_tflops_by_waves_per_simd': {str(w): med[w] for w in sorted(med)},
                         'source': 'profiles/r04a_mfma_sweep.jsonl (tools/probes/mfma_peak.hip: back-to-back '
                                   'v_mfma_f32_32x32x16_f16, waves/SIMD 8/4/3/2/1, ~70 ms launches on random '
                                   'operands; the max over the sweep of each point\'s median; clock and MFMA busy '
                                   'per point: profiles/r04a_mfma_sweep_table.txt)'}
    return {
        'kernel': name,
        'kernel_desc': _describe(name),
        'bound': 'mfma',
        'achieved': round(achieved, 2),
        'peak': peak,
        'unit': 'TFLOP/s',
        'frac': round(achieved / peak, 4),
        # the matrix pipe's view: dense 16-bit MFMA FLOPs this kernel ISSUES per launch (pieces x, for the
        # Winograd conv, 2/3 of the direct form's products on its 3x3 segment) / time, against the 2516.6
        # TF/s dense f16/bf16 peak and against the sustained one-wave stream (frac above can exceed what
        # the pipe does: it prices the direct conv's FLOPs)
        'mfma_pipe': _pipe_leg(issued / n, mean_dur, sustained),
        'sustained_mfma_stream': sustained,
        'traffic': traffic,
        'traffic_source': traffic_src,
        'launches_per_step': n * groups,
        'images_per_launch': int(x.shape[0]),
        'mean_launch_ms': round(mean_dur * 1e3, 4),
        'mean_launch_ms_source': src,
        'mean_launch_ms_reissue': round(rn[2] / rn[0] * 1e3, 4) if rn else None,
        'ingraph_stamped_forward_ms': round(graph_wall * 1e3, 3) if graph_wall else None,
        'ingraph_launch_sum_ms': round(graph_sum * 1e3, 3) if graph_sum else None,
        'ingraph_stamp_node_us': round(over * 1e6, 3) if over is not None else None,
        'gflop_per_launch': round(fl / n / 1e9, 3),
        'algorithmic_gb_per_launch': round(abytes / n / 1e9, 4) if abytes else None,
        'traffic_over_algorithmic': round(traffic / (abytes / n / 1e9), 3) if (traffic and abytes) else None,
        'share_of_mfma_time': round(sec / max(total_mfma, 1e-12), 3),
        'mfma_ms_per_forward': round(total_mfma * 1e3 * groups, 3),
        'mfma_kernels': {k: {'launches': v[0] * groups, 'ms': round(v[2] * 1e3 * groups, 3),
                             'tflops': round(v[1] / v[2] / 1e12, 1), 'peak': _mode_peak(k),
                             'frac': round(v[1] / v[2] / 1e12 / _mode_peak(k), 4),
                             'mfma_pipe_frac': round(v[4] / v[2] / 1e12 / DENSE16_PEAK_TFLOPS, 4),
                             'desc': _describe(k)}
                         for k, v in sorted(per.items(), key=lambda kv: -kv[1][2])},
        'hbm_kernels': hbm_leg(hbm, groups),
    }


def _pieces(name: str) -> int:
    """16-bit MFMAs per fp32-equivalent product of an instantiation's arithmetic mode (fp32 MFMA: 0, not
    on the 16-bit pipe)."""
    p = _mode_peak(name)
    return 3 if p == F16X3_PEAK_TFLOPS else (6 if p == BF16X6_PEAK_TFLOPS else 0)


def _pipe_leg(issued_per_launch: float, mean_dur: float, sustained) -> dict:
    rate = issued_per_launch / mean_dur / 1e12
    out = {'issued_gflop_per_launch': round(issued_per_launch / 1e9, 3), 'issued_tflops': round(rate, 1),
           'peak': DENSE16_PEAK_TFLOPS, 'mfma_pipe_frac': round(rate / DENSE16_PEAK_TFLOPS, 4)}
    if sustained:
        out['vs_sustained_stream'] = round(rate / sustained['f16_mfma_tflops'], 4)
        out['sustained_stream_tflops'] = sustained['f16_mfma_tflops']
    return out


def _mode_peak(name: str) -> float:
    """The emulated-fp32 ceiling of a profiled MFMA kernel instantiation: f16x3 (3 f16 MFMAs per
    block), bf16x6 (6 bf16 MFMAs) or plain fp32 MFMA."""
    if '<' not in name:
        return FP32_PEAK_TFLOPS
    targs = name[name.index('<') + 1:name.rindex('>')].split(', ')
    if name.startswith('conv3x3_x6'):
        return F16X3_PEAK_TFLOPS if len(targs) >= 5 and targs[4] == 'true' else BF16X6_PEAK_TFLOPS
    if name.startswith('conv_igemm_x6'):
        return F16X3_PEAK_TFLOPS if len(targs) >= 6 and targs[5] == 'true' else BF16X6_PEAK_TFLOPS
    if name.startswith('attention_x6'):
        return F16X3_PEAK_TFLOPS if targs[1] == 'true' else BF16X6_PEAK_TFLOPS
    if name.startswith(('conv3x3_w1_kernel', 'proj_pa_kernel', 'conv3x3_wino_kernel')):  # f16x3-only forms
        return F16X3_PEAK_TFLOPS
    # training kernels (tools/bench_train.py): the attention backward <D, F3, ...>, the 3x3 weight gradient
    # <WM, TH, PRO, F3>, the generic weight gradient <BM, BN, PRO, X6, F3>
    if name.startswith(('attn_bwd6_dq_kernel', 'attn_bwd6_dkdv_kernel')):
        return F16X3_PEAK_TFLOPS if len(targs) >= 2 and targs[1] == 'true' else BF16X6_PEAK_TFLOPS
    if name.startswith('conv_wgrad3_kernel'):
        return F16X3_PEAK_TFLOPS if len(targs) >= 4 and targs[3] == 'true' else BF16X6_PEAK_TFLOPS
    if name.startswith('conv_wgrad_kernel'):
        if len(targs) >= 5 and targs[4] == 'true':
            return F16X3_PEAK_TFLOPS
        return BF16X6_PEAK_TFLOPS if len(targs) >= 4 and targs[3] == 'true' else FP32_PEAK_TFLOPS
    return FP32_PEAK_TFLOPS


def hbm_leg(hbm, groups: int = 1):
    """The HBM-bound kernels of the forward: GroupNorm+SiLU are applied in the convs' prologues, so
    what stays on HBM is the statistics pass (one read of the activation, 4 B/element) and the
    pre-split of the projection operand (read 4 + write 4 B/element); achieved GB/s over every
    launch of one forward against the 8 TB/s HBM peak.  The byte count is the launch's stated nbytes,
    else its 'flops' field (the HBM wrappers state bytes there)."""
    if not hbm:
        return None
    out = {}
    for k, (n, fl, sec, nb, *_) in hbm.items():
        by = nb or fl
        out[k] = {'launches': n * groups, 'ms': round(sec * 1e3 * groups, 3), 'gbytes': round(by * groups / 1e9, 3),
                  'achieved': round(by / sec / 1e9, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                  'frac': round(by / sec / 1e9 / HBM_PEAK_GBS, 4)}
    return out


def _cpu_share() -> dict:
    """CPUs this process may actually use: its affinity mask, capped by the cgroup CPU quota (a GPU box
    shows the whole machine in nproc / os.cpu_count() but grants each GPU a share of it)."""
    host = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = host
    quota = None
    try:
        q, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = affinity if quota is None else max(1, min(affinity, int(math.floor(quota))))
    model = None
    try:
        for line in subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if line.startswith('Model name:'):
                model = line.split(':', 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    nproc = None
    try:
        nproc = int(subprocess.run(['nproc'], capture_output=True, text=True, timeout=10).stdout.strip())
    except (OSError, subprocess.SubprocessError, ValueError):
        pass
    return {'host_cpus': host, 'nproc': nproc, 'affinity_cpus': affinity, 'cgroup_cpu_quota': quota,
            'usable_cpus': usable, 'cpu_model': model}


def cpu_baseline_leg(args):
    """The reference UNet step restated op for op in PyTorch-CPU (oracle/), at the timed batch, on every
    CPU this process may use.  The oracle calls the same torch CPU ops as the reference import
    (including nn.MultiheadAttention's fused fast path): its forwards are bitwise-equal to the
    reference's at equal thread count (tests/test_oracle_golden.py, 8 threads), and timed side by
    side with the imported reference in the build container it takes 1.005x the reference's time at
    256 px B=2 (profiles/r03_cpu_provenance.json, tools/cpu_provenance.py)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle.unet_oracle import unet_forward, unet_state_dict_keys
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.synthetic import synth_tensor
    share = _cpu_share()
    threads = share['usable_cpus']
    torch.set_num_threads(threads)
    B = args.cpu_batch or args.batch
    mc = model_config(args.size)
    sd = {k: synth_tensor(k, s) for k, s in unet_state_dict_keys(mc).items()}
    x = torch.randn((B, 3, args.size, args.size), generator=torch.Generator().manual_seed(1))
    t = torch.tensor([500])
    times = []
    with torch.no_grad():
        unet_forward(sd, mc, x, t)  # warm
        t_start = time.perf_counter()
        while len(times) < max(1, args.cpu_steps):
            t0 = time.perf_counter()
            unet_forward(sd, mc, x, t)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_start > args.cpu_budget:
                break
    dt = sum(times) / len(times)
    return {
        'value': round(B / (dt * args.timesteps), 7),
        'unit': 'images/s',
        'cores': threads,
        'kind': 'port',
        'ms_per_step': round(dt * 1e3, 1),
        'host': share,
        'provenance': 'profiles/r03_cpu_provenance.json: oracle bitwise-equal to the imported reference, '
                      '1.005x its CPU time (256 px, B=2, 8 threads, build container)',
        'sample': f'oracle PyTorch-CPU UNet step (reference unet_base.Unet restated op for op), {args.size}px, '
                  f'B={B}, {len(times)} timed step(s) after 1 warmup on {threads} threads (the CPUs this process '
                  f'may use: affinity capped by the cgroup quota), extrapolated x{args.timesteps} (T) -- '
                  f'extrapolated, not a full sample'
    }


def parity_leg(model, dev):
    """The committed 256-px golden (reference unet_base.Unet on the keyed synthetic weights,
    tests/golden/make_golden.py) through the engine and arithmetic that was just timed."""
    import numpy as np
    from weatherconverter_amd.synthetic import state_dict_digest, synthetic_images
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'tests', 'golden', 'unet_256.npz')
    g = np.load(path)
    digest_ok = state_dict_digest({k: v.detach().cpu() for k, v in model.state_dict().items()}) == str(g['digest'])
    x = synthetic_images((1, 3, 256, 256), seed=301).to(dev)
    with torch.no_grad():
        y = model(x, torch.tensor([611], device=dev)).double().cpu()
    ref = torch.from_numpy(g['y']).double()
    rel = float((y - ref).norm() / ref.norm())
    return {'rel_l2': float(f'{rel:.3e}'), 'tolerance': 1e-5, 'pass': bool(digest_ok and rel <= 1e-5),
            'weights_digest_match': digest_ok,
            'case': 'tests/golden/unet_256.npz: reference Unet (config.yaml @256px) forward, x seed 301, t=611, B=1'}


def _launch_cmd(gpus: int, argv, port: int):
    """The torch.distributed.run command line for --gpus N>1 (one rank per GPU, loopback rendezvous)."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={gpus}',
            '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + list(argv)


def _profiler_preloaded() -> bool:
    """True when a profiler library is preloaded into this process (``rocprofv3 -- python bench.py``):
    it has initialised the GPU before main() runs, so spawning the launcher from here is the
    fork-after-GPU-init pattern this pool forbids."""
    if 'rocprof' in os.environ.get('LD_PRELOAD', ''):
        return True
    try:
        with open('/proc/self/maps') as f:
            # librocprofiler-register ships inside torch itself; the profiler's tool library is the SDK's
            return 'rocprofiler-sdk' in f.read()
    except OSError:
        return False


def _self_launch(args) -> int:
    """--gpus N>1 outside torch.distributed.run: start it as a child (nothing here has touched the GPU;
    the parent only waits and passes the exit code on).  Refused under a profiler preload."""
    if _profiler_preloaded():
        raise SystemExit('bench.py: --gpus N>1 would start torch.distributed.run from a process whose GPU '
                         'runtime is already loaded (profiler preload?); run it under torch.distributed.run '
                         'directly instead')
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    return subprocess.call(_launch_cmd(args.gpus, sys.argv[1:], port))


def _world(args) -> int:
    """WORLD_SIZE, checked against --gpus when both are given."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}')
    return world


def _gather_x0(x, world: int, backend: str):
    """The one collective of the path: all-gather every rank's x0 block into the full batch.  RCCL
    gathers the device tensors in place over xGMI; gloo cannot gather device tensors, so its blocks are
    staged through host memory and the result copied back (as distributed.gather_samples does)."""
    if backend == 'nccl':
        out = torch.empty((x.shape[0] * world, ) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        dist.all_gather_into_tensor(out, x)
        return out
    xs = x.detach().cpu()
    parts = [torch.empty_like(xs) for _ in range(world)]
    dist.all_gather(parts, xs)
    return torch.cat(parts, 0).to(x.device)


def _gather_times(vals, world: int, backend: str, dev):
    """(world, len(vals)) float64 of every rank's timings (for the max-over-ranks rule)."""
    if backend == 'nccl':
        tt = torch.tensor(vals, device=dev, dtype=torch.float64)
        allt = torch.empty((world, len(vals)), device=dev, dtype=torch.float64)
        dist.all_gather_into_tensor(allt, tt)
        return allt.cpu()
    tt = torch.tensor(vals, dtype=torch.float64)
    parts = [torch.empty_like(tt) for _ in range(world)]
    dist.all_gather(parts, tt)
    return torch.stack(parts)


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and (args.gpus or 1) > 1:
        sys.exit(_self_launch(args))
    world = _world(args)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # one rank per GPU; under gloo more ranks than GPUs may share a card (rehearsal of the N-rank path
    # on a one-GPU box).  device_count() does not initialise the GPU on this image.
    ndev = max(1, torch.cuda.device_count())
    dev = torch.device('cuda', local % ndev if args.backend == 'gloo' else local)
    torch.cuda.set_device(dev)
    # the distributed code path: every rank count above one, or --pg at world size 1
    dist_on = world > 1 or args.pg
    if dist_on:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if 'MASTER_PORT' not in os.environ:
            with socket.socket() as sk:
                sk.bind(('127.0.0.1', 0))
                os.environ['MASTER_PORT'] = str(sk.getsockname()[1])
        os.environ.setdefault('RANK', str(rank))
        os.environ.setdefault('WORLD_SIZE', str(world))
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')

    from weatherconverter_amd import kernels
    from weatherconverter_amd.diffusion_model.config import model_config
    from weatherconverter_amd.diffusion_model.models.unet_base import Unet
    from weatherconverter_amd.diffusion_model.sample_ddpm import _GraphStep
    from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from weatherconverter_amd.synthetic import init_synthetic_

    mc = model_config(args.size)
    model = Unet(mc)
    init_synthetic_(model, seed=0)
    precision = args.precision or kernels.default_conv_precision()
    model.set_conv_precision(precision)
    model = model.to(dev).eval()
    sched = LinearNoiseScheduler(args.timesteps, 0.0001, 0.02, device=dev)
    B = args.batch
    T = args.timesteps
    K = min(args.steps, T)
    sample0 = rank * B
    shape = (B, mc.im_channels, mc.im_size, mc.im_size)
    ts = torch.arange(T, device=dev, dtype=torch.long)

    def barrier():
        if dist_on:
            dist.barrier()

    with torch.no_grad():
        x = kernels.philox_normal(shape, dev, args.seed, sample0=sample0, step=T)
        runner = _GraphStep(model, x, split=args.split) if args.graph else None
        if runner is not None:
            fwd = runner
        else:  # eager (PMC passes): --vp-wide 1 launches the kernel forms the two-group graph captures
            def fwd(xx, tt):
                with kernels.wino_vp_wide(bool(args.vp_wide)):
                    return model(xx, tt)
        nxt = torch.empty_like(x)
        # untimed warmup: W steps from a scratch copy
        xw = x.clone()
        for j in range(args.warmup):
            i = T - 1 - (j % T)
            eps = fwd(xw, ts[i:i + 1])
            sched.step(xw, eps, i, out=nxt, noise='philox', seed=args.seed, sample0=sample0)
            xw, nxt = nxt, xw
        del xw
        gathered = None
        gather_sec = 0.0
        if dist_on:  # communicator set up outside the timed region
            _gather_x0(x, world, args.backend)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(T - 1, T - 1 - K, -1):
            eps = fwd(x, ts[i:i + 1])
            if i == 0:
                sched.step(x, eps, 0, out=nxt)
            else:
                sched.step(x, eps, i, out=nxt, noise='philox', seed=args.seed, sample0=sample0)
            x, nxt = nxt, x
        if dist_on:
            torch.cuda.synchronize()
            g0 = time.perf_counter()
            gathered = _gather_x0(x, world, args.backend)
            torch.cuda.synchronize()
            gather_sec = time.perf_counter() - g0
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        per_rank = [elapsed]
        per_rank_gather = [gather_sec]
        if dist_on:
            allt = _gather_times([elapsed, gather_sec], world, args.backend, dev)
            per_rank = [float(v) for v in allt[:, 0].tolist()]
            per_rank_gather = [float(v) for v in allt[:, 1].tolist()]
            elapsed = max(per_rank)
        finite = bool(torch.isfinite(x).all())
        if gathered is not None:
            finite = finite and bool(torch.isfinite(gathered).all())

        result = None
        if rank == 0:
            images = B * world * K / T
            ms_step = elapsed / K * 1e3
            unet_tflops = GFLOP_PER_IMAGE_STEP_256 * B / (ms_step * 1e-3) / 1e3 if args.size == 256 else None
            result = {
                'metric': '256x256 images/sec (T=1000 DDPM sample)',
                'value': round(images / elapsed, 5),
                'unit': 'images/s',
                'n_gpus': world,
                'steps': K,
                'warmup': args.warmup,
                'ms_per_step': round(ms_step, 3),
                'higher_is_better': True,
                'scaling': 'weak',
                'vs_baseline': None,
                'dtype': {'f16x3': 'fp32-class (f16x3: 2-piece fp16 split MFMA, fp32 accumulate)',
                          'bf16x6': 'fp32-class (bf16x6: 3-piece bf16 split MFMA, fp32 accumulate)',
                          'fp32': 'f32 (fp32 MFMA)'}[precision],
                'data': 'synthetic (keyed random-init weights, Philox N(0,1) x_T and per-step noise)',
                'extrapolated_from_steps': None if K == T else
                f'{K} of T={T} steps timed; images/s = images x {K}/{T} / elapsed (UNet cost does not depend on t)',
                'config': {
                    'workload': f'DDPM reverse sampling, UNet config.yaml @ {args.size}px, {B} images/GPU, '
                                f'T={T}, {K} timed steps from t={T - 1}' + (' (complete sample)' if K == T else ''),
                    'global_batch': B * world,
                    'image_size': args.size,
                    'timesteps': T,
                    'parallelism': (f'batch-sharded x{world}, 1 all-gather of x0 over '
                                    + ('RCCL (xGMI)' if args.backend == 'nccl' else 'gloo (host-staged)'))
                    if dist_on else 'single GPU',
                    'backend': args.backend if dist_on else None,
                    'devices': torch.cuda.device_count(),
                    'hip_graph': bool(args.graph),
                    'stream_groups': runner.split if runner is not None else 1,
                    'arithmetic': {
                        'f16x3': 'fp32-class: 3x3 convs (with the fused 1x1 residual), attention projections and '
                                 'attention on f16x3 (2-piece fp16 split under power-of-two range bounds: Samuelson '
                                 'GN bound, in-projection row norms, per-image GN/absmax bounds measured by the '
                                 'producer for the residual, down convs and ConvT); operands without a bound on '
                                 'bf16x6 (exact 3-piece bf16 split); fp32 accumulation; fp32 activations in HBM',
                        'bf16x6': 'fp32-class: every conv and attention on bf16x6 (exact 3-piece bf16 split), fp32 '
                                  'accumulation; fp32 activations in HBM',
                        'fp32': 'fp32 MFMA (v_mfma_f32_32x32x2_f32) everywhere'}[precision],
                    'x_finite': finite,
                },
                'ms_per_unet_step': round(ms_step, 3),
                'per_rank_ms_per_step': [round(v / K * 1e3, 3) for v in per_rank],
                'all_gather_ms': [round(v * 1e3, 3) for v in per_rank_gather] if dist_on else None,
                'gathered_shape': list(gathered.shape) if gathered is not None else None,
                'unet_step_tflops_algorithmic': round(unet_tflops, 2) if unet_tflops else None,
            }
            if not args.no_roofline:
                # the dominant kernel as the timed graph launches it: one image group
                g = runner.split if runner is not None else 1
                from weatherconverter_amd.kernels import wino_vp_wide
                with wino_vp_wide(g > 1):  # the same instantiations as the timed graph (its groups' form)
                    result['roofline'] = roofline_leg(model, x[:B // g], ts[500:501], groups=g)
            if not args.no_parity and args.size == 256:
                result['parity'] = parity_leg(model, dev)
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            result['cpu_baseline'] = cpu_baseline_leg(args)
        else:
            result['cpu_baseline'] = None
        print(json.dumps(result), flush=True)
    if dist_on:
        # ranks 1..N-1 wait here for rank 0's roofline / parity / CPU-baseline legs before tearing the
        # communicator down
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
