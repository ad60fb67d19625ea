"""Per-step kernel table of the timed, graph-replayed sampling steps from a rocprofv3 kernel trace.

Usage: python tools/step_table.py <rocprof output dir or kernel_trace.csv> <timed steps K> [--json out]

A sampling step ends with exactly one ``ddpm_step_kernel`` (the fused scheduler update).  The timed
region of ``bench.py --steps K`` is the LAST K such steps of the trace; every kernel that starts
after the previous step's ddpm kernel ended and ends no later than this step's ddpm kernel belongs to
this step.  Untimed work (the packing forward, warmup, graph capture, roofline re-issues and
``torch.cuda._sleep`` spin kernels) lies outside those windows.  Prints, per kernel instantiation
(full template arguments, so the two instantiations of one kernel are separate rows), calls per
step, mean duration, ms per step and share, plus the per-step span (ddpm end to ddpm end) and the
summed kernel time, which must agree with bench.py's ms_per_step.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(path):
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)
        if not cands:
            raise SystemExit(f'no *kernel_trace.csv under {path}')
        path = cands[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    return rows


def short(name):
    n = name[5:] if name.startswith('void ') else name
    n = n.replace('(anonymous namespace)::', '')
    return re.sub(r'\(.*', '', n)


def table(rows, K):
    ends = [(s, e) for s, e, n in rows if 'ddpm_step_kernel' in n]
    if len(ends) < K + 1:
        raise SystemExit(f'only {len(ends)} ddpm_step launches in the trace, need {K + 1}')
    windows = [(ends[i - 1][1], ends[i][1]) for i in range(len(ends) - K, len(ends))]
    agg = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for lo, hi in windows:
        for s, e, n in rows:
            if s >= lo and e <= hi:
                a = agg[short(n)]
                a[0] += 1
                a[1] += (e - s) * 1e-3
                busy += (e - s) * 1e-3
    span_us = sum(hi - lo for lo, hi in windows) * 1e-3 / K
    out = {'steps': K, 'span_ms_per_step': round(span_us / 1e3, 4), 'kernel_ms_per_step': round(busy / K / 1e3, 4),
           'kernels': []}
    for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out['kernels'].append({'kernel': name, 'calls_per_step': round(n / K, 3), 'avg_us': round(us / n, 2),
                               'ms_per_step': round(us / K / 1e3, 4), 'share': round(us / busy, 4)})
    return out


def main():
    path, K = sys.argv[1], int(sys.argv[2])
    res = table(load(path), K)
    print(f'{"kernel":100s} {"calls/step":>10s} {"avg_us":>9s} {"ms/step":>8s} {"share":>6s}')
    for k in res['kernels']:
        print(f'{k["kernel"][:100]:100s} {k["calls_per_step"]:10.2f} {k["avg_us"]:9.2f} {k["ms_per_step"]:8.3f} '
              f'{100 * k["share"]:6.2f}')
    print(f'steps {res["steps"]}: span {res["span_ms_per_step"]:.3f} ms/step (ddpm end to ddpm end), '
          f'kernel time {res["kernel_ms_per_step"]:.3f} ms/step')
    if '--json' in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index('--json') + 1], 'w'), indent=1)


if __name__ == '__main__':
    main()
