"""GPU idle time inside the timed sampling steps of a rocprofv3 kernel trace (tools/steptable.sh):
per step (ddpm end to ddpm end) the span, the union of kernel intervals (busy), the idle remainder, and
the idle gaps longer than 2 us with the kernels on either side.  Usage: idle_gaps.py <trace dir> <K>"""
import sys
from collections import Counter

from step_table import load, short


def main():
    rows = load(sys.argv[1])
    K = int(sys.argv[2])
    ddpm = [i for i, r in enumerate(rows) if 'ddpm_step_kernel' in r[2]]
    ddpm = ddpm[-(K + 1):]
    spans, busy_t, gaps = [], [], Counter()
    gap_us = Counter()
    for a, b in zip(ddpm, ddpm[1:]):
        t0, t1 = rows[a][1], rows[b][1]
        ks = sorted((s, e, n) for s, e, n in rows if s >= t0 and e <= t1)
        busy, cur_s, cur_e, prev = 0, None, None, rows[a][2]
        for s, e, n in ks:
            if cur_e is None:
                if s - t0 > 2000:
                    gaps[(short(prev)[:40], short(n)[:40])] += 1
                    gap_us[(short(prev)[:40], short(n)[:40])] += (s - t0) / 1e3
                cur_s, cur_e = s, e
            elif s > cur_e:
                busy += cur_e - cur_s
                if s - cur_e > 2000:
                    gaps[(short(prev)[:40], short(n)[:40])] += 1
                    gap_us[(short(prev)[:40], short(n)[:40])] += (s - cur_e) / 1e3
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev = n
        if cur_e is not None:
            busy += cur_e - cur_s
        spans.append((t1 - t0) / 1e6)
        busy_t.append(busy / 1e6)
    n = len(spans)
    print(f'steps {n}: span {sum(spans) / n:.3f} ms, GPU busy (union of kernels) {sum(busy_t) / n:.3f} ms, '
          f'idle {(sum(spans) - sum(busy_t)) / n:.3f} ms per step')
    print('idle gaps > 2 us (per step: count, us):')
    for k, c in gaps.most_common(15):
        print(f'  {c / n:5.2f} x {gap_us[k] / c:7.1f} us   after {k[0]:40s} before {k[1]}')


if __name__ == '__main__':
    sys.path.insert(0, __file__.rsplit('/', 1)[0])
    main()
