"""Per-kernel stats from rocprofv3's SQLite output (run_results.db): calls, total ms, average us, for
kernels matching a substring; two databases side by side for an A/B.
Usage: python tools/rocpd_stats.py A.db [B.db] [--match gnb_]"""
import argparse
import sqlite3
from collections import defaultdict


def stats(db):
    c = sqlite3.connect(db)
    out = defaultdict(lambda: [0, 0.0])
    for name, dur in c.execute('select name, duration from kernels'):
        out[name][0] += 1
        out[name][1] += dur / 1e6
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dbs', nargs='+')
    ap.add_argument('--match', default='')
    ap.add_argument('--top', type=int, default=40)
    a = ap.parse_args()
    ss = [stats(d) for d in a.dbs]
    names = sorted(ss[0], key=lambda k: -ss[0][k][1])
    names = [n for n in names if a.match in n][:a.top]
    hdr = f"{'kernel':80s}" + ''.join(f"{'calls':>7s}{'total_ms':>10s}{'avg_us':>9s}" for _ in ss)
    print(hdr)
    for n in names:
        row = f'{n[:80]:80s}'
        for s in ss:
            k, t = s.get(n, [0, 0.0])
            row += f'{k:7d}{t:10.3f}{(1000 * t / k if k else 0):9.2f}'
        print(row)
    print(f"{'TOTAL':80s}" + ''.join(f"{sum(v[0] for v in s.values()):7d}{sum(v[1] for v in s.values()):10.3f}{'':9s}" for s in ss))


if __name__ == '__main__':
    main()
