"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_stats.csv) per kernel symbol."""
import csv, glob, os, re, sqlite3, sys
from collections import defaultdict


def from_db(path):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith('rocpd_kernel_dispatch')][0]
    ks = [t for t in tabs if t.startswith('rocpd_info_kernel_symbol')][0]
    names = {r[0]: r[1] for r in c.execute(f'select id, kernel_name from {ks}')}
    agg = defaultdict(list)
    for kid, st, en in c.execute(f'select kernel_id, start, end from {kd}'):
        agg[names.get(kid, str(kid))].append((en - st) * 1e-3)  # ns -> us
    return agg


def short(name):
    n = name[5:] if name.startswith('void ') else name
    n = n.replace('(anonymous namespace)::', '')
    return re.sub(r'\(.*', '', n)[:90]


def from_csv(path):
    agg = defaultdict(list)
    span = [None, None]
    with open(path) as f:
        for r in csv.DictReader(f):
            st, en = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            agg[r['Kernel_Name']].append((en - st) * 1e-3)
            span[0] = st if span[0] is None else min(span[0], st)
            span[1] = en if span[1] is None else max(span[1], en)
    return agg, span


def main(path):
    span = None
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, '**', '*.db'), recursive=True)
        csvs = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True)
        path = dbs[0] if dbs else csvs[0]
    if path.endswith('.csv'):
        agg, span = from_csv(path)
    else:
        agg = from_db(path)
    tot = sum(sum(v) for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    print(f'{"kernel":90s} {"calls":>6s} {"total_ms":>10s} {"avg_us":>10s} {"pct":>6s}')
    for k, v in rows:
        print(f'{short(k):90s} {len(v):6d} {sum(v)/1e3:10.3f} {sum(v)/len(v):10.2f} {100*sum(v)/tot:6.2f}')
    print(f'total kernel time {tot/1e3:.3f} ms' + (f'; trace span {(span[1] - span[0]) * 1e-6:.3f} ms' if span else ''))


if __name__ == '__main__':
    main(sys.argv[1])
