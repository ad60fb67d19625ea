"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KB) reports half the bytes of 16-B-per-lane
streaming reads on gfx950 -> doubled (every hot-path load here is a 16-B buffer/global load);
WRITE_SIZE is exact for 16-B-per-lane stores, and the 4-B-per-lane epilogue stores of the conv kernels
are reported as measured (their calibration is printed against the known output bytes by bench).
Writes profiles/<tag>_hbm_traffic.json when a tag is given.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_kernel(d, counter):
    rows = list(csv.DictReader(open(glob.glob(d + '/**/p_counter_collection.csv', recursive=True)[0])))
    agg = defaultdict(float)
    names = {}
    for r in rows:
        if r['Counter_Name'] != counter:
            continue
        agg[r['Dispatch_Id']] += float(r['Counter_Value'])
        names[r['Dispatch_Id']] = r['Kernel_Name'].replace('void (anonymous namespace)::', '').split('(')[0]
    out = defaultdict(list)
    for k, v in agg.items():
        out[names[k]].append(v * 1024.0)  # KB -> bytes
    return out


def main(fetch_dir, write_dir, tag=None):
    f = per_kernel(fetch_dir, 'FETCH_SIZE')
    w = per_kernel(write_dir, 'WRITE_SIZE')
    res = {}
    for name in sorted(set(f) | set(w), key=lambda n: -sum(f.get(n, [0])) - sum(w.get(n, [0]))):
        fl, wl = f.get(name, []), w.get(name, [])
        fb = 2.0 * sum(fl) / len(fl) if fl else 0.0
        wb = sum(wl) / len(wl) if wl else 0.0
        res[name] = {'launches': len(fl) or len(wl), 'read_bytes': fb, 'write_bytes': wb, 'total_bytes': fb + wb}
    for name, r in list(res.items())[:20]:
        print(f"{name[:60]:60s} n={r['launches']:4d} read {r['read_bytes']/1e6:9.2f} MB  write "
              f"{r['write_bytes']/1e6:9.2f} MB per launch (avg over instantiations' launches)")
    if tag:
        json.dump(res, open(f'profiles/{tag}_hbm_traffic.json', 'w'), indent=1)


if __name__ == '__main__':
    main(*sys.argv[1:])
