"""Achieved HBM bandwidth per kernel: bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE x 2 per
MI355X_MICROARCH.md §HBM, WRITE_SIZE) over the same command, durations from the passes' kernel traces.
usage: python tools/traffic_bw.py DIR_FETCH DIR_WRITE [top]   (tools/traffic_summary.py's inputs)"""
import csv
import glob
import sys
from collections import defaultdict

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from traffic_summary import per_kernel  # noqa: E402


def durations(d):
    out = defaultdict(list)
    for f in glob.glob(d + '/**/p_kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            name = r['Kernel_Name'].replace('void (anonymous namespace)::', '').split('(')[0]
            out[name].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9)
    return out


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    fetch, write, dur = per_kernel(fd, 'FETCH_SIZE'), per_kernel(wd, 'WRITE_SIZE'), durations(fd)
    rows = []
    for k, fs in fetch.items():
        ws = write.get(k, [0.0])
        ds = dur.get(k)
        if not ds:
            continue
        rd = 2.0 * sum(fs) / len(fs)  # FETCH_SIZE halves 16-B-per-lane reads on gfx950
        wr = sum(ws) / len(ws)
        t = sum(ds) / len(ds)
        rows.append((t * len(ds), k, len(ds), rd, wr, t))
    rows.sort(reverse=True)
    print(f'{"kernel":70s} {"n":>4s} {"read MB":>9s} {"write MB":>9s} {"avg us":>8s} {"GB/s":>7s} {"total ms":>9s}')
    for tot, k, n, rd, wr, t in rows[:top]:
        print(f'{k[:70]:70s} {n:4d} {rd / 1e6:9.1f} {wr / 1e6:9.1f} {t * 1e6:8.1f} {(rd + wr) / t / 1e9:7.0f} {tot * 1e3:9.2f}')


if __name__ == '__main__':
    main()
