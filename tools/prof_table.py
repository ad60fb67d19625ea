"""Per-step table of a rocprofv3 kernel_stats.csv: python tools/prof_table.py CSV [launches_of_a_reference_kernel_per_step]."""
import csv
import sys


def main(path, steps=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    if steps is None:  # conv_in runs once per UNet forward
        steps = next(int(r['Calls']) for r in rows if 'conv_in' in r['Name'] and 'kernel' in r['Name'])
    print(f'{"kernel":48s} {"calls/fwd":>9s} {"avg_us":>9s} {"ms/fwd":>7s} {"pct":>6s}')
    for r in rows:
        n = r['Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
        ms = float(r['TotalDurationNs']) / steps / 1e6
        if ms < 0.05:
            continue
        print(f"{n[:48]:48s} {int(r['Calls']) / steps:9.1f} {float(r['AverageNs']) / 1e3:9.1f} {ms:7.2f} "
              f"{float(r['Percentage']):6.2f}")
    print(f'forwards {steps}, total kernel ms per forward {tot / steps / 1e6:.2f}')


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
