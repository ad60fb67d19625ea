"""Summarise tools/probes/mfma_peak.hip's waves-per-SIMD sweep: the un-profiled rates (jsonl) and,
from a separate rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES pass over the same binary,
each launch's effective clock and MFMA-busy fraction.  Dispatches are matched to sweep points in
launch order (per point: one warm-up launch then three timed ones).
usage: python tools/mfma_sweep_table.py <sweep.jsonl> <pmc dir>"""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict

rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')]
points = []  # (mfma, wps) in launch order
for r in rows:
    k = (r['mfma'], r['waves_per_simd'])
    if not points or points[-1] != k:
        points.append(k)
rate = defaultdict(list)
for r in rows:
    rate[(r['mfma'], r['waves_per_simd'])].append(r['tflops'])
clk = {}
if len(sys.argv) > 2:
    d = sys.argv[2]
    agg = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0])):
        agg[int(r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
    dur = {int(r['Dispatch_Id']): (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
           for r in csv.DictReader(open(glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0]))}
    disp = sorted(k for k in agg if k in dur)
    # 4 launches per point (warm-up + 3); keep the timed three
    for i, pt in enumerate(points):
        ds = disp[4 * i + 1:4 * i + 4]
        c = [agg[x]['GRBM_GUI_ACTIVE'] / 8 / dur[x] / 1e9 for x in ds]
        b = [agg[x]['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (agg[x]['GRBM_GUI_ACTIVE'] / 8) for x in ds]
        clk[pt] = (statistics.median(c), statistics.median(b))
print(f'{"mfma":22s} {"waves/SIMD":>10s} {"TF/s (median of 3)":>19s} {"of peak":>8s} {"clock GHz":>10s} {"MFMA busy":>10s}')
best = {}
for pt in points:
    tf = statistics.median(rate[pt])
    peak = 157.3 if pt[0].endswith('f32') else 2516.6
    c, b = clk.get(pt, (float('nan'), float('nan')))
    print(f'{pt[0]:22s} {pt[1]:>10d} {tf:>19.1f} {tf / peak:>8.3f} {c:>10.2f} {b:>10.2f}')
    if tf > best.get(pt[0], (0, 0))[0]:
        best[pt[0]] = (tf, pt[1])
print('max over the sweep:', json.dumps({k: {'tflops': v[0], 'waves_per_simd': v[1]} for k, v in best.items()}))
