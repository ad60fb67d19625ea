"""Clock and MFMA-busy per kernel from tools/clock_probe.sh output (gpurun_out/clk)."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/clk'
rows = list(csv.DictReader(open(glob.glob(d + '/**/p_counter_collection.csv', recursive=True)[0])))
agg = defaultdict(lambda: defaultdict(float))
names = {}
for r in rows:
    agg[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
    names[r['Dispatch_Id']] = r['Kernel_Name'].replace('void (anonymous namespace)::', '').split('(')[0]
dur = {r['Dispatch_Id']: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
       for r in csv.DictReader(open(glob.glob(d + '/**/p_kernel_trace.csv', recursive=True)[0]))}
seen = defaultdict(list)
for k, v in agg.items():
    if k in dur and ('conv' in names[k] or 'attention' in names[k]):
        clk = v['GRBM_GUI_ACTIVE'] / 8 / dur[k] / 1e9
        busy = v['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (v['GRBM_GUI_ACTIVE'] / 8)
        seen[names[k]].append((clk, busy, dur[k] * 1e3))
for n, l in seen.items():
    l = l[2:] or l
    print(f'{n:60s} clock {sum(x[0] for x in l) / len(l):.2f} GHz  mfma_busy {sum(x[1] for x in l) / len(l):.2f}  '
          f'ms {sum(x[2] for x in l) / len(l):.3f}')
