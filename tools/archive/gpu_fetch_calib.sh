#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/calib/f -o p -- python3 tools/fetch_calib.py > gpurun_out/calib/f.log 2>&1
rc=$?; echo rc=$rc; [ $rc -ne 0 ] && { tail -5 gpurun_out/calib/f.log; exit $rc; }
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob('gpurun_out/calib/f/**/p_counter_collection.csv', recursive=True)[0])))
agg = {}
for r in rows:
    if r['Counter_Name'] == 'FETCH_SIZE' and 'absmax' in r['Kernel_Name']:
        agg[r['Dispatch_Id']] = agg.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
for d, v in agg.items():
    print(f'dispatch {d}: FETCH_SIZE {v:.0f} KB = {v * 1024 / 2**30:.3f} GiB for a 4.000 GiB read (x2 = {2 * v * 1024 / 2**30:.3f})')
PY
