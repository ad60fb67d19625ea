#!/bin/bash
# FETCH_SIZE of the pre-split Winograd conv vs batch: what part of its L2 fill traffic is the per-XCD
# weight stream (fixed per launch) and what part scales with the images
export TMPDIR=/tmp
O=gpurun_out/vpfetch; mkdir -p $O
for shp in "32 768 768" "64 512 512"; do
  for B in 4 8 16; do
    tag=$(echo "$shp $B" | tr ' ' '_')
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/$tag -o p -- python3 tools/wino_one.py $shp $B ${shp##* } > $O/$tag.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$tag rc=$rc"; tail -3 $O/$tag.log; exit $rc; }
    python3 - "$O/$tag" "$tag" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r['Kernel_Name'][:60]].append(float(r['Counter_Value']))
for k, v in acc.items():
    if 'wino' in k:
        print(sys.argv[2], k, 'launches', len(v), 'FETCH_SIZE KB mean', round(sum(v) / len(v)))
PY
  done
done
