#!/bin/bash
# Same-box A/B of image groups on concurrent streams inside the graph (bench --split 1 / 2 / 4).
mkdir -p gpurun_out
for s in 1 2 1 2 4; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --split $s --no-roofline --no-parity --no-cpu-baseline > gpurun_out/split_$s.json 2> gpurun_out/split_$s.err
  rc=$?; echo "split $s rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/split_$s.json'));print(d['ms_per_step'])")"; [ $rc -ne 0 ] && { tail -5 gpurun_out/split_$s.err; exit $rc; }
done
exit 0
