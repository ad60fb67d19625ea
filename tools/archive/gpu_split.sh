#!/bin/bash
# Same-box A/B of the graph batch split (WC_GRAPH_SPLIT = 1, 2, 4, 1) on a 60-step bench, after an
# equality check of the split graph against the unsplit one.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probes/split_check.py > gpurun_out/split_check.log 2>&1
rc=$?; echo check_rc=$rc; grep -v amdgpu.ids gpurun_out/split_check.log
if [ $rc -ne 0 ]; then exit $rc; fi
for sp in 1 2 4 1; do
  WC_GRAPH_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/split_$sp.log 2>&1
  rc=$?; echo split_${sp}_rc=$rc; grep -o '"ms_per_step": [0-9.]*' gpurun_out/split_$sp.log
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/split_$sp.log; exit $rc; fi
done
