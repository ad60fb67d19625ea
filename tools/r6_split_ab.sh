#!/bin/bash
# same-box A/B of the graph's stream groups (WC_GRAPH_SPLIT 1 / 2 / 4), 60-step bench each, two rounds
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for s in 1 2 4; do
    WC_GRAPH_SPLIT=$s timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline --no-parity > gpurun_out/r6split_${s}_$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r6split_${s}_$r.log; exit $rc; }
    echo "split $s round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6split_${s}_$r.log)"
  done
done
