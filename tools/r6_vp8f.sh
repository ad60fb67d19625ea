#!/bin/bash
# bench line: the two-group graph with (WC_WINO_VP8=1) and without (=0) the 8-wave pre-split form
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 1 0; do
    WC_WINO_VP8=$v timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/vp8f_${v}_$r.log 2>&1 || { tail -3 gpurun_out/vp8f_${v}_$r.log; exit 1; }
    echo "WC_WINO_VP8=$v $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vp8f_${v}_$r.log)"
  done
done
