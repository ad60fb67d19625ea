#!/bin/bash
# same-box A/B of the pre-split threshold WC_WINO_VP (min 128-channel output tiles) under the default
# two-group graph: sampling 60-step bench (4 / 2 / 1), then the bf16 training line (4 / 1)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 4 2 1; do
    WC_WINO_VP=$v timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline --no-parity > gpurun_out/r6vp_${v}_$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r6vp_${v}_$r.log; exit $rc; }
    echo "sampling VP $v round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6vp_${v}_$r.log)"
  done
done
for v in 4 1; do
  WC_WINO_VP=$v timeout -k 10 600 python -u tools/bench_train.py --precision bf16 --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/r6vp_train_${v}.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r6vp_train_${v}.log; exit $rc; }
  echo "train bf16 VP $v: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r6vp_train_${v}.log)"
done
