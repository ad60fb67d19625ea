#!/bin/bash
# Training after: absmax pass without per-element division, unrolled GN-backward finalize, forward GroupNorm
# statistics from the producing convs' epilogues.  Training tests, then the iteration A/B (partials off / on).
mkdir -p gpurun_out/r04k
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04k/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/r04k/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r04k/tests.log | head -20; exit $rc; }
for r in 1 2; do
  for v in 0 1; do
    WC_TRAIN_GN_PARTIALS=$v timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/r04k/b$v$r.log 2>&1
    rc=$?; echo "partials=$v rc=$rc $(tail -1 gpurun_out/r04k/b$v$r.log | cut -c1-260)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
