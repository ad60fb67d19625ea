#!/bin/bash
# round-6: GroupNorm-backward sums in the data-gradient conv's epilogue -- tests, then same-box A/B of both
# training lines (WC_TRAIN_GNB_EPI 1 vs 0)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_wino.py tests/test_gpu_train.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r6gnb_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r6gnb_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/r6gnb_tests.txt | head -20; exit $rc; }
for v in 1 0 1 0; do
  WC_TRAIN_GNB_EPI=$v timeout -k 10 600 python -u tools/bench_train.py --precision bf16 --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/r6gnb_bf16_$v.log 2>&1 || { tail -5 gpurun_out/r6gnb_bf16_$v.log; exit 1; }
  echo "bf16 GNB_EPI=$v: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r6gnb_bf16_$v.log)"
done
for v in 1 0; do
  WC_TRAIN_GNB_EPI=$v timeout -k 10 600 python -u tools/bench_train.py --steps 6 --warmup 2 --no-roofline --no-cpu-baseline > gpurun_out/r6gnb_f32_$v.log 2>&1 || { tail -5 gpurun_out/r6gnb_f32_$v.log; exit 1; }
  echo "fp32-class GNB_EPI=$v: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r6gnb_f32_$v.log)"
done
