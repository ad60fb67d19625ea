#!/bin/bash
# Training (config 3): GPU train tests, then the training-step bench with the halo wgrad (default) and
# without it (WC_WGRAD3=0) on the same box.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/train_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/train_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/train_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 --profile > gpurun_out/train_b1.log 2>&1
rc=$?; echo b1_rc=$rc; tail -1 gpurun_out/train_b1.log | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
WC_WGRAD3=0 timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/train_b0.log 2>&1
rc=$?; echo b0_rc=$rc; tail -1 gpurun_out/train_b0.log | cut -c1-400
exit $rc
