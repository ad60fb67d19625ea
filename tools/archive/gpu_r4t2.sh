#!/bin/bash
# wgrad3 A/B (lib/alt = HEAD's wgrad3), then the training-path tests and the training line.
bash tools/archive/gpu_ab_w3.sh || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py \
    -k "groupnorm_backward or channel_sums or wgrad3 or unet_grads or deterministic or accumulate" > gpurun_out/t2_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/t2_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/t2_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/t2_train.log 2>&1
rc=$?; echo train_rc=$rc; tail -1 gpurun_out/t2_train.log | cut -c1-260; exit $rc
