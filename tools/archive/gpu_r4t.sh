#!/bin/bash
# Training backward small-op pass: GN backward / channel-sum / bsum tests, the training gradient tests,
# the training line, and its kernel summary.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py \
    -k "groupnorm_backward or channel_sums or unet_grads or deterministic or accumulate" > gpurun_out/t_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/t_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/t_tests.log | head; exit $rc; }
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/t_train.log 2>&1
rc=$?; echo train_rc=$rc; tail -1 gpurun_out/t_train.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/t_prof -o run -- python3 tools/bench_train.py --steps 3 --warmup 1 > gpurun_out/t_prof.log 2>&1
rc=$?; echo prof_rc=$rc; exit $rc
