#!/bin/bash
# Training (config 3): GPU train tests, the training-step bench (A/B: WC_DGRAD_F16X3=0 on the same
# box), and a rocprofv3 kernel trace of the step (kernel time vs wall: host gaps).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/train_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/train_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/train_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 --profile > gpurun_out/train_b1.log 2>&1
rc=$?; echo b1_rc=$rc; tail -1 gpurun_out/train_b1.log | cut -c1-1800; [ $rc -ne 0 ] && exit $rc
WC_DGRAD_F16X3=0 timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/train_b0.log 2>&1
rc=$?; echo b0_rc=$rc; tail -1 gpurun_out/train_b0.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
WC_ATTN_BWD6=0 timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/train_b2.log 2>&1
rc=$?; echo b2_rc=$rc; tail -1 gpurun_out/train_b2.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/train_prof -o run -- python3 -u tools/bench_train.py --steps 3 --warmup 2 > gpurun_out/train_prof.log 2>&1
rc=$?; echo prof_rc=$rc
python3 tools/prof_summary.py gpurun_out/train_prof > gpurun_out/train_prof_summary.txt 2>&1 || true
head -30 gpurun_out/train_prof_summary.txt | cut -c1-160
exit $rc
