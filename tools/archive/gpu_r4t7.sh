#!/bin/bash
# Coalesced attention-backward prep + lazy ConvT re-layouts: attention / training-gradient tests, then a
# kernel trace of the training line (attn_bwd_prep_kernel average; was 173 us).
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py \
    -k "attention or unet_grads or deterministic" > gpurun_out/t7_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/t7_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/t7_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/t7_train.log 2>&1
rc=$?; echo "train rc=$rc $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/t7_train.log)"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/t7_prof -o run -- python3 tools/bench_train.py --steps 3 --warmup 1 > gpurun_out/t7_prof.log 2>&1
rc=$?; echo prof_rc=$rc; exit $rc
