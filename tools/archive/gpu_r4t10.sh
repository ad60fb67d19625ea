#!/bin/bash
# Padded LDS rows + 16-byte reads in the Winograd packs: pack bit-identity tests + the Winograd conv tests, the training line,
# and a kernel trace (pack_wino_batch_kernel per iteration; was 1.25 ms).
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_wino.py \
    -k "pack or wino" -m gpu > gpurun_out/t10_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/t10_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/t10_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/t10_train.log 2>&1
rc=$?; echo "train rc=$rc $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/t10_train.log)"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/t10_prof -o run -- python3 tools/bench_train.py --steps 3 --warmup 1 > gpurun_out/t10_prof.log 2>&1
rc=$?; echo prof_rc=$rc; exit $rc
