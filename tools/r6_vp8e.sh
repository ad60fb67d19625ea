#!/bin/bash
# 8-wave pre-split form picked by the two-group graph: tests, then the bench line against HEAD (lib/alt)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_wino.py tests/test_gpu_unet.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r6vp8e_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/r6vp8e_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/r6vp8e_tests.txt | head; exit $rc; }
TAG=vp8e REPS=3 ARMS="tree alt" bash tools/ab_bench.sh
