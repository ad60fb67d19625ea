#!/bin/bash
# round-6: 8-wave 256-channel pre-split Winograd conv -- bit-identity tests, then same-box A/B against HEAD
# (lib/alt): the 40 Winograd launches of one B=16 forward, and the 60-step bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wino.py -m gpu -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/r6vp8_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/r6vp8_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/r6vp8_tests.txt | head; exit $rc; }
TAG=vp8 REPS=2 VARS="tree alt" bash tools/wino_ab.sh || exit 1
bash tools/ab_lib.sh
