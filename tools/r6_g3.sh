#!/bin/bash
# round-6: SRGAN / guided tests after the depthwise spill fix, then the config-4 guided line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_guided.py tests/test_guided_config4.py -m gpu -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/r06_g3_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/r06_g3_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/r06_g3_tests.txt | head; exit $rc; }
timeout -k 10 900 python3 -u tools/bench_guided.py > gpurun_out/r06b_guided.jsonl 2> gpurun_out/r06b_guided.err; rc=$?
echo guided_rc=$rc; [ $rc -ne 0 ] && { tail -8 gpurun_out/r06b_guided.err; exit $rc; }
cut -c1-300 gpurun_out/r06b_guided.jsonl
