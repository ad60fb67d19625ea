#!/bin/bash
# Round 3: the whole GPU test suite (per-test durations), logs under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -x --timeout 120 --timeout-method thread --durations=25 > gpurun_out/r3_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -30 gpurun_out/r3_test.log
exit $rc
