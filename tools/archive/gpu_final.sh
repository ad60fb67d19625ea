#!/bin/bash
# Round-end check: the whole GPU test suite, then the round evidence (tools/archive/gpu_r2_evidence.sh).
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/final_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 gpurun_out/final_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/final_test.log | head -20; exit $rc; fi
bash tools/archive/gpu_r2_evidence.sh
