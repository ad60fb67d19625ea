#!/bin/bash
# Training-backward GPU tests (kernels first, then the whole model).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -v -x --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/pytest_train.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "PASS|FAIL|ERROR|passed|failed|overall|Error|error" gpurun_out/pytest_train.log | head -40
exit $rc
