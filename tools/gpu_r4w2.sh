#!/bin/bash
# EXPERIMENTAL 2D Winograd: GPU parity test, then the conv1-shape timing probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino.py \
    -m gpu -k "wino2d or vs_float64" > gpurun_out/w2_test.log 2>&1 && \
timeout -k 10 300 python -u tools/wino2d_probe.py > gpurun_out/w2_probe.log 2>&1
