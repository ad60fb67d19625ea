#!/bin/bash
# Attention with buffer-load DMA, folded softmax scaling and fma_mix splits: GPU tests, then
# same-box A/B against the library in lib/alt (the previous attention), per-shape times.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/at2_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 gpurun_out/at2_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/at2_test.log | head -20; exit $rc; fi
bash tools/archive/gpu_ab_lib.sh || exit 1
timeout -k 10 300 python -u tools/prof_shapes.py > gpurun_out/at2_shapes.log 2>&1 || exit 1
grep -E "attention|split" gpurun_out/at2_shapes.log
