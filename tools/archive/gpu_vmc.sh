#!/bin/bash
# Conv loads issued unconditionally (static vmcnt counts): GPU tests, same-box A/B against lib/alt,
# per-shape times.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_x6.py tests/test_gpu_unet.py tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread > gpurun_out/fu_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -1 gpurun_out/fu_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/fu_test.log | head -20; exit $rc; fi
bash tools/archive/gpu_ab_lib.sh || exit 1
timeout -k 10 300 python -u tools/prof_shapes.py > gpurun_out/fu_shapes.log 2>&1 || exit 1
grep -E "conv3x3" gpurun_out/fu_shapes.log | head -24
