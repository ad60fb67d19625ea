#!/bin/bash
# Two-waves-per-group GN finalize: the GroupNorm / UNet parity tests, then a same-box A/B of the
# sampling line (lib/alt = HEAD's wc_gn, A) against this tree (B), A B A B.
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
    -k "gn or groupnorm or golden or unet or wino" > gpurun_out/g_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/g_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/g_tests.log | head -20; exit $rc; }
bash tools/archive/gpu_ab_lib.sh
