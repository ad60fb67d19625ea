#!/bin/bash
# round-6: the 2D Winograd position-major conv -- its tests, the UNet goldens through it, then a same-box
# A/B of the sampling bench (WC_WINO2D 1 / 0) and the Winograd launch table
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wino2d.py -m gpu -x -v -rf --timeout 120 --timeout-method thread > gpurun_out/r6w2d_tests.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r6w2d_tests.txt | tail -14; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/r6w2d_unet.txt 2>&1; rc=$?
tail -2 gpurun_out/r6w2d_unet.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/r6w2d_unet.txt | head; exit $rc; }
for r in 1 2; do
  for v in 1 0; do
    WC_WINO2D=$v timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline --no-parity > gpurun_out/r6w2d_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r6w2d_${v}_$r.log; exit 1; }
    echo "WC_WINO2D=$v round $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6w2d_${v}_$r.log)"
  done
done
WINO_SHAPES=1 timeout -k 10 300 python -u tools/launch_shapes.py wino > gpurun_out/r6w2d_shapes.txt 2>&1 || { tail -5 gpurun_out/r6w2d_shapes.txt; exit 1; }
tail -1 gpurun_out/r6w2d_shapes.txt
