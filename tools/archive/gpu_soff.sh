#!/bin/bash
# Conv loads with wave-uniform scalar offsets: GPU tests (default and WC_CONV3_LA2=1r), same-box
# A/B against lib/alt (the previous conv), then LA2 1r / 0 on this library.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_x6.py tests/test_gpu_unet.py tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread > gpurun_out/so_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -1 gpurun_out/so_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/so_test.log | head -20; exit $rc; fi
WC_CONV3_LA2=1r timeout -k 10 500 python -u -m pytest tests/test_x6.py tests/test_gpu_unet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/so_test2.log 2>&1
rc=$?; echo test2_rc=$rc; tail -1 gpurun_out/so_test2.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/so_test2.log | head -20; exit $rc; fi
bash tools/archive/gpu_ab_lib.sh || exit 1
for m in 1r 0 1r 0; do
  WC_CONV3_LA2=$m timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/so_la2_$m.log 2>&1 || exit 1
  echo "la2=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/so_la2_$m.log)"
done
