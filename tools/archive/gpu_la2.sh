#!/bin/bash
# Weights two taps ahead around the halo issue: GPU tests under the variant, bench A/B
# (WC_CONV3_LA2 0 / 1 / 1r interleaved), conv shapes per variant.
mkdir -p gpurun_out
WC_CONV3_LA2=1r timeout -k 10 500 python -u -m pytest tests/test_x6.py tests/test_gpu_unet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/la2_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 gpurun_out/la2_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/la2_test.log | head -20; exit $rc; fi
for m in 0 1 1r 0 1 1r; do
  WC_CONV3_LA2=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/la2_bench_$m.log 2>&1 || exit 1
  echo "la2=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/la2_bench_$m.log) $(grep -o '"rel_l2": [0-9.e-]*' gpurun_out/la2_bench_$m.log)"
done
for m in 0 1r; do
  WC_CONV3_LA2=$m timeout -k 10 300 python -u tools/prof_shapes.py > gpurun_out/la2_shapes_$m.log 2>&1 || exit 1
  echo "== la2=$m"; grep -E "conv3x3" gpurun_out/la2_shapes_$m.log | head -12
done
