#!/bin/bash
# Weights-in-registers for the fp16-residual 3x3 forms: GPU tests, then bench A/B (WC_CONV3_WR_RES 1 / 0).
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_x6.py tests/test_gpu_unet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/wr_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 gpurun_out/wr_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/wr_test.log | head -20; exit $rc; fi
for m in 1 0 1 0; do
  WC_CONV3_WR_RES=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/wr_bench_$m.log 2>&1 || exit 1
  echo "wr_res=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wr_bench_$m.log) $(grep -o '"rel_l2": [0-9.e-]*' gpurun_out/wr_bench_$m.log)"
done
timeout -k 10 300 python -u tools/prof_shapes.py > gpurun_out/wr_shapes.log 2>&1 || exit 1
grep -E "conv3x3" gpurun_out/wr_shapes.log | head -20
