#!/bin/bash
# Pre-split projections: GPU tests, then bench A/B (WC_PROJ_PA 1 / 0 interleaved) and per-shape times.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_x6.py tests/test_gpu_unet.py tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pa_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 gpurun_out/pa_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/pa_test.log | head -20; exit $rc; fi
for m in 1 0 1 0; do
  WC_PROJ_PA=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/pa_bench_$m.log 2>&1 || exit 1
  echo "pa=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pa_bench_$m.log) $(grep -o '"rel_l2": [0-9.e-]*' gpurun_out/pa_bench_$m.log)"
done
timeout -k 10 300 python -u tools/prof_shapes.py > gpurun_out/pa_shapes.log 2>&1 || exit 1
grep -E "igemm|split|head_conv|attention" gpurun_out/pa_shapes.log
