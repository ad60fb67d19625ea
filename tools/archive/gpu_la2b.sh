#!/bin/bash
# LA2 as default: GPU tests, bench A/B (WC_CONV3_LA2 1 / 0 interleaved)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/la2b_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 gpurun_out/la2b_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/la2b_test.log | head -20; exit $rc; fi
for m in 1 0 1 0; do
  WC_CONV3_LA2=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/la2b_bench_$m.log 2>&1 || exit 1
  echo "la2=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/la2b_bench_$m.log) $(grep -o '"rel_l2": [0-9.e-]*' gpurun_out/la2b_bench_$m.log)"
done
