#!/bin/bash
# One-launch ConvT (and s2d down conv): kernel tests, the GPU suite, then a same-box A/B of the
# whole bench (WC_UP_CT=0: four implicit-GEMM parities, 1: one halo-kernel launch).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_x6.py -q -x --timeout 120 --timeout-method thread -k "s2d or resampling or convT" > gpurun_out/s2d_tests.log 2>&1
rc=$?; echo kernel_tests_rc=$rc; tail -3 gpurun_out/s2d_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in 0 1; do
    WC_UP_CT=$v timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/ct_$v$r.log 2>&1
    rc=$?; echo ct_${v}_${r}_rc=$rc; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ct_$v$r.log
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/ct_$v$r.log; exit $rc; fi
  done
done
