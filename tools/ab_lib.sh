#!/bin/bash
# Same-box A/B of a whole 60-step bench: the library in weatherconverter_amd/lib/alt (A) against
# this tree's library (B), alternating A B A B.
mkdir -p gpurun_out
ALT=$PWD/weatherconverter_amd/lib/alt/libwc_kernels.so
for r in 1 2; do
  WC_KERNEL_LIB=$ALT WC_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/ab_lib_a$r.log 2>&1
  rc=$?; echo a${r}_rc=$rc; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_lib_a$r.log
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_lib_a$r.log; exit $rc; fi
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/ab_lib_b$r.log 2>&1
  rc=$?; echo b${r}_rc=$rc; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_lib_b$r.log
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_lib_b$r.log; exit $rc; fi
done
