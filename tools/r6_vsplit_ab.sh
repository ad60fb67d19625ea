#!/bin/bash
# Pre-split pass (wino_vsplit_kernel) A/B: tree (GN scale/shift once per thread, 4 items in flight) vs
# lib/alt (HEAD) vs lib/alt2 (the tree's form at 8 items in flight): presplit bit-identity tests, the
# 60-step bench x3, kernel stats of each arm.   usage: TAG=x bash tools/r6_vsplit_ab.sh
export TMPDIR=/tmp
TAG=${TAG:-vsab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_wino.py -k presplit \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
TAG=${TAG}_b ARMS="tree alt alt2" REPS=3 bash tools/ab_bench.sh || exit 1
for arm in tree alt alt2; do
  if [ $arm != tree ]; then export WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$arm/libwc_kernels.so WC_ALLOW_STALE_LIB=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$arm -o run -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/${TAG}_prof_$arm.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$arm.log; exit 1; }
done
echo done
