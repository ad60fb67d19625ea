#!/bin/bash
# Projection GEMM tile raster (WC_IG_GM bands): tests, then a same-box sampling bench A/B of this tree
# against lib/alt (tools/build_alt.sh WORK wc_igemm6 with EXTRA=-DWC_IG_GM=1: the plain N-fastest order)
# and a kernel-stats pass of each.   usage: TAG=x bash tools/r6_igemm_ab.sh
export TMPDIR=/tmp
TAG=${TAG:-igab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_x6.py tests/test_gpu_unet.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
TAG=${TAG}_b ARMS="tree alt" REPS=3 bash tools/ab_bench.sh || exit 1
for arm in tree alt; do
  if [ $arm = alt ]; then export WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/alt/libwc_kernels.so WC_ALLOW_STALE_LIB=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$arm -o run -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/${TAG}_prof_$arm.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$arm.log; exit 1; }
done
echo done
