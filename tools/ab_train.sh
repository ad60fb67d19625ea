#!/bin/bash
# Same-box A/B of the bf16 training line: this tree's bf16 library (new) against lib/altbf (old, a
# tools/build_alt.sh VARIANT=bf16 build), alternating; then one rocprofv3 kernel-stats pass of each.
# Usage: TAG=x bash tools/ab_train.sh
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p gpurun_out
ALT=$PWD/weatherconverter_amd/lib/altbf/libwc_kernels.so
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 600 python -u tools/bench_train.py --precision bf16 --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/${TAG}_$tag.log 2>&1 || { tail -5 gpurun_out/${TAG}_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/${TAG}_$tag.log)"
}
for r in 1 2 3; do
  run new_$r WC_X=1
  run old_$r WC_KERNEL_LIB_BF16=$ALT WC_ALLOW_STALE_LIB=1
done
for v in new old; do
  if [ $v = old ]; then export WC_KERNEL_LIB_BF16=$ALT WC_ALLOW_STALE_LIB=1; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$v -o run -- python -u tools/bench_train.py --precision bf16 --steps 2 --warmup 1 --no-roofline --no-cpu-baseline > gpurun_out/${TAG}_prof_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$v.log; exit 1; }
done
