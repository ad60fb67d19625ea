#!/bin/bash
# bf16 training line, three-way same-box A/B of the generic weight gradient: this tree (XCD-aware block
# order), lib/altbf32 (the same at 32 pixels per barrier, tools/build_alt.sh WORK -DWG_KP1=32) and lib/altbf
# (HEAD's wc_backward); tests first.   usage: TAG=x bash tools/r6_wgrad_ab.sh
export TMPDIR=/tmp
TAG=${TAG:-wgab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py \
  -k "wgrad or 16bit_training_lines" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
L=$PWD/weatherconverter_amd/lib
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 600 python -u tools/bench_train.py --precision bf16 --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/${TAG}_$tag.log 2>&1 || { tail -5 gpurun_out/${TAG}_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/${TAG}_$tag.log)"
}
for r in 1 2; do
  run new_$r WC_X=1 || exit 1
  run kp32_$r WC_KERNEL_LIB_BF16=$L/altbf32/libwc_kernels.so WC_ALLOW_STALE_LIB=1 || exit 1
  run old_$r WC_KERNEL_LIB_BF16=$L/altbf/libwc_kernels.so WC_ALLOW_STALE_LIB=1 || exit 1
done
for v in new old; do
  if [ $v = old ]; then export WC_KERNEL_LIB_BF16=$L/altbf/libwc_kernels.so WC_ALLOW_STALE_LIB=1; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$v -o run -- python -u tools/bench_train.py --precision bf16 --steps 2 --warmup 1 --no-roofline --no-cpu-baseline > gpurun_out/${TAG}_prof_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$v.log; exit 1; }
done
echo done
