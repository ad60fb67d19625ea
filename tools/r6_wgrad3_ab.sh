#!/bin/bash
# Halo-row-major 3x3 weight gradient: tests, bit-identity digests against HEAD's kernel (lib/alt,
# lib/altbf: tools/build_alt.sh HEAD wc_wgrad3), then same-box A/Bs of both training lines and a
# kernel-stats pass of each bf16 arm.   usage: TAG=x bash tools/r6_wgrad3_ab.sh
export TMPDIR=/tmp
TAG=${TAG:-w3ab}
mkdir -p gpurun_out
L=$PWD/weatherconverter_amd/lib
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py \
  -k "wgrad3 or 16bit_training_lines or 256_baseline" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for line in f16x3 bf16; do
  timeout -k 10 120 python -u tools/wgrad3_digest.py --line $line > gpurun_out/${TAG}_dig_new_$line.txt 2>&1 || { tail -5 gpurun_out/${TAG}_dig_new_$line.txt; exit 1; }
  WC_KERNEL_LIB=$L/alt/libwc_kernels.so WC_KERNEL_LIB_BF16=$L/altbf/libwc_kernels.so WC_ALLOW_STALE_LIB=1 timeout -k 10 120 python -u tools/wgrad3_digest.py --line $line > gpurun_out/${TAG}_dig_old_$line.txt 2>&1 || { tail -5 gpurun_out/${TAG}_dig_old_$line.txt; exit 1; }
  if cmp -s gpurun_out/${TAG}_dig_new_$line.txt gpurun_out/${TAG}_dig_old_$line.txt; then echo "digest $line: identical"; else echo "digest $line: DIFFERENT"; cat gpurun_out/${TAG}_dig_new_$line.txt gpurun_out/${TAG}_dig_old_$line.txt; fi
done
run() {  # tag, precision, env...
  local tag=$1 prec=$2; shift 2
  env "$@" timeout -k 10 600 python -u tools/bench_train.py $prec --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/${TAG}_$tag.log 2>&1 || { tail -5 gpurun_out/${TAG}_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/${TAG}_$tag.log)"
}
for r in 1 2; do
  run bf_new_$r "--precision bf16" WC_X=1 || exit 1
  run bf_old_$r "--precision bf16" WC_KERNEL_LIB_BF16=$L/altbf/libwc_kernels.so WC_ALLOW_STALE_LIB=1 || exit 1
done
for r in 1 2; do
  run f3_new_$r "" WC_X=1 || exit 1
  run f3_old_$r "" WC_KERNEL_LIB=$L/alt/libwc_kernels.so WC_ALLOW_STALE_LIB=1 || exit 1
done
for v in new old; do
  if [ $v = old ]; then export WC_KERNEL_LIB_BF16=$L/altbf/libwc_kernels.so WC_ALLOW_STALE_LIB=1; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$v -o run -- python -u tools/bench_train.py --precision bf16 --steps 2 --warmup 1 --no-roofline --no-cpu-baseline > gpurun_out/${TAG}_prof_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$v.log; exit 1; }
done
echo done
