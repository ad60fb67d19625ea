#!/bin/bash
# round-6: single-plane pre-split for the single-piece builds -- tests, then same-box A/B of the bf16
# training line (this tree's library at WC_WINO_VP 4 / 2 / 1 against HEAD's wc_wino in lib/altbf)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_wino.py tests/test_gpu_train.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/r6vp1_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r6vp1_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/r6vp1_tests.txt | head -20; exit $rc; }
ALT=$PWD/weatherconverter_amd/lib/altbf/libwc_kernels.so
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 600 python -u tools/bench_train.py --precision bf16 --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/r6vp1_$tag.log 2>&1 || { tail -5 gpurun_out/r6vp1_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r6vp1_$tag.log)"
}
for r in 1 2; do
  run new4_$r WC_WINO_VP=4
  run old4_$r WC_WINO_VP=4 WC_KERNEL_LIB_BF16=$ALT WC_ALLOW_STALE_LIB=1
  run new2_$r WC_WINO_VP=2
  run new1_$r WC_WINO_VP=1
  run old2_$r WC_WINO_VP=2 WC_KERNEL_LIB_BF16=$ALT WC_ALLOW_STALE_LIB=1
done
