#!/bin/bash
# Training forward attention projections on the pre-split path (split once + wc_proj_f16x3) vs the fused
# GN-prologue implicit GEMM (WC_PROJ_PA=0): training-gradient tests, then same-box A/Bs of both lines.
# usage: TAG=x bash tools/r6_train_pa_ab.sh
export TMPDIR=/tmp
TAG=${TAG:-tpa}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_train.py \
  -k "unet_grads or deterministic or accumulate or train" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
run() {  # tag, precision, env...
  local tag=$1 prec=$2; shift 2
  env "$@" timeout -k 10 600 python -u tools/bench_train.py $prec --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > gpurun_out/${TAG}_$tag.log 2>&1 || { tail -5 gpurun_out/${TAG}_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/${TAG}_$tag.log)"
}
for r in 1 2; do
  run bf_new_$r "--precision bf16" WC_X=1 || exit 1
  run bf_old_$r "--precision bf16" WC_PROJ_PA=0 || exit 1
done
for r in 1 2; do
  run f3_new_$r "" WC_X=1 || exit 1
  run f3_old_$r "" WC_PROJ_PA=0 || exit 1
done
echo done
