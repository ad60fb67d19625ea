#!/bin/bash
# Training (config 3) iteration: GPU train tests, then the training-step bench with a same-box A/B of
# env switches (AB_ENV, default: this round's f16x3 wgrad and attention backward off) and an optional
# rocprofv3 kernel trace.
# usage: [AB_ENV='A=0 B=0'] [PROF=1] [TAG=x] bash tools/archive/gpu_r3_train2.sh
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-t}
AB_ENV=${AB_ENV:-WC_WGRAD3_F16X3=0 WC_ATTN_BWD_F16X3=0}
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -v -x --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 --profile > gpurun_out/${TAG}_b1.log 2>&1
rc=$?; echo b1_rc=$rc; tail -1 gpurun_out/${TAG}_b1.log | cut -c1-2500; [ $rc -ne 0 ] && exit $rc
env ${AB_ENV} timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/${TAG}_b0.log 2>&1
rc=$?; echo b0_rc=$rc; tail -1 gpurun_out/${TAG}_b0.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u tools/bench_train.py --steps 3 --warmup 2 > gpurun_out/${TAG}_prof.log 2>&1
  rc=$?; echo prof_rc=$rc
  python3 tools/prof_summary.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_prof_summary.txt 2>&1 || true
  head -40 gpurun_out/${TAG}_prof_summary.txt | cut -c1-160
  exit $rc
fi
exit 0
