#!/bin/bash
# Training after batching the pack bounds and pooling the zeroed bound rows: tests, then three iterations lines.
mkdir -p gpurun_out/r04l
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r04l/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/r04l/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r04l/tests.log | head -20; exit $rc; }
for r in 1 2; do
  timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/r04l/b$r.log 2>&1
  rc=$?; echo "rc=$rc $(tail -1 gpurun_out/r04l/b$r.log | cut -c1-230)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u tools/train_small_ops.py > gpurun_out/r04l/small_ops.log 2>&1
grep -v "amdgpu.ids\|Warning\|_warn_once" gpurun_out/r04l/small_ops.log | head -8
exit 0
