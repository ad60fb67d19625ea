#!/bin/bash
# Raw-weight Winograd packs: bit-identity + training-gradient tests, then a same-box A/B of the training
# line (off = WC_PACK_RAW=0; on = default), off on off on.
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py \
    -k "pack_wino_raw or unet_grads or deterministic or accumulate" > gpurun_out/t4_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/t4_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/t4_tests.log | head -20; exit $rc; }
for r in 1 2; do
  for v in off on; do
    if [ $v = off ]; then L="WC_PACK_RAW=0"; else L="WC_X=1"; fi
    env $L timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/t4_$v$r.log 2>&1
    rc=$?; echo "$v$r rc=$rc $(grep -o '"ms_per_iter": [0-9.]*' gpurun_out/t4_$v$r.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/t4_$v$r.log; exit $rc; }
  done
done
exit 0
