#!/bin/bash
# Env-toggled conv variants after the static-vmcnt fix: tests under WR16 / LA2=1r, then bench
# default / WC_CONV3_WR16=1 / WC_CONV3_LA2=1 / =1r interleaved.
mkdir -p gpurun_out
WC_CONV3_WR16=1 WC_CONV3_LA2=1r timeout -k 10 500 python -u -m pytest tests/test_x6.py tests/test_gpu_unet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/w16_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -1 gpurun_out/w16_test.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAIL" gpurun_out/w16_test.log | head -20; exit $rc; fi
for r in 1 2; do
  for v in base WC_CONV3_WR16=1 WC_CONV3_LA2=1 WC_CONV3_LA2=1r; do
    if [ $v = base ]; then e=""; else e=$v; fi
    env $e timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/w16_$r.log 2>&1 || exit 1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/w16_$r.log)"
  done
done
