#!/bin/bash
# Winograd conv: GPU tests + per-shape timing against the direct f16x3 halo kernel, then the model-level
# suites that now run through it (UNet goldens, training gradients).
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wino.py -v -x --timeout 120 --timeout-method thread > $O/wino_tests.log 2>&1
rc=$?; echo test_rc=$rc; tail -3 $O/wino_tests.log; [ $rc -ne 0 ] && { grep -E "Error|error|assert" $O/wino_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_conv.py --modes f3,wino --no-misc --check > $O/bench_conv.log 2>&1
rc=$?; echo bench_rc=$rc; cat $O/bench_conv.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_train.py -v -x --timeout 120 --timeout-method thread > $O/model_tests.log 2>&1
rc=$?; echo model_rc=$rc; tail -3 $O/model_tests.log; [ $rc -ne 0 ] && { grep -E "Error|error|assert" $O/model_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench20.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric $O/bench20.log | cut -c1-300
exit $rc
