#!/bin/bash
# Winograd one-wave (MB=4, 16-row) form: bit-identity tests, per-shape A/B against the two-wave form, bench A/B.
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wino.py -q -x --timeout 120 --timeout-method thread > $O/wino_tests.log 2>&1
rc=$?; echo test_rc=$rc; tail -2 $O/wino_tests.log; [ $rc -ne 0 ] && { grep -E "Error|error|assert" $O/wino_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/bench_conv.py --modes wino --no-misc > $O/bench_conv_w2.log 2>&1
rc=$?; echo bench_rc=$rc; cat $O/bench_conv_w2.log; [ $rc -ne 0 ] && exit $rc
WC_WINO_ONEWAVE=1 timeout -k 10 300 python -u tools/bench_conv.py --modes wino --no-misc > $O/bench_conv_w1.log 2>&1
rc=$?; echo bench_rc=$rc; cat $O/bench_conv_w1.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > $O/bench20_w2.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric $O/bench20_w2.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
WC_WINO_ONEWAVE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > $O/bench20_w1.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric $O/bench20_w1.log | cut -c1-300
exit $rc
