#!/bin/bash
# Pre-split projection GEMM forms: bitwise tests, per-shape probe (LDS-DMA 128 / 256 rows, 128 rows
# with B in registers), bench A/B of the B-in-registers form.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_x6.py -k "pa256 or presplit or igemm_f16x3" -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/pa_test.log 2>&1
rc=$?; echo test_rc=$rc; grep -E "passed|failed|FAILED|Error" gpurun_out/pa_test.log | tail -8; [ $rc -ne 0 ] && exit $rc
WC_PROJ_BM256=0 timeout -k 10 200 python -u tools/proj_probe.py > gpurun_out/pa_probe128.log 2>&1 || exit 1
WC_PROJ_BM256=0 WC_PROJ_WR=2 timeout -k 10 200 python -u tools/proj_probe.py > gpurun_out/pa_probewr.log 2>&1 || exit 1
paste -d'#' <(grep -E "^(out|qkv|plain)" gpurun_out/pa_probe128.log | cut -c1-60) <(grep -E "^(out|qkv|plain)" gpurun_out/pa_probewr.log | cut -c28-60)
for m in 0 2 0 2; do
  WC_PROJ_WR=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/pa_bench_$m.json 2> gpurun_out/pa_bench_$m.err
  rc=$?; echo "wr $m rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/pa_bench_$m.json'));print(d['ms_per_step'])")"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pa_bench_$m.err; exit $rc; }
done
exit 0
