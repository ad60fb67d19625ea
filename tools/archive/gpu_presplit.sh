#!/bin/bash
# pre-split attention: its bit-identity test first, then the GPU suite and a short bench (A/B vs WC_ATTN_PRESPLIT=0).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_x6.py -m gpu -q -x -k presplit --timeout 120 --timeout-method thread > gpurun_out/pytest_presplit.log 2>&1
rc=$?; echo presplit_rc=$rc; tail -15 gpurun_out/pytest_presplit.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for PS in 1 0; do
WC_ATTN_PRESPLIT=$PS timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ps$PS.log 2>&1
rc=$?; echo bench_ps${PS}_rc=$rc; grep metric gpurun_out/bench_ps$PS.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'img/s', d['value'])
for k,v in d['roofline']['mfma_kernels'].items():
    if 'attention' in k or 'igemm' in k: print(k, v)"
[ $rc -ne 0 ] && exit $rc
done
exit 0
