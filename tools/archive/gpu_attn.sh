#!/bin/bash
# attention iteration: micro-bench, GPU tests, short bench with per-kernel table.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_conv.py --modes f3,igf3 > gpurun_out/bench_attn.log 2>&1
rc=$?; echo bench_attn_rc=$rc; grep -E 'attn f16|aggregate' gpurun_out/bench_attn.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric gpurun_out/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'img/s', d['value'], 'conv', d['roofline']['achieved'], d['roofline']['frac'])
for k,v in d['roofline']['mfma_kernels'].items(): print(k, v)"
