#!/bin/bash
# Quick iteration call: micro-bench (with correctness spot checks), GPU tests, short bench.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_conv.py --check > gpurun_out/bench_conv.log 2>&1
rc=$?; echo bench_conv_rc=$rc; grep -v amdgpu.ids gpurun_out/bench_conv.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'img/s', d['value'], 'conv', d['roofline']['achieved'], d['roofline']['frac'])"
