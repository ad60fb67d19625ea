#!/bin/bash
# Quick GPU check: GPU tests (optionally a -k filter as $1) + a short bench line.
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric gpurun_out/bench_quick.log | cut -c1-400
exit $rc
