#!/bin/bash
# GPU call: tests, bench (roofline + cpu baseline), rocprofv3 kernel-trace stats.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 30 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo bench_rc=$rc; tail -2 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
rc=$?; echo prof_rc=$rc; tail -1 gpurun_out/bench_prof.log
find gpurun_out/prof -name "*.csv" | head
