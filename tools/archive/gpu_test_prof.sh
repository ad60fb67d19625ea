#!/bin/bash
# GPU tests, then rocprofv3 kernel stats of a short bench (per-forward kernel table).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
rc=$?; echo prof_rc=$rc; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_prof.log
python3 tools/prof_table.py gpurun_out/prof/run_kernel_stats.csv | head -24
exit $rc
