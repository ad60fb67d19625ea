#!/bin/bash
# Full T=1000 bench (default args) + rocprofv3 kernel stats of a short run.
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric gpurun_out/bench_full.log | cut -c1-400
if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_full.log; exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
rc=$?; echo prof_rc=$rc; grep metric gpurun_out/bench_prof.log | cut -c1-300
