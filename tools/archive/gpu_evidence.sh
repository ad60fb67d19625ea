#!/bin/bash
# Round evidence: GPU tests, full T=1000 bench (roofline + cpu baseline), rocprofv3 kernel stats of
# a short bench, two-pass PMC HBM traffic.  Outputs under gpurun_out/ (copy into profiles/<tag>_*).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric gpurun_out/bench_full.log | cut -c1-300
if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_full.log; exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
rc=$?; echo prof_rc=$rc; grep metric gpurun_out/bench_prof.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/pmc_traffic.sh > gpurun_out/traffic.log 2>&1
rc=$?; echo traffic_rc=$rc; head -5 gpurun_out/traffic.log
exit $rc
