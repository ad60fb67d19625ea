#!/bin/bash
# rocprofv3 kernel stats of a short bench run (no full T=1000 run).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
rc=$?; echo prof_rc=$rc; grep metric gpurun_out/bench_prof.log | cut -c1-300
exit $rc
