#!/bin/bash
# Round-2 evidence: full T=1000 bench (roofline + parity + cpu baseline), rocprofv3 kernel stats of a
# short bench, two-pass PMC HBM traffic, configs 1/4 line, training-step line.
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric gpurun_out/bench_full.log | cut -c1-200
if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_full.log; exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_prof.log 2>&1
rc=$?; echo prof_rc=$rc
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/pmc_traffic.sh > gpurun_out/traffic.log 2>&1
rc=$?; echo traffic_rc=$rc; head -3 gpurun_out/traffic.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/bench_configs.py --configs 1,4 > gpurun_out/configs.log 2>&1
rc=$?; echo configs_rc=$rc; grep config gpurun_out/configs.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/bench_train.py --steps 5 --warmup 2 --profile > gpurun_out/bench_train.log 2>&1
rc=$?; echo train_rc=$rc; tail -1 gpurun_out/bench_train.log | cut -c1-300
exit $rc
