#!/bin/bash
# Round-3 evidence on the final tree: the whole GPU suite, smoke(), the full T=1000 bench (all legs),
# rocprofv3 trace of the timed replays -> step table + reconciliation, PMC traffic, training lines
# (fp32-class and the 16-bit line).
# usage: TAG=r03d bash tools/archive/gpu_r3_final.sh
TAG=${TAG:-r03d}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread --durations=15 > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/${TAG}_tests.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench_full.json 2> gpurun_out/${TAG}_bench_full.err
rc=$?; echo bench_rc=$rc; cut -c1-250 gpurun_out/${TAG}_bench_full.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_bench_full.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -ne 0 ] && exit $rc
python3 tools/step_table.py gpurun_out/${TAG}_prof 20 --json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_step_table.txt 2>&1
python3 tools/reconcile.py gpurun_out/${TAG}_bench_full.json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_reconcile.txt 2>&1
tail -1 gpurun_out/${TAG}_step_table.txt; tail -2 gpurun_out/${TAG}_reconcile.txt
bash tools/pmc_traffic.sh > gpurun_out/${TAG}_traffic.log 2>&1
rc=$?; echo traffic_rc=$rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 --profile > gpurun_out/${TAG}_train.log 2>&1
rc=$?; echo train_rc=$rc; tail -1 gpurun_out/${TAG}_train.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 --precision f16 > gpurun_out/${TAG}_train_f16.log 2>&1
rc=$?; echo train_f16_rc=$rc; tail -1 gpurun_out/${TAG}_train_f16.log | cut -c1-300
exit $rc
