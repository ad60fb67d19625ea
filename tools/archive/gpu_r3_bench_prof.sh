#!/bin/bash
# Final-tree bench evidence without the test suite: smoke, the full T=1000 bench (all legs), rocprofv3
# trace of the timed graph replays -> step table + reconciliation.  usage: TAG=r03m bash tools/archive/gpu_r3_bench_prof.sh
TAG=${TAG:-r03x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench_full.json 2> gpurun_out/${TAG}_bench_full.err
rc=$?; echo bench_rc=$rc; cut -c1-250 gpurun_out/${TAG}_bench_full.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_bench_full.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -ne 0 ] && exit $rc
python3 tools/step_table.py gpurun_out/${TAG}_prof 20 --json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_step_table.txt 2>&1
python3 tools/reconcile.py gpurun_out/${TAG}_bench_full.json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_reconcile.txt 2>&1
tail -1 gpurun_out/${TAG}_step_table.txt; tail -1 gpurun_out/${TAG}_reconcile.txt
exit 0
