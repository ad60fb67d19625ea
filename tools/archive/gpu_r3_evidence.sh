#!/bin/bash
# Round 3 evidence: quick GPU tests, bench line (20 steps, all legs), rocprofv3 trace of the timed
# graph replays -> per-step table + reconciliation with the bench's per-kernel table, PMC traffic.
# usage: TAG=r03a bash tools/archive/gpu_r3_evidence.sh
TAG=${TAG:-r03x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_x6.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps ${STEPS:-20} --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo bench_rc=$rc; cut -c1-300 gpurun_out/${TAG}_bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -ne 0 ] && { tail -20 gpurun_out/${TAG}_prof.log; exit $rc; }
python3 tools/step_table.py gpurun_out/${TAG}_prof 20 --json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_step_table.txt 2>&1
python3 tools/reconcile.py gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_reconcile.txt 2>&1
tail -3 gpurun_out/${TAG}_step_table.txt; tail -4 gpurun_out/${TAG}_reconcile.txt
if [ "${TRAFFIC:-1}" = "1" ]; then
  bash tools/pmc_traffic.sh > gpurun_out/${TAG}_traffic.log 2>&1
  rc=$?; echo traffic_rc=$rc; head -5 gpurun_out/${TAG}_traffic.log
  python3 tools/traffic_summary.py gpurun_out/traffic_FETCH_SIZE gpurun_out/traffic_WRITE_SIZE ${TAG} > /dev/null 2>&1
fi
exit 0
