#!/bin/bash
# Round-6 evidence of one tree on one box, part A (sampling): PMC HBM traffic per kernel (two --pmc
# passes), the full T=1000 bench line (driver command), the rocprofv3 step tables of 20 graph-replayed
# steps for the default two-group graph and for --split 1 (the isolated launches the roofline times),
# the reconcile of the latter against the bench's in-graph table, the GPU suite and smoke().
# usage: TAG=r06z bash tools/r6_evidence.sh   (outputs in gpurun_out/, summaries to copy into profiles/)
TAG=${TAG:-r06z}
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${TAG}_traffic_$c -o p -- python3 -u bench.py --steps 2 --warmup 1 --graph 0 --batch 8 --vp-wide 1 --no-roofline --no-cpu-baseline --no-parity > gpurun_out/${TAG}_traffic_$c.log 2>&1 || { echo "pmc $c failed"; tail -3 gpurun_out/${TAG}_traffic_$c.log; exit 1; }
done
python3 tools/traffic_summary.py gpurun_out/${TAG}_traffic_FETCH_SIZE gpurun_out/${TAG}_traffic_WRITE_SIZE $TAG > gpurun_out/${TAG}_traffic.txt 2>&1 || exit 1
cp profiles/${TAG}_hbm_traffic.json gpurun_out/
head -4 gpurun_out/${TAG}_traffic.txt | cut -c1-150
timeout -k 10 900 python3 -u bench.py > gpurun_out/${TAG}_bench_full_T1000.json 2> gpurun_out/${TAG}_bench_full.err; rc=$?; echo bench_rc=$rc; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_bench_full.err; exit $rc; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench_full_T1000.json | head -1
TAG=$TAG bash tools/steptable.sh > gpurun_out/${TAG}_steptable_run.log 2>&1 || { tail -5 gpurun_out/${TAG}_steptable_run.log; exit 1; }
tail -3 gpurun_out/${TAG}_steptable_run.log
export WC_GRAPH_SPLIT=1
TAG=${TAG}s1 bash tools/steptable.sh > gpurun_out/${TAG}s1_steptable_run.log 2>&1 || { tail -5 gpurun_out/${TAG}s1_steptable_run.log; exit 1; }
unset WC_GRAPH_SPLIT
tail -3 gpurun_out/${TAG}s1_steptable_run.log
python3 tools/reconcile.py gpurun_out/${TAG}s1_prof.log gpurun_out/${TAG}s1_step_table.json > gpurun_out/${TAG}_reconcile.txt 2>&1; tail -2 gpurun_out/${TAG}_reconcile.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
