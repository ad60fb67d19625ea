#!/bin/bash
# Round-5 evidence of one tree, on one box: PMC HBM traffic per kernel (two --pmc passes), the full
# T=1000 bench line (roofline + cpu_baseline + parity), the rocprofv3 step table of 20 graph-replayed
# steps reconciled against the bench's per-kernel table, and the two config-3 training lines.
# usage: TAG=r05z bash tools/r5_evidence.sh   (outputs in gpurun_out/, summaries to copy into profiles/)
TAG=${TAG:-r05z}
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${TAG}_traffic_$c -o p -- python3 -u bench.py --steps 2 --warmup 1 --graph 0 --no-roofline --no-cpu-baseline --no-parity > gpurun_out/${TAG}_traffic_$c.log 2>&1 || { echo "pmc $c failed"; tail -3 gpurun_out/${TAG}_traffic_$c.log; exit 1; }
done
python3 tools/traffic_summary.py gpurun_out/${TAG}_traffic_FETCH_SIZE gpurun_out/${TAG}_traffic_WRITE_SIZE $TAG > gpurun_out/${TAG}_traffic.txt 2>&1 || exit 1
cp profiles/${TAG}_hbm_traffic.json gpurun_out/
head -6 gpurun_out/${TAG}_traffic.txt
timeout -k 10 900 python3 -u bench.py > gpurun_out/${TAG}_bench_full_T1000.json 2> gpurun_out/${TAG}_bench_full.err; rc=$?; echo bench_rc=$rc; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_bench_full.err; exit $rc; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench_full_T1000.json
TAG=$TAG bash tools/steptable.sh || exit 1
python3 tools/reconcile.py gpurun_out/${TAG}_bench_full_T1000.json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_reconcile.txt 2>&1; tail -2 gpurun_out/${TAG}_reconcile.txt
timeout -k 10 900 python3 -u tools/bench_train.py --precision bf16 --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_train_bf16.json 2> gpurun_out/${TAG}_train_bf16.err || { tail -3 gpurun_out/${TAG}_train_bf16.err; exit 1; }
timeout -k 10 900 python3 -u tools/bench_train.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_train.json 2> gpurun_out/${TAG}_train.err || { tail -3 gpurun_out/${TAG}_train.err; exit 1; }
grep -o '"ms_per_iter": [0-9.]*' gpurun_out/${TAG}_bench_train_bf16.json gpurun_out/${TAG}_bench_train.json
