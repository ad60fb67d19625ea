#!/bin/bash
# Round-6 evidence, part B: the two config-3 training lines (roofline + CPU baseline) and the config-4
# guided translation line (breakdown, roofline, CPU baseline).   usage: TAG=r06z bash tools/r6_evidence_b.sh
TAG=${TAG:-r06z}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/bench_train.py --precision bf16 --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_train_bf16.json 2> gpurun_out/${TAG}_train_bf16.err || { tail -3 gpurun_out/${TAG}_train_bf16.err; exit 1; }
timeout -k 10 900 python3 -u tools/bench_train.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_train.json 2> gpurun_out/${TAG}_train.err || { tail -3 gpurun_out/${TAG}_train.err; exit 1; }
grep -o '"ms_per_iter": [0-9.]*' gpurun_out/${TAG}_bench_train_bf16.json gpurun_out/${TAG}_bench_train.json
timeout -k 10 900 python3 -u tools/bench_guided.py > gpurun_out/${TAG}_guided.jsonl 2> gpurun_out/${TAG}_guided.err || { tail -5 gpurun_out/${TAG}_guided.err; exit 1; }
grep -o '"value": [0-9.]*, "unit": "[a-z/]*"' gpurun_out/${TAG}_guided.jsonl
