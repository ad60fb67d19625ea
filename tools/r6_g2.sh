#!/bin/bash
# round-6 call 2: item-rotation A/B of the Winograd convs, then the config-4 guided line with its breakdown
export TMPDIR=/tmp
mkdir -p gpurun_out
VARS="tree rot128 rot64" TAG=r6rot REPS=2 bash tools/wino_ab.sh || exit 1
timeout -k 10 900 python3 -u tools/bench_guided.py > gpurun_out/r06_guided.jsonl 2> gpurun_out/r06_guided.err; rc=$?
echo guided_rc=$rc; [ $rc -ne 0 ] && { tail -8 gpurun_out/r06_guided.err; exit $rc; }
cut -c1-400 gpurun_out/r06_guided.jsonl
