#!/bin/bash
# kernel-trace summary of the bf16 training line (3 timed iterations + 1 warm-up) on the current tree
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6trainprof -o p -- python3 -u tools/bench_train.py --precision bf16 --steps 3 --warmup 1 --no-roofline --no-cpu-baseline > gpurun_out/r6trainprof.log 2>&1 || { tail -5 gpurun_out/r6trainprof.log; exit 1; }
grep -o '"ms_per_iter": [0-9.]*' gpurun_out/r6trainprof.log

python3 tools/prof_summary.py gpurun_out/r6trainprof > gpurun_out/r6_train_bf16_kernel_summary.txt 2>&1; head -45 gpurun_out/r6_train_bf16_kernel_summary.txt | cut -c1-150
