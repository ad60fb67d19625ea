#!/bin/bash
# HBM traffic per kernel launch (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE in two separate
# --pmc passes over a short eager bench run (no HIP graph; 8 images with --vp-wide 1: the launches of one
# image group of the default two-group graph, same instantiations and per-launch sizes as bench.py's
# roofline), summarised by tools/traffic_summary.py.
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/traffic_$c -o p -- python3 -u bench.py --steps 2 --warmup 1 --graph 0 --batch 8 --vp-wide 1 --no-roofline --no-cpu-baseline > gpurun_out/traffic_$c.log 2>&1 || exit 1
done
python3 tools/traffic_summary.py gpurun_out/traffic_FETCH_SIZE gpurun_out/traffic_WRITE_SIZE
