#!/bin/bash
# PMC HBM traffic of one image group (8 images, the graph's forms), then the full T=1000 bench line that
# reads it.  usage: TAG=r06d bash tools/r6_pmc_bench.sh
TAG=${TAG:-r06z}
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${TAG}_traffic_$c -o p -- python3 -u bench.py --steps 2 --warmup 1 --graph 0 --batch 8 --vp-wide 1 --no-roofline --no-cpu-baseline --no-parity > gpurun_out/${TAG}_traffic_$c.log 2>&1 || { echo "pmc $c failed"; tail -3 gpurun_out/${TAG}_traffic_$c.log; exit 1; }
done
python3 tools/traffic_summary.py gpurun_out/${TAG}_traffic_FETCH_SIZE gpurun_out/${TAG}_traffic_WRITE_SIZE $TAG > gpurun_out/${TAG}_traffic.txt 2>&1 || exit 1
cp profiles/${TAG}_hbm_traffic.json gpurun_out/
head -5 gpurun_out/${TAG}_traffic.txt | cut -c1-150
timeout -k 10 900 python3 -u bench.py > gpurun_out/${TAG}_bench_full_T1000.json 2> gpurun_out/${TAG}_bench_full.err; rc=$?; echo bench_rc=$rc; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_bench_full.err; exit $rc; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench_full_T1000.json | head -1
