#!/bin/bash
# rocprofv3 kernel trace of 20 graph-replayed sampling steps -> step table (and the bench line).
# usage: TAG=x bash tools/steptable.sh
TAG=${TAG:-st}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-parity --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_prof.log; exit $rc; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_prof.log
python3 tools/step_table.py gpurun_out/${TAG}_prof 20 --json gpurun_out/${TAG}_step_table.json > gpurun_out/${TAG}_step_table.txt 2>&1
cut -c1-120 gpurun_out/${TAG}_step_table.txt
