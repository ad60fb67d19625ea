#!/bin/bash
# Round 3: rocprofv3 kernel trace of the timed graph replays (no roofline / parity / CPU legs) ->
# per-step kernel table; per-launch-shape event table of one forward.
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${K:-20}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 -u bench.py --steps $K --warmup 3 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/prof3_bench.log 2>&1
rc=$?; echo prof_rc=$rc; grep metric gpurun_out/prof3_bench.log | cut -c1-250
if [ $rc -ne 0 ]; then tail -20 gpurun_out/prof3_bench.log; exit $rc; fi
python3 tools/step_table.py gpurun_out/prof3 $K --json gpurun_out/step_table.json > gpurun_out/step_table.txt 2>&1
rc=$?; cat gpurun_out/step_table.txt | cut -c1-160 | head -50
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u tools/prof_shapes.py > gpurun_out/prof_shapes.txt 2>&1
rc=$?; echo shapes_rc=$rc; cat gpurun_out/prof_shapes.txt | cut -c1-200 | head -60
exit $rc
