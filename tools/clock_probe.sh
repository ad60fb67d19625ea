#!/bin/bash
# Clock / MFMA-busy of one conv micro-bench case: bash tools/clock_probe.sh <case> <modes>
CASE=${1:-0}; MODES=${2:-x6,f3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/clk -o p -- python3 tools/bench_conv.py --only $CASE --modes $MODES > gpurun_out/clk.log 2>&1 || exit 1
grep 'conv' gpurun_out/clk.log
