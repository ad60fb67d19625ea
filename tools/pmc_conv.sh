#!/bin/bash
# PMC counters of one conv micro-bench case (two separate --pmc passes, kernel-trace/stats only).
# usage: bash tools/pmc_conv.sh [case_index] [mode: fp32|x6]
CASE=${1:-0}; MODE=${2:-x6}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmc1 -o p -- python3 tools/bench_conv.py --only $CASE --modes $MODE > gpurun_out/pmc1.log 2>&1; rc=$?; echo rc1=$rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc2 -o p -- python3 tools/bench_conv.py --only $CASE --modes $MODE > gpurun_out/pmc2.log 2>&1; rc=$?; echo rc2=$rc
tail -2 gpurun_out/pmc1.log gpurun_out/pmc2.log
exit $rc
