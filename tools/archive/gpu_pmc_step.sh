#!/bin/bash
# MFMA busy / LDS wait / bank conflicts / wave cycles per kernel of one eager UNet forward (256 px, B=16),
# one --pmc pass (7 SQ counters + GRBM_GUI_ACTIVE), summarised per kernel by tools/pmc_table.py.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_step -o p -- python3 -u bench.py --steps 1 --warmup 1 --graph 0 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/pmc_step.log 2>&1 || exit 1
python3 tools/pmc_table.py gpurun_out/pmc_step > gpurun_out/pmc_step.txt 2>&1
cat gpurun_out/pmc_step.txt
