#!/bin/bash
# PMC of f16x3 3x3 conv micro-bench cases: SQ stall breakdown, MFMA busy, L1/L2 request traffic.
# usage: CASES="0 3 4" bash tools/archive/gpu_r3_pmc.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc3
for C in ${CASES:-0 3 4}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3/c${C}a -o p -- python3 tools/bench_conv.py --only $C --modes ${MODES:-f3} > gpurun_out/pmc3/c${C}a.log 2>&1
  rc=$?; echo case$C a rc=$rc; grep TF gpurun_out/pmc3/c${C}a.log; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d gpurun_out/pmc3/c${C}b -o p -- python3 tools/bench_conv.py --only $C --modes ${MODES:-f3} > gpurun_out/pmc3/c${C}b.log 2>&1
  rc=$?; echo case$C b rc=$rc; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/pmc3/c${C}c -o p -- python3 tools/bench_conv.py --only $C --modes ${MODES:-f3} > gpurun_out/pmc3/c${C}c.log 2>&1
  rc=$?; echo case$C c rc=$rc; [ $rc -ne 0 ] && exit $rc
done
for C in ${CASES:-0 3 4}; do
  echo "== case $C" >> gpurun_out/pmc3/table.txt
  python3 tools/pmc_table.py gpurun_out/pmc3/c${C}a gpurun_out/pmc3/c${C}b gpurun_out/pmc3/c${C}c >> gpurun_out/pmc3/table.txt 2>&1
done
cat gpurun_out/pmc3/table.txt
exit 0
