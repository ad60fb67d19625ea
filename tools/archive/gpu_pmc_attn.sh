#!/bin/bash
# PMC passes for the f16x3 attention (d=128 N=4096 and d=32 N=4096).
export TMPDIR=/tmp
mkdir -p gpurun_out
for CASE in 0 3; do
  for PASS in 1 2; do
    if [ $PASS = 1 ]; then C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"; else C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM"; fi
    timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_attn_c${CASE}_p${PASS} -o p -- python3 tools/bench_conv.py --attn-only $CASE > gpurun_out/pmc_attn_c${CASE}_p${PASS}.log 2>&1
    rc=$?; echo case=$CASE pass=$PASS rc=$rc
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
