#!/bin/bash
# PMC of the f16x3 attention backward kernels (tools/attn_bwd_probe.py): stall breakdown, MFMA busy,
# LDS traffic and bank conflicts, one counter group per pass.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
timeout -k 10 120 python -u tools/attn_bwd_probe.py > gpurun_out/pmcab/time.log 2>&1
rc=$?; echo time_rc=$rc; tail -1 gpurun_out/pmcab/time.log; [ $rc -ne 0 ] && exit $rc
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmcab/p$i -o p -- python3 tools/attn_bwd_probe.py --reps 1 > gpurun_out/pmcab/p$i.log 2>&1
  rc=$?; echo pass$i rc=$rc; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_table.py gpurun_out/pmcab/p1 gpurun_out/pmcab/p2 > gpurun_out/pmcab/table.txt 2>&1
grep -A24 "attn_bwd6" gpurun_out/pmcab/table.txt | head -70
exit 0
