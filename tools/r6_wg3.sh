#!/bin/bash
# wgrad3 alone: f16x3 vs the bf16 single-piece line at B=32, kernel trace, then PMC passes of the bf16 line
export TMPDIR=/tmp
O=gpurun_out/wg3; mkdir -p $O
for line in f16x3 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$line -o k -- python3 -u tools/wgrad3_probe.py --batch 32 --line $line > $O/kt_$line.log 2>&1 || { tail -5 $O/kt_$line.log; exit 1; }
  cat $O/kt_$line.log
done
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/bf16_$i -o p -- python3 tools/wgrad3_probe.py --batch 32 --line bf16 --only 1 > $O/bf16_$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "pass $i rc=$rc"; tail -3 $O/bf16_$i.log; exit $rc; }
done
python3 tools/pmc_table.py $O/bf16_1 $O/bf16_2 $O/bf16_3 > $O/bf16_table.txt 2>&1; cat $O/bf16_table.txt | head -60
