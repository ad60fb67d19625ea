#!/bin/bash
# wgrad3 alone: timing over the ResBlock shapes, then three PMC passes on shape 0.
export TMPDIR=/tmp
O=gpurun_out/w3
mkdir -p $O
timeout -k 10 200 python3 -u tools/wgrad3_probe.py > $O/time.log 2>&1
rc=$?; cat $O/time.log; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/a -o p -- python3 tools/wgrad3_probe.py --only 0 > $O/a.log 2>&1
rc=$?; echo a rc=$rc; [ $rc -ne 0 ] && { tail -5 $O/a.log; exit $rc; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum --output-format csv -d $O/b -o p -- python3 tools/wgrad3_probe.py --only 0 > $O/b.log 2>&1
rc=$?; echo b rc=$rc; [ $rc -ne 0 ] && { tail -5 $O/b.log; exit $rc; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum --output-format csv -d $O/c -o p -- python3 tools/wgrad3_probe.py --only 0 > $O/c.log 2>&1
rc=$?; echo c rc=$rc; [ $rc -ne 0 ] && { tail -5 $O/c.log; exit $rc; }
python3 tools/pmc_table.py $O/a $O/b $O/c > $O/table.txt 2>&1
cat $O/table.txt
exit 0
