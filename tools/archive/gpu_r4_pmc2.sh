#!/bin/bash
# Side-by-side PMC of the direct f16x3 halo conv and the Winograd conv on one micro-bench case:
# issue / wait breakdown, VALU vs MFMA activity, TA / L1 / L2 load path.  usage: CASE=0 bash tools/archive/gpu_r4_pmc2.sh
export TMPDIR=/tmp
C=${CASE:-0}
O=gpurun_out/pmc4
mkdir -p $O
for M in f3 wino; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/${M}a -o p -- python3 tools/bench_conv.py --only $C --modes $M --no-misc > $O/${M}a.log 2>&1
  rc=$?; echo $M a rc=$rc; [ $rc -ne 0 ] && { tail -5 $O/${M}a.log; exit $rc; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum --output-format csv -d $O/${M}b -o p -- python3 tools/bench_conv.py --only $C --modes $M --no-misc > $O/${M}b.log 2>&1
  rc=$?; echo $M b rc=$rc; [ $rc -ne 0 ] && { tail -5 $O/${M}b.log; exit $rc; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum --output-format csv -d $O/${M}c -o p -- python3 tools/bench_conv.py --only $C --modes $M --no-misc > $O/${M}c.log 2>&1
  rc=$?; echo $M c rc=$rc; [ $rc -ne 0 ] && { tail -5 $O/${M}c.log; exit $rc; }
  python3 tools/pmc_table.py $O/${M}a $O/${M}b $O/${M}c > $O/${M}_table.txt 2>&1
  cat $O/${M}_table.txt
done
exit 0
