#!/bin/bash
# PMC passes (each its own run, kernel-trace only) over one pre-split attention shape (tools/attn_one.py),
# for the tree's library and the variant arms in $VARS (LIB[+VAR=VALUE...], as tools/wino_ab.sh).
# usage: SHAPE="4096 512 4 16" bash tools/pmc_attn.sh ; tables in gpurun_out/pmca_<arm>_table.txt
export TMPDIR=/tmp
SHAPE=${SHAPE:-4096 512 4 16}
O=gpurun_out/pmca
mkdir -p $O
for arm in tree $VARS; do
  lib=${arm%%+*}; e=""
  [ "$arm" != "$lib" ] && e=$(echo "${arm#*+}" | tr '+' ' ')
  [ "$lib" != tree ] && e="$e WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$lib/libwc_kernels.so WC_ALLOW_STALE_LIB=1"
  arm=$(echo "$arm" | tr '+=' '__')
  i=0
  for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum"; do
    i=$((i+1))
    env $e timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/${arm}_$i -o p -- python3 tools/attn_one.py $SHAPE > $O/${arm}_$i.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$arm pass $i rc=$rc"; tail -3 $O/${arm}_$i.log; exit $rc; }
  done
  python3 tools/pmc_table.py $O/${arm}_1 $O/${arm}_2 $O/${arm}_3 > $O/${arm}_table.txt 2>&1
  echo "== $arm ($SHAPE)"; cat $O/${arm}_table.txt
done
