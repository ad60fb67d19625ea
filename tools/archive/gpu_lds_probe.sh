#!/bin/bash
# LDS counters available + one pass on the dominant-shape f16x3 3x3 conv (bench_conv f3 case 0).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1; echo list_rc=$?
grep -o "SQ_[A-Z_]*LDS[A-Z_]*" gpurun_out/counters_avail.txt | sort -u > gpurun_out/lds_counters.txt
cat gpurun_out/lds_counters.txt
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/pmc_lds_f3c0 -o p -- python3 tools/bench_conv.py --only 0 --modes f3 --no-misc > gpurun_out/pmc_lds.log 2>&1
echo pmc_rc=$?
