#!/bin/bash
# Projection implicit GEMM vs the halo conv: igf3 timings, then PMC passes on the out-projection
# shape (igf3 case 3: 1x1 512->512 at 64x64, raw input) and the halo 3x3 conv (f3 case 0).
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_conv.py --modes igf3 --no-misc > gpurun_out/igf3.log 2>&1
rc=$?; echo igf3_rc=$rc; grep -v amdgpu.ids gpurun_out/igf3.log
if [ $rc -ne 0 ]; then exit $rc; fi
MODES=igf3 bash tools/pmc_two.sh "3" && MODES=f3 bash tools/pmc_two.sh "0"
