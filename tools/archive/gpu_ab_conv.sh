#!/bin/bash
# A/B of the f16x3 3x3 conv weight staging (registers 1 tap/step = default vs LDS-DMA 3 taps/step), with checks.
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_conv.py --check --modes f3 > gpurun_out/ab_default.log 2>&1
rc=$?; echo default_rc=$rc; grep -v amdgpu.ids gpurun_out/ab_default.log
if [ $rc -ne 0 ]; then exit $rc; fi
WC_CONV3_GL=1 timeout -k 10 200 python -u tools/bench_conv.py --modes f3 > gpurun_out/ab_gl1.log 2>&1
rc=$?; echo gl1_rc=$rc; grep -v amdgpu.ids gpurun_out/ab_gl1.log
exit $rc
