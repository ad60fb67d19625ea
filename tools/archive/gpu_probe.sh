#!/bin/bash
# Conv A/B on one box: the epilogue/residual probe and the f16x3 conv table with the default
# library (B = this tree) and with the build in weatherconverter_amd/lib/alt (A, WC_KERNEL_LIB),
# then the conv / UNet GPU tests on the default library.
mkdir -p gpurun_out
ALT="WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/alt/libwc_kernels.so"
env $ALT timeout -k 10 200 python -u tools/probes/conv_epi_probe.py > gpurun_out/probe_a.log 2>&1
rc=$?; echo probe_a_rc=$rc; grep -v amdgpu.ids gpurun_out/probe_a.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/probes/conv_epi_probe.py > gpurun_out/probe_b.log 2>&1
rc=$?; echo probe_b_rc=$rc; grep -v amdgpu.ids gpurun_out/probe_b.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/bench_conv.py --check --modes f3,x6 --no-misc > gpurun_out/ab_b.log 2>&1
rc=$?; echo b_rc=$rc; grep -v amdgpu.ids gpurun_out/ab_b.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/pytest_gpu.log
exit $rc
