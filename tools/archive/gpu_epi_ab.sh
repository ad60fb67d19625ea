#!/bin/bash
# Epilogue changes: GPU suite on this tree, the out-projection probe on lib/alt (A) and this tree (B),
# then the same-box whole-bench A/B (tools/archive/gpu_ab_lib.sh).
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/alt/libwc_kernels.so timeout -k 10 200 python -u tools/probes/proj_epi_probe.py > gpurun_out/proj_a.log 2>&1
rc=$?; echo proj_a_rc=$rc; grep -v amdgpu.ids gpurun_out/proj_a.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/probes/proj_epi_probe.py > gpurun_out/proj_b.log 2>&1
rc=$?; echo proj_b_rc=$rc; grep -v amdgpu.ids gpurun_out/proj_b.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/archive/gpu_ab_lib.sh
