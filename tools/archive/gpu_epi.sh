#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_conv.py --check --modes igf3,igx6 --no-misc > gpurun_out/epi_conv.log 2>&1
rc=$?; echo conv_rc=$rc; grep -E "relL2|aggregate" gpurun_out/epi_conv.log | grep -v amdgpu
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/conv_shape_probe.py > gpurun_out/epi_shape.log 2>&1
rc=$?; echo shape_rc=$rc; grep -v amdgpu gpurun_out/epi_shape.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo bench_rc=$rc; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log
exit $rc
