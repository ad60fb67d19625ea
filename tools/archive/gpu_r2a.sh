#!/bin/bash
# Round-2 checks: new GPU tests (distributed world-2, chunked batch, LCG, config-4 size) + full bench line.
mkdir -p gpurun_out
echo "nproc=$(nproc) affinity=$(python -c 'import os;print(len(os.sched_getaffinity(0)))') cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_guided_config4.py tests/test_gpu_unet.py -m gpu -v --timeout 300 --timeout-method thread -k "world2 or descriptor or lcg or config4 or batch16" > gpurun_out/pytest_r2a.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_r2a.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r2a.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric gpurun_out/bench_r2a.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d.get('parity'), d['cpu_baseline'])"
exit $rc
