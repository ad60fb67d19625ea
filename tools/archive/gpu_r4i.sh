#!/bin/bash
# Training: the GPU training tests, then a rocprofv3 kernel trace of the fp32-class iteration -> per-kernel table.
mkdir -p gpurun_out/r04i
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r04i/train_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/r04i/train_tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAIL" gpurun_out/r04i/train_tests.log | head; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i/train_prof -o run -- python3 -u tools/bench_train.py --steps 3 --warmup 2 > gpurun_out/r04i/train_prof.log 2>&1
rc=$?; echo prof_rc=$rc; [ $rc -ne 0 ] && exit $rc
python3 tools/prof_summary.py gpurun_out/r04i/train_prof > gpurun_out/r04i/train_prof_summary.txt 2>&1
head -30 gpurun_out/r04i/train_prof_summary.txt | cut -c1-150
