#!/bin/bash
# Final-tree verification (third pass, after the pack and attention-prep changes): the whole GPU suite,
# smoke(), a 20-step bench line with roofline and CPU baseline, the fp32-class / bf16 training lines,
# and a kernel trace of the training line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/r04x_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r04x_tests.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04x_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/r04x_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r04x_bench.json 2> gpurun_out/r04x_bench.err
rc=$?; echo bench_rc=$rc; cut -c1-200 gpurun_out/r04x_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/r04x_train.log 2>&1
rc=$?; echo train_rc=$rc; tail -1 gpurun_out/r04x_train.log | cut -c100-230; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 --precision bf16 > gpurun_out/r04x_train_bf16.log 2>&1
rc=$?; echo train_bf16_rc=$rc; tail -1 gpurun_out/r04x_train_bf16.log | cut -c100-230; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04x_trainprof -o run -- python3 tools/bench_train.py --steps 3 --warmup 1 > gpurun_out/r04x_trainprof.log 2>&1
rc=$?; echo trainprof_rc=$rc; exit $rc
