#!/bin/bash
# Round-4 first GPU pass: the RCCL (world size 1) tests, the MFMA waves-per-SIMD sweep (rates + a
# separate clock / MFMA-busy PMC pass), a 20-step bench, the whole GPU suite.
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_bench_dist.py -v --timeout 120 --timeout-method thread > $O/rccl.log 2>&1
rc=$?; echo rccl_rc=$rc; tail -3 $O/rccl.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 ./tools/probes/bin/mfma_peak > $O/mfma_sweep.jsonl 2> $O/mfma_sweep.err
rc=$?; echo sweep_rc=$rc; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/mfma_pmc -o p -- ./tools/probes/bin/mfma_peak > $O/mfma_pmc.log 2>&1
rc=$?; echo sweep_pmc_rc=$rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench20.log 2>&1
rc=$?; echo bench_rc=$rc; grep metric $O/bench20.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 $O/pytest_gpu.log
exit $rc
