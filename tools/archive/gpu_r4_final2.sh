#!/bin/bash
# Last check of the final tree: the whole GPU suite and smoke().
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r04y_tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -1 gpurun_out/r04y_tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r04y_tests.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04y_smoke.log 2>&1
rc=$?; echo smoke_rc=$rc; tail -1 gpurun_out/r04y_smoke.log; exit $rc
