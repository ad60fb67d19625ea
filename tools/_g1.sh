timeout -k 10 600 python -u -m pytest tests/test_wino.py -q -rf -x --timeout 120 --timeout-method thread -k "presplit or onewave" > gpurun_out/g17_tests.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed|Error" gpurun_out/g17_tests.log | tail -4
VARS="tree tree+WC_WINO_ONEWAVE=1" TAG=g17 REPS=2 bash tools/wino_ab.sh
