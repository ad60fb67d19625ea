timeout -k 10 600 python -u -m pytest tests/test_wino.py -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/g12_wino_tests.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed|Error" gpurun_out/g12_wino_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
VARS="tree tree+WC_WINO_VP=6 tree+WC_WINO_VP=4 tree+WC_WINO_VP=2" TAG=g12 REPS=2 bash tools/wino_ab.sh
