timeout -k 10 600 python -u -m pytest tests/test_wino.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g1_wino_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g1_wino_tests.log; [ $rc -ne 0 ] && exit $rc
VARS="var_head var_sgb0" TAG=g1 REPS=2 bash tools/wino_ab.sh
