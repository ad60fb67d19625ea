timeout -k 10 200 python -u -m pytest tests/test_wino.py -v -x --timeout 120 --timeout-method thread -k "pack_wino_device" > gpurun_out/pk.log 2>&1; tail -30 gpurun_out/pk.log
