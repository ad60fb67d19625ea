#!/bin/bash
# round-6: head conv with 32-channel chunks -- tests through it, the launch's time, then a same-box bench A/B
# against the 16-channel-chunk kernel (weatherconverter_amd/lib/alt, tools/build_alt.sh HEAD wc_misc)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_gpu_train.py -m gpu -x -q -rf --timeout 240 --timeout-method thread -k "head or unet or golden or grads" > gpurun_out/r6head_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/r6head_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/r6head_tests.txt | head; exit $rc; }
timeout -k 10 300 python -u tools/launch_shapes.py head > gpurun_out/r6head_tree.txt 2>&1 && grep head_conv gpurun_out/r6head_tree.txt
WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/alt/libwc_kernels.so WC_ALLOW_STALE_LIB=1 timeout -k 10 300 python -u tools/launch_shapes.py head > gpurun_out/r6head_alt.txt 2>&1 && grep head_conv gpurun_out/r6head_alt.txt
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r6head_fetch -o p -- python3 -u tools/launch_shapes.py head > gpurun_out/r6head_fetch.log 2>&1 || { tail -3 gpurun_out/r6head_fetch.log; exit 1; }
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob('gpurun_out/r6head_fetch/**/p_counter_collection.csv', recursive=True)[0])))
v = [float(r['Counter_Value']) * 1024 * 2 for r in rows if 'head_conv' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE']
print('head_conv FETCH_SIZE x2 per launch (MB):', [round(x / 1e6, 1) for x in v])
PY
bash tools/ab_lib.sh
