#!/bin/bash
# One-wave conv A/B: bitwise test vs the halo kernel, then bench with the one-wave form off / on.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_x6.py -k "onewave or conv3x3_f16x3" -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/w1_test.log 2>&1
rc=$?; echo test_rc=$rc; tail -8 gpurun_out/w1_test.log; [ $rc -ne 0 ] && exit $rc
for m in 0 -1 0 -1; do
  WC_CONV3_W1=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-roofline --no-parity --no-cpu-baseline > gpurun_out/w1_bench_$m.json 2> gpurun_out/w1_bench_$m.err
  rc=$?; echo "mode $m rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/w1_bench_$m.json'));print(d['ms_per_step'])")"; [ $rc -ne 0 ] && { tail -5 gpurun_out/w1_bench_$m.err; exit $rc; }
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-parity --no-cpu-baseline > gpurun_out/w1_bench_roof.json 2> gpurun_out/w1_bench_roof.err
rc=$?; echo roof_rc=$rc
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/w1_bench_roof.json'))
print(d['ms_per_step'])
for k,v in d['roofline']['mfma_kernels'].items():
    print(k[:70], v['launches'], v['ms'], v['tflops'], v['frac'])
PY
exit $rc
