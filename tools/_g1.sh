timeout -k 10 900 python3 -u tools/bench_train.py --precision bf16 --steps 10 --warmup 3 > gpurun_out/r05c_train_bf16.json 2> gpurun_out/r05c_train_bf16.err; rc=$?; echo bf16_rc=$rc; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05c_train_bf16.err; exit $rc; }
timeout -k 10 900 python3 -u tools/bench_train.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05c_train_f3.json 2> gpurun_out/r05c_train_f3.err; rc=$?; echo f3_rc=$rc; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05c_train_f3.err; exit $rc; }
python3 -c "
import json
for f in ('gpurun_out/r05c_train_bf16.json','gpurun_out/r05c_train_f3.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['roofline']
    print(f, d['ms_per_iter'], r['kernel'], r['achieved'], r['frac'], r['iteration'], (d['cpu_baseline'] or {}).get('value'))"
