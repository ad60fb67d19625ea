# round-5 tree check: the GPU suite, smoke, a 20-step bench line, split-2 A/B
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/r05b_tests.log; grep "^FAILED" gpurun_out/r05b_tests.log | head
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b_smoke.log 2>&1; echo smoke_rc=$?; tail -1 gpurun_out/r05b_smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err; echo bench_rc=$?; python3 -c "
import json; d=json.loads(open('gpurun_out/r05b_bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['ms_per_step'], r['kernel'], r['frac'], r.get('mfma_pipe'), d['cpu_baseline']['value'])"
for r in 1 2; do for sp in 1 2; do timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --split $sp --no-cpu-baseline --no-roofline --no-parity > gpurun_out/r05b_split${sp}_$r.json 2>/dev/null; echo "split $sp rep $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05b_split${sp}_$r.json)"; done; done
