#!/bin/bash
# Round-6 check of one tree on one box: GPU suite, smoke(), default bench line (the driver's command).
# usage: TAG=r06a bash tools/r6_check.sh   (outputs in gpurun_out/)
TAG=${TAG:-r06z}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench.json
python3 - <<EOF
import json
d = json.loads(open("gpurun_out/${TAG}_bench.json").readline())
r = d["roofline"]
print(r["kernel"], r["frac"], r.get("mean_launch_ms"), r.get("mean_launch_ms_source"))
for k, v in sorted(r.get("mfma_kernels", {}).items(), key=lambda kv: -kv[1]["ms"])[:14]:
    print(f"  {k:60s} {v['ms']:.3f} ms  {v.get('frac')}")
for k, v in sorted(d.get("hbm_kernels", r.get("hbm_kernels", {})).items(), key=lambda kv: -kv[1].get("ms", 0))[:10]:
    print(f"  {k:60s} {v}")
EOF
