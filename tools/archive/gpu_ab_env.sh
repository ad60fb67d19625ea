#!/bin/bash
# Same-box A/B of an environment switch on the bench line: tools/archive/gpu_ab_env.sh VAR A B [reps]
# (alternating runs, 20 timed steps each; per-kernel table from the roofline leg).
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; R=${4:-2}
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/ab_${v}_$i.log 2>&1 || exit 1
    python - "$VAR=$v" gpurun_out/ab_${v}_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
r = d['roofline']
top = sorted(r['mfma_kernels'].items(), key=lambda kv: -kv[1]['ms'])[:6]
print(sys.argv[1], 'ms/step', d['ms_per_step'], '|', '; '.join(f"{k.split(' ')[0][:60]} {v['ms']}ms {v['tflops']}TF" for k, v in top))
PY
  done
done
