#!/bin/bash
# the selectable forms re-measured under the two-group graph (60-step bench line), alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--steps 60 --warmup 3 --no-cpu-baseline --no-roofline"
for r in 1 2; do
  for arm in ${ARMS:-default s2d0 ct0 proj128 proj256 presplit0}; do
    case $arm in
      default) cmd="python -u bench.py $B";;
      s2d0) cmd="env WC_DOWN_S2D=0 python -u bench.py $B";;
      ct0) cmd="env WC_UP_CT=0 python -u bench.py $B";;
      proj128) cmd="python -u tools/bench_with.py --proj-tile 128 -- $B";;
      proj256) cmd="python -u tools/bench_with.py --proj-tile 256 -- $B";;
      presplit0) cmd="env WC_ATTN_PRESPLIT=0 python -u bench.py $B";;
    esac
    timeout -k 10 300 $cmd > gpurun_out/forms_${arm}_$r.log 2>&1 || { echo "$arm failed"; tail -3 gpurun_out/forms_${arm}_$r.log; exit 1; }
    echo "$arm $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/forms_${arm}_$r.log)"
  done
done
