#!/bin/bash
# Same-box A/B of the Winograd conv: lib/alt (A) vs this tree (B): per-launch totals of one forward's
# Winograd convs (tools/wino_shapes.py) and a 30-step bench, alternating A B A B.
mkdir -p gpurun_out/abw
ALT=$PWD/weatherconverter_amd/lib/alt/libwc_kernels.so
for r in 1 2; do
  for v in a b; do
    if [ $v = a ]; then L="WC_KERNEL_LIB=$ALT"; else L="WC_X=1"; fi
    env $L timeout -k 10 200 python -u tools/wino_shapes.py > gpurun_out/abw/shapes_$v$r.log 2>&1
    rc=$?; echo "$v$r shapes rc=$rc $(tail -1 gpurun_out/abw/shapes_$v$r.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/abw/shapes_$v$r.log; exit $rc; }
    env $L timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-roofline --no-parity > gpurun_out/abw/bench_$v$r.log 2>&1
    rc=$?; echo "$v$r bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abw/bench_$v$r.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/abw/bench_$v$r.log; exit $rc; }
  done
done
