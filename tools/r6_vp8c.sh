#!/bin/bash
# 8-wave pre-split rule A/B: tree (<= 256 workgroups), alt (HEAD: 4-wave only), altall (8-wave wherever
# N % 256 == 0): the default line (split 2), B=1 and B=16 unsplit
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=vp8c REPS=2 ARMS="tree alt altall" bash tools/ab_bench.sh || exit 1
for r in 1 2; do
  for arm in tree alt altall; do
    e=""; [ $arm != tree ] && e="WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$arm/libwc_kernels.so WC_ALLOW_STALE_LIB=1"
    env $e timeout -k 10 300 python -u bench.py --batch 1 --steps 100 --warmup 3 --no-cpu-baseline --no-roofline --no-parity > gpurun_out/vp8c_b1_${arm}_$r.log 2>&1 || { tail -3 gpurun_out/vp8c_b1_${arm}_$r.log; exit 1; }
    echo "B=1 $arm $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vp8c_b1_${arm}_$r.log)"
    env $e timeout -k 10 300 python -u bench.py --split 1 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --no-parity > gpurun_out/vp8c_s1_${arm}_$r.log 2>&1 || { tail -3 gpurun_out/vp8c_s1_${arm}_$r.log; exit 1; }
    echo "B=16 split1 $arm $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vp8c_s1_${arm}_$r.log)"
  done
done
