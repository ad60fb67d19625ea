#!/bin/bash
# 8-wave pre-split: B=8 and B=4 unsplit, alt (4-wave) vs altall (8-wave wherever N % 256 == 0)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for B in 8 4 2; do
    for arm in alt altall; do
      e="WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$arm/libwc_kernels.so WC_ALLOW_STALE_LIB=1"
      env $e timeout -k 10 300 python -u bench.py --batch $B --split 1 --steps 60 --warmup 3 --no-cpu-baseline --no-roofline --no-parity > gpurun_out/vp8d_b${B}_${arm}_$r.log 2>&1 || { tail -3 gpurun_out/vp8d_b${B}_${arm}_$r.log; exit 1; }
      echo "B=$B split1 $arm $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vp8d_b${B}_${arm}_$r.log)"
    done
  done
done
