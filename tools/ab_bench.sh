#!/bin/bash
# Same-box A/B of the 60-step bench line over library arms, alternating, $REPS rounds:
# ARMS="tree alt alt512" (tree = this tree's library, else weatherconverter_amd/lib/<name>/).
mkdir -p gpurun_out
TAG=${TAG:-abb}
for r in $(seq 1 ${REPS:-2}); do
  for arm in ${ARMS:-tree alt}; do
    e=""; [ $arm != tree ] && e="WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$arm/libwc_kernels.so WC_ALLOW_STALE_LIB=1"
    env $e timeout -k 10 300 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/${TAG}_${arm}_$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$arm rc=$rc"; tail -5 gpurun_out/${TAG}_${arm}_$r.log; exit $rc; }
    echo "$arm $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_${arm}_$r.log)"
  done
done
