#!/bin/bash
# Sampling attention built without SLP vectorisation (lib/alt: tools/build_alt.sh WORK wc_attention6 with
# EXTRA=-fno-slp-vectorize: no packed-f32 VALU beside the MFMAs) vs the tree: bench A/B x3 and kernel
# stats of each arm; the bench's parity leg prints the golden rel-L2 of each.   usage: TAG=x bash tools/r6_attn_noslp_ab.sh
export TMPDIR=/tmp
TAG=${TAG:-nslp}
mkdir -p gpurun_out
TAG=${TAG}_b ARMS="tree alt" REPS=3 bash tools/ab_bench.sh || exit 1
for arm in tree alt; do
  if [ $arm != tree ]; then export WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$arm/libwc_kernels.so WC_ALLOW_STALE_LIB=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$arm -o run -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/${TAG}_prof_$arm.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$arm.log; exit 1; }
  grep -o '"rel_l2": [0-9.e-]*' gpurun_out/${TAG}_prof_$arm.log
done
echo done
