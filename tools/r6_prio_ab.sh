#!/bin/bash
# Sampling bench A/B: this tree vs lib/alt and lib/alt2 (attention with static s_setprio for every other
# dispatched workgroup pair / quad, -DWC_ATT_PRIO=1 / 2), 3 rounds, then kernel stats of each arm.
export TMPDIR=/tmp
TAG=${TAG:-prio}
mkdir -p gpurun_out
TAG=${TAG}_b ARMS="tree alt alt2" REPS=3 bash tools/ab_bench.sh || exit 1
for arm in tree alt alt2; do
  if [ $arm != tree ]; then export WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$arm/libwc_kernels.so WC_ALLOW_STALE_LIB=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$arm -o run -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/${TAG}_prof_$arm.log 2>&1 || { tail -5 gpurun_out/${TAG}_prof_$arm.log; exit 1; }
done
echo done
