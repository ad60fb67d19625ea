#!/bin/bash
# Same-box A/B of the Winograd conv launches of one 256-px forward (tools/wino_shapes.py): the arms in
# $VARS, alternating, $REPS rounds; each arm is LIB[+VAR=VALUE...], LIB = tree (this tree's library) or
# the name of a variant library under weatherconverter_amd/lib/ (tools/build_alt.sh), e.g.
#   VARS="tree tree+WC_WINO_ONEWAVE=1 var_head" bash tools/wino_ab.sh
# Prints each run's total over the 40 launches (the per-launch lines stay in gpurun_out/).
mkdir -p gpurun_out
TAG=${TAG:-wab}
SCRIPT=${SCRIPT:-tools/wino_shapes.py}
for r in $(seq 1 ${REPS:-2}); do
  for arm in ${VARS:-tree}; do
    lib=${arm%%+*}
    envs=""
    [ "$arm" != "$lib" ] && envs=$(echo "${arm#*+}" | tr '+' ' ')
    if [ "$lib" != tree ]; then
      envs="$envs WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$lib/libwc_kernels.so WC_ALLOW_STALE_LIB=1"
    fi
    out=gpurun_out/${TAG}_$(echo "$arm" | tr '+=/' '___')_$r.txt
    env $envs timeout -k 10 300 python3 -u $SCRIPT > $out 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$arm rc=$rc"; tail -5 $out; exit $rc; }
    echo "$arm $r: $(tail -1 $out)"
  done
done
