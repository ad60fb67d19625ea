#!/bin/bash
# Same-box A/B of the Winograd conv launches of one 256-px forward (tools/wino_shapes.py): the tree's
# library against the variant libraries named in $VARS (weatherconverter_amd/lib/<name>, built by
# tools/build_alt.sh), alternating, $REPS rounds.  Prints each run's total over the 40 launches.
mkdir -p gpurun_out
TAG=${TAG:-wab}
for r in $(seq 1 ${REPS:-2}); do
  for v in tree $VARS; do
    if [ "$v" = tree ]; then
      timeout -k 10 300 python3 -u tools/wino_shapes.py > gpurun_out/${TAG}_${v}_$r.txt 2>&1
    else
      WC_KERNEL_LIB=$PWD/weatherconverter_amd/lib/$v/libwc_kernels.so WC_ALLOW_STALE_LIB=1 timeout -k 10 300 python3 -u tools/wino_shapes.py > gpurun_out/${TAG}_${v}_$r.txt 2>&1
    fi
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 gpurun_out/${TAG}_${v}_$r.txt; exit $rc; }
    echo "$v $r: $(tail -1 gpurun_out/${TAG}_${v}_$r.txt)"
  done
done
