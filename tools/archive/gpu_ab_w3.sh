#!/bin/bash
# Same-box A/B of the 3x3 weight gradient: lib/alt (A) vs this tree (B), tools/wgrad3_probe.py, A B A B.
mkdir -p gpurun_out/abw3
ALT=$PWD/weatherconverter_amd/lib/alt/libwc_kernels.so
for r in 1 2; do
  for v in a b; do
    if [ $v = a ]; then L="WC_KERNEL_LIB=$ALT"; else L="WC_X=1"; fi
    env $L timeout -k 10 200 python -u tools/wgrad3_probe.py > gpurun_out/abw3/$v$r.log 2>&1
    rc=$?; echo "$v$r rc=$rc"; grep wgrad3 gpurun_out/abw3/$v$r.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/abw3/$v$r.log; exit $rc; }
  done
done
exit 0
