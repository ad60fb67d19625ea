#!/bin/bash
# wgrad3 G-prefetch depth A/B on the bf16 line: HEAD (1 step), tree (2), altbf4 (4); probe and training
export TMPDIR=/tmp
O=gpurun_out/wg3ab; mkdir -p $O
for r in 1 2; do
  for v in tree altbf altbf4; do
    e=""; [ $v != tree ] && e="WC_KERNEL_LIB_BF16=$PWD/weatherconverter_amd/lib/$v/libwc_kernels.so WC_ALLOW_STALE_LIB=1"
    env $e timeout -k 10 300 python3 -u tools/wgrad3_probe.py --batch 32 --line bf16 > $O/p_${v}_$r.log 2>&1 || { tail -5 $O/p_${v}_$r.log; exit 1; }
    echo "== $v $r"; cat $O/p_${v}_$r.log
  done
done
for r in 1 2; do
  for v in tree altbf altbf4; do
    e=""; [ $v != tree ] && e="WC_KERNEL_LIB_BF16=$PWD/weatherconverter_amd/lib/$v/libwc_kernels.so WC_ALLOW_STALE_LIB=1"
    env $e timeout -k 10 600 python -u tools/bench_train.py --precision bf16 --steps 8 --warmup 3 --no-roofline --no-cpu-baseline > $O/t_${v}_$r.log 2>&1 || { tail -5 $O/t_${v}_$r.log; exit 1; }
    echo "train $v $r: $(grep -o '"ms_per_iter": [0-9.]*' $O/t_${v}_$r.log)"
  done
done
