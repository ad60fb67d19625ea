#!/bin/bash
# D = 192 attention backward on f16x3 (V rows in LDS): parity for DS 2 and 1, then training A/B
# (DS 2, DS 1, the fp32-MFMA dK / dV).
mkdir -p gpurun_out/r04h
for ds in 2 1; do
  WC_DKDV192_DS=$ds timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q -x -k "split_attention_lse or attention_backward" --timeout 120 --timeout-method thread > gpurun_out/r04h/t$ds.log 2>&1
  rc=$?; echo ds${ds}_test_rc=$rc; tail -2 gpurun_out/r04h/t$ds.log; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/r04h/t$ds.log | head; exit $rc; }
done
for cfg in "WC_DKDV192_DS=2" "WC_DKDV192_DS=1" "WC_ATTN_BWD192_FP32=1"; do
  env $cfg timeout -k 10 300 python -u tools/bench_train.py --steps 5 --warmup 2 --profile > gpurun_out/r04h/b.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; tail -1 gpurun_out/r04h/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_iter'], d['ms_backward'], {k: v['ms'] for k, v in d['kernel_classes'].items() if 'attn' in k})"; [ $rc -ne 0 ] && exit $rc
done
exit 0
