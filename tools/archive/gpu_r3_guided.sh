#!/bin/bash
# Config 4 at length: complete N=500 guided translations (tools/bench_guided.py), MIOpen find on/off.
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_guided.py --miopen-benchmark 1 > gpurun_out/guided_b1.log 2>&1
rc=$?; echo b1_rc=$rc; grep '^{' gpurun_out/guided_b1.log | cut -c1-400; grep -c IsEnoughWorkspace gpurun_out/guided_b1.log
[ $rc -ne 0 ] && { tail -20 gpurun_out/guided_b1.log; exit $rc; }
timeout -k 10 300 python -u tools/bench_guided.py --miopen-benchmark 0 --modes applied --lcg-steps 0 > gpurun_out/guided_b0.log 2>&1
rc=$?; echo b0_rc=$rc; grep '^{' gpurun_out/guided_b0.log | cut -c1-400; grep -c IsEnoughWorkspace gpurun_out/guided_b0.log
exit $rc
