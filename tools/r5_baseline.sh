#!/bin/bash
# Round-5 baseline on a fresh box: step table (rocprofv3 kernel trace of 20 graph-replayed steps) and
# the per-launch Winograd conv times of one forward.
mkdir -p gpurun_out
TAG=r05a bash tools/steptable.sh || exit 1
timeout -k 10 300 python3 -u tools/wino_shapes.py > gpurun_out/r05a_wino_shapes.txt 2>&1; rc=$?; echo wino_rc=$rc; tail -8 gpurun_out/r05a_wino_shapes.txt
exit $rc
