#!/bin/bash
# conv_in probe (graph vs isolated gap) + rocprofv3 kernel trace of the fp32-class training iteration.
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/conv_in_probe.py > gpurun_out/r04f/conv_in.log 2>&1
rc=$?; echo probe_rc=$rc; cat gpurun_out/r04f/conv_in.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f/train_prof -o run -- python3 -u tools/bench_train.py --steps 3 --warmup 2 > gpurun_out/r04f/train_prof.log 2>&1
rc=$?; echo prof_rc=$rc
python3 tools/prof_summary.py gpurun_out/r04f/train_prof > gpurun_out/r04f/train_prof_summary.txt 2>&1
head -45 gpurun_out/r04f/train_prof_summary.txt | cut -c1-150
exit $rc
