export TMPDIR=/tmp
mkdir -p gpurun_out
for z in "" "--zeros"; do
  timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/clk$z -o p -- python3 tools/bench_conv.py --only 0 --modes x6,fp32 $z > gpurun_out/clk$z.log 2>&1 || exit 1
  grep 'conv3x3' gpurun_out/clk$z.log
done
