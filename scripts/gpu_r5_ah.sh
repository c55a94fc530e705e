#!/bin/bash
# config-4 (LDP) step launch sequence on the current tree
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/prof_ah; rm -rf $O; mkdir -p $O
run prof_ah 200 rocprofv3 --kernel-trace --output-format csv -d $O -o ah -- python -u bench.py --config 4 --steps 10 --warmup 5 --round off --no-valid
python benchmarks/launch_seq.py $O/ah_kernel_trace.csv > gpurun_out/r5_cfg4_launch_seq.txt 2>&1
cat gpurun_out/r5_cfg4_launch_seq.txt
