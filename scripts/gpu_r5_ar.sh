#!/bin/bash
# final tree: rocprofv3 --kernel-trace --stats of the config-2 bench (cache build + 20 steps)
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/prof_ar; rm -rf $O; mkdir -p $O
run prof_ar 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ar -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
python benchmarks/launch_seq.py $O/ar_kernel_trace.csv > gpurun_out/r5_cfg2_launch_seq_final.txt 2>&1
python benchmarks/step_breakdown.py $O/ar_kernel_trace.csv --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_final.json > gpurun_out/r5_breakdown_final.txt 2>&1
ls $O; head -30 gpurun_out/r5_breakdown_final.txt
