#!/bin/bash
# round-6 opening tree: driver-default bench + kernel-trace breakdown of config 2
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run r6base_c2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
O=$PWD/gpurun_out/prof_r6base; rm -rf $O; mkdir -p $O
run prof_r6base 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o ar -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
python benchmarks/launch_seq.py $O/ar_kernel_trace.csv > gpurun_out/r6_cfg2_launch_seq_base.txt 2>&1
python benchmarks/step_breakdown.py $O/ar_kernel_trace.csv --steps 10 --json gpurun_out/r6_cfg2_step_breakdown_base.json > gpurun_out/r6_breakdown_base.txt 2>&1
head -30 gpurun_out/r6_breakdown_base.txt
