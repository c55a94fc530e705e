#!/bin/bash
# Config-5 step breakdown (kernel trace) of the current tree.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
O=$PWD/gpurun_out/prof_c5
rm -rf $O; mkdir -p $O
run prof_c5 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c5 -- python -u bench.py --config 5 --steps 6 --warmup 3 --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 4 --json gpurun_out/r5_c5_breakdown.json > gpurun_out/breakdown_c5.txt 2>&1
head -45 gpurun_out/breakdown_c5.txt
