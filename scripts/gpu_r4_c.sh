#!/bin/bash
# Step profile of the current tree (in-graph Adam, split-K seams, loss sum in score_ce):
# bench + kernel trace + per-step breakdown, compared against the round-4 base breakdown.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
run bench 300 python -u bench.py
O=$PWD/gpurun_out/prof_c2b
rm -rf $O; mkdir -p $O
run prof_c2b 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_b.json > gpurun_out/breakdown_c2b.txt 2>&1
python benchmarks/phase_breakdown.py "$f" --until sample_kernel --json gpurun_out/r4_cache_build_b.json > gpurun_out/cache_build_b.txt 2>&1
head -60 gpurun_out/breakdown_c2b.txt
head -12 gpurun_out/cache_build_b.txt
