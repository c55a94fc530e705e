#!/bin/bash
# user attention with two accumulator chains: tests, attention bench, bench, profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_x 600 $T tests/test_kernels_gpu.py -k "user_attention" tests/test_user_step_gpu.py
check t_x2 600 $T tests/test_step_graph.py tests/test_user_step_gpu.py
run uabench 200 python -u benchmarks/user_attn_bench.py
run bench 300 python -u bench.py
O=$PWD/gpurun_out/prof_c2x
rm -rf $O; mkdir -p $O
run prof_c2x 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_x.json > gpurun_out/breakdown_c2x.txt 2>&1
head -32 gpurun_out/breakdown_c2x.txt
