#!/bin/bash
# user weight gradients deferred into the text fc's backward launch (one launch + one reduce fewer):
# tests, bench, profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_aa 600 $T tests/test_user_step_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py tests/test_text_head_gpu.py tests/test_multirank_gpu.py
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_c2aa
rm -rf $O; mkdir -p $O
run prof_c2aa 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_aa.json > gpurun_out/breakdown_c2aa.txt 2>&1
head -32 gpurun_out/breakdown_c2aa.txt
