#!/bin/bash
# fused user tail (pool + scores + CE + pool backward): tests, bench, profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_y 600 $T tests/test_user_step_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py
check t_y2 600 $T tests/test_no_library_kernels_gpu.py
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_c2y
rm -rf $O; mkdir -p $O
run prof_c2y 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_y.json > gpurun_out/breakdown_c2y.txt 2>&1
head -32 gpurun_out/breakdown_c2y.txt
