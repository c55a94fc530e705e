#!/bin/bash
# the step graph's input launch also casts the step's weights (no in-graph cast launch):
# tests, bench, profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_ab 600 $T tests/test_kernels_gpu.py::test_copy_cast tests/test_kernels_gpu.py::test_multi_cast tests/test_user_step_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py tests/test_multirank_gpu.py tests/test_no_library_kernels_gpu.py
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_c2ab
rm -rf $O; mkdir -p $O
run prof_c2ab 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_ab.json > gpurun_out/breakdown_c2ab.txt 2>&1
head -32 gpurun_out/breakdown_c2ab.txt
