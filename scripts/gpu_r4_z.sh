#!/bin/bash
# sampler writes cand | his side by side (no cat launch): tests, bench, profile.
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_z 600 $T tests/test_step_graph.py tests/test_engine_gpu.py tests/test_multirank_gpu.py tests/test_kernels_gpu.py
run bench 300 python -u bench.py
run bench50 300 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_c2z
rm -rf $O; mkdir -p $O
run prof_c2z 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r4_cfg2_step_breakdown_z.json > gpurun_out/breakdown_c2z.txt 2>&1
head -32 gpurun_out/breakdown_c2z.txt
