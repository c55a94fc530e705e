#!/bin/bash
# weight gradients on a side stream: focused tests, A/B/A/B, step trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_p 900 $T tests/test_engine_gpu.py tests/test_step_graph.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py
run r5p_s1 300 python -u bench.py --steps 50
run r5p_m1 300 env FEDREC_SIDE_WGRAD=0 python -u bench.py --steps 50
run r5p_s2 300 python -u bench.py --steps 50
run r5p_m2 300 env FEDREC_SIDE_WGRAD=0 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_r5p
rm -rf $O; mkdir -p $O
run prof_r5p 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_p.json > gpurun_out/breakdown_r5p.txt 2>&1
head -30 gpurun_out/breakdown_r5p.txt
python benchmarks/launch_seq.py "$f" > gpurun_out/r5p_launch_seq.txt
