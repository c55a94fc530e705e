#!/bin/bash
# G path in the step after the VALU cut: focused tests, A/B/A/B, breakdown
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_h 900 $T tests/test_text_head_gpu.py tests/test_step_graph.py tests/test_engine_gpu.py tests/test_no_library_kernels_gpu.py tests/test_user_step_gpu.py
run r5h_g1 300 python -u bench.py --steps 50
run r5h_r4a 300 env FEDREC_HEAD_G=0 python -u bench.py --steps 50
run r5h_g2 300 python -u bench.py --steps 50
run r5h_r4b 300 env FEDREC_HEAD_G=0 python -u bench.py --steps 50
run r5h_def 300 python -u bench.py
O=$PWD/gpurun_out/prof_r5h
rm -rf $O; mkdir -p $O
run prof_r5h 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_h.json > gpurun_out/breakdown_r5h.txt 2>&1
head -30 gpurun_out/breakdown_r5h.txt
