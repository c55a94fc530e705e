#!/bin/bash
# side-stream weight gradients + register-direct small GEMMs (W^T casts): tests, A/B, trace
source "$(dirname "$0")/gpu_lib.sh"
export PYTHONPATH=$PWD:$PYTHONPATH
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
check t_q1 600 $T tests/test_small_gemm_gpu.py tests/test_kernels_gpu.py -k "rd_ or multi_cast"
check t_q2 900 $T tests/test_engine_gpu.py tests/test_step_graph.py tests/test_user_step_gpu.py tests/test_no_library_kernels_gpu.py tests/test_text_head_gpu.py
run r5q_new1 300 python -u bench.py --steps 50
run r5q_old1 300 env FEDREC_SIDE_WGRAD=0 FEDREC_SG_RD=0 python -u bench.py --steps 50
run r5q_side1 300 env FEDREC_SG_RD=0 python -u bench.py --steps 50
run r5q_new2 300 python -u bench.py --steps 50
run r5q_old2 300 env FEDREC_SIDE_WGRAD=0 FEDREC_SG_RD=0 python -u bench.py --steps 50
run r5q_side2 300 env FEDREC_SG_RD=0 python -u bench.py --steps 50
O=$PWD/gpurun_out/prof_r5q
rm -rf $O; mkdir -p $O
run prof_r5q 400 rocprofv3 --kernel-trace --output-format csv -d $O -o c2 -- python -u bench.py --steps 20 --warmup 5 --round off --no-valid
f=$(find $O -name "*kernel_trace.csv" | head -1)
python benchmarks/step_breakdown.py "$f" --steps 10 --json gpurun_out/r5_cfg2_step_breakdown_q.json > gpurun_out/breakdown_r5q.txt 2>&1
python benchmarks/launch_seq.py "$f" > gpurun_out/r5q_launch_seq.txt
head -30 gpurun_out/breakdown_r5q.txt
