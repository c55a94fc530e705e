#!/bin/bash
# partial-column-tile ping-pong GEMM: numerics, all GEMM/kernel tests, config-2 bench + profile
source "$(dirname "$0")/../../gpu_lib.sh"
check parttest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_partial_gpu.py
check ktests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_user_step_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py -m gpu
run bench 400 python bench.py --steps 50 --warmup 10
O=$PWD/gpurun_out/prof_part
rm -rf $O; mkdir -p $O
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
