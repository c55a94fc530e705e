#!/bin/bash
# materialised user input dropout: user-step / engine / graph tests, config-2 bench + profile
source "$(dirname "$0")/../../gpu_lib.sh"
check utests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_user_step_gpu.py tests/test_small_gemm_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py tests/test_dropout.py tests/test_kernels_gpu.py tests/test_multirank_gpu.py -m gpu
run bench 400 python bench.py --steps 50 --warmup 10
O=$PWD/gpurun_out/prof_u2
rm -rf $O; mkdir -p $O
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
