#!/bin/bash
# fp32 additive-pool forward split over several blocks per impression: tests + config-2 bench
source "$(dirname "$0")/../../gpu_lib.sh"
check tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_user_step_gpu.py tests/test_engine_gpu.py tests/test_step_graph.py
run c2_a 300 python bench.py --steps 50 --warmup 10
run c2_b 300 python bench.py --steps 50 --warmup 10
O=$PWD/gpurun_out/prof_pool
rm -rf $O; mkdir -p $O
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c2 -- python bench.py --steps 30 --warmup 10 --round off --no-valid
